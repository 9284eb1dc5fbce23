// the three-role kernel's one-step agent-loop instantiations at APAD = 8 --
// the C3 agent loop's K = 1 (launch_trio_agent_k, mgn_launch_impl.h): their
// own unit, built without machine LICM (madigan_amd/build.py)
#include "mgn_launch_impl.h"
namespace mgn {
void launch_trio_agent_k1_a8(const StepArgs& a) { launch_trio_agent_k<8, true>(a); }
}  // namespace mgn
