// the three-role kernel for one-asset envs with n-step rings
// (launch_trio_one_impl, mgn_launch_impl.h): its own unit for its own flags
// (madigan_amd/build.py UNIT_FLAGS)
#include "mgn_launch_impl.h"
namespace mgn {
void launch_trio_one_nst(const StepArgs& a) { launch_trio_one_impl<2, true>(a); }
}  // namespace mgn
