// the three-role kernel's one-step agent-loop instantiations at APAD = 8 --
// the C3 agent loop's K = 1 (launch_trio_agent_k, mgn_launch_impl.h): their
// own unit, built without machine LICM (madigan_amd/build.py)
#include "mgn_launch_impl.h"
namespace mgn {
void launch_trio_agent_k1_a8(const StepArgs& a) { launch_trio_agent_k<8, true>(a); }
}  // namespace mgn
#ifdef MGN_ITERSTAMP
// diagnostic build: this unit's copy of the iteration stamps (the one-step
// launches run here; mgn_diag_iter reads mgn_launch_a8t.hip's)
extern "C" int mgn_diag_iter_k1(unsigned long long* h) {
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(mgn::g_iter), 256 * 64 * sizeof(unsigned long long)) != hipSuccess)
    return 1;
  static unsigned long long z[256 * 64] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(mgn::g_iter), z, sizeof(z)) != hipSuccess;
}
#endif
