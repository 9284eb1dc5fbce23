// the three-role kernel's multi-step agent-loop instantiations at APAD = 8 --
// the C3 headline (launch_trio_agent_k, mgn_launch_impl.h): their own unit,
// the one built with machine LICM (madigan_amd/build.py)
#include "mgn_launch_impl.h"
namespace mgn {
void launch_trio_agent_a8(const StepArgs& a) { launch_trio_agent_k<8, false>(a); }
}  // namespace mgn
// diagnostic builds: this unit's copies of the stamp buffers (the headline's)
#if defined(MGN_STAMPS) || defined(MGN_WALLX)
extern "C" int mgn_diag_stamps(unsigned long long* h) {
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(mgn::g_duo_stamps), 24 * sizeof(unsigned long long)) != hipSuccess)
    return 1;
  unsigned long long z[24] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(mgn::g_duo_stamps), z, sizeof(z)) != hipSuccess;
}
extern "C" int mgn_diag_wall(unsigned long long* h) {
  return hipMemcpyFromSymbol(h, HIP_SYMBOL(mgn::g_duo_wall), 2048 * 32 * sizeof(unsigned long long)) != hipSuccess;
}
#endif
#ifdef MGN_ITERSTAMP
extern "C" int mgn_diag_iter(unsigned long long* h) {
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(mgn::g_iter), 256 * 64 * sizeof(unsigned long long)) != hipSuccess)
    return 1;
  static unsigned long long z[256 * 64] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(mgn::g_iter), z, sizeof(z)) != hipSuccess;
}
#endif
