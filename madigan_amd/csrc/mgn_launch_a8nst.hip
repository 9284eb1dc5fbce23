// the three-role kernel's n-step instantiations at APAD = 8 (launch_trio_nst,
// mgn_launch_impl.h): their own unit for their own flags
// (madigan_amd/build.py UNIT_FLAGS)
#include "mgn_launch_impl.h"
namespace mgn {
void launch_trio_nst_a8(const StepArgs& a) { launch_trio_nst<8>(a); }
}  // namespace mgn
#if defined(MGN_STAMPS)
// diagnostic build: this unit's own copy of the per-role stamps (the n-step
// kernels run here; mgn_diag_stamps reads the A = 8 unit's)
extern "C" int mgn_diag_stamps_nst(unsigned long long* h) {
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(mgn::g_duo_stamps), 24 * sizeof(unsigned long long)) != hipSuccess)
    return 1;
  unsigned long long z[24] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(mgn::g_duo_stamps), z, sizeof(z)) != hipSuccess;
}
#endif
