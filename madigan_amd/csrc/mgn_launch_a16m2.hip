// the three-role kernel's two-slots-per-lane layout for 9..16 assets
// (launch_trio_m2, mgn_launch_impl.h): its own unit for its own flags
// (madigan_amd/build.py UNIT_FLAGS)
#include "mgn_launch_impl.h"
namespace mgn {
void launch_trio_m2_a16(const StepArgs& a) { launch_trio_m2<8>(a); }
}  // namespace mgn
#if defined(MGN_STAMPS)
// diagnostic build: this unit's own copy of the per-role stamps (the
// two-slot kernels run here; mgn_diag_stamps reads the A = 8 unit's)
extern "C" int mgn_diag_stamps_m2(unsigned long long* h) {
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(mgn::g_duo_stamps), 24 * sizeof(unsigned long long)) != hipSuccess)
    return 1;
  unsigned long long z[24] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(mgn::g_duo_stamps), z, sizeof(z)) != hipSuccess;
}
#endif
