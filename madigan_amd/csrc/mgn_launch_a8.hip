// launchers for APAD = 8 (see mgn_launch.h)
#include "mgn_launch_impl.h"
MGN_DEFINE_APAD(8)
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
