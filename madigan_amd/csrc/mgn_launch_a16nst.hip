// the three-role kernel's n-step instantiations at APAD = 16 (launch_trio_nst,
// mgn_launch_impl.h): their own unit for their own flags
// (madigan_amd/build.py UNIT_FLAGS)
#include "mgn_launch_impl.h"
namespace mgn {
void launch_trio_nst_a16(const StepArgs& a) { launch_trio_nst<16>(a); }
}  // namespace mgn
