// the three-role kernel's two-slots-per-lane layout for 9..16 assets
// (launch_trio_m2, mgn_launch_impl.h): its own unit for its own flags
// (madigan_amd/build.py UNIT_FLAGS)
#include "mgn_launch_impl.h"
namespace mgn {
void launch_trio_m2_a16(const StepArgs& a) { launch_trio_m2<8>(a); }
}  // namespace mgn
