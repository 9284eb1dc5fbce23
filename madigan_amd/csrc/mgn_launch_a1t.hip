// the three-role kernel for one-asset envs (launch_trio_one_impl,
// mgn_launch_impl.h: two lanes per env and role, the second a pad): its own
// unit, compiled beside the others
#include "mgn_launch_impl.h"
namespace mgn {
void launch_trio_one(const StepArgs& a) {
  if (a.p.nstep > 1) launch_trio_one_nst(a);  // mgn_launch_a1tnst.hip
  else launch_trio_one_impl<2, false>(a);
}
}  // namespace mgn
