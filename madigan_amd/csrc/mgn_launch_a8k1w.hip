// the one-step agent-loop launches of large batches at APAD = 8 (N >= 65536
// envs, launch_trio_agent): one wave per role (192-thread workgroups) at four
// waves per SIMD (MGN_TRIO_WPE4: 128 VGPRs), so five workgroups share a CU
// and their serial chains (state loads, orders, the finish) overlap -- where
// the 768-thread layout holds one workgroup per CU and the grid runs in many
// rounds (262144 envs: 145 against 159 us per launch, 65536: 40.7 against
// 43.0; at 8192 envs, one round, 7.6 against 6.7: profiles/r06qr_k1_ddr_ab.txt)
#define MGN_TRIO_WPE4 1
#include "mgn_launch_impl.h"
namespace mgn {
void launch_trio_agent_k1w_a8(const StepArgs& a) { launch_trio_agent_k<8, true, 64>(a); }
}  // namespace mgn
