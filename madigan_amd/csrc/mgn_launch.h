// mgn_launch.h -- host-side launchers of the templated step kernels.  Each
// padded asset count APAD has its own translation unit (mgn_launch_a<APAD>.hip)
// so the (M, S) instantiations compile in parallel.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "mgn_duo.h"
#include "mgn_kernels.h"

namespace mgn {

struct StepArgs {
  KParams p;
  mgn_traj out;
  int in_kind;
  const double* units;
  const int32_t* aidx;
  const int8_t* act;
  int K;
  hipStream_t stream;
  // mgn_set_timing(env, 2): start / stop events recorded by the launch
  // itself (hipExtLaunchKernel: the kernel's own begin / end, no marker
  // packets around it); null otherwise
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // the source kind shared by every asset of the handle, else -1 (selects the
  // kind-specialized generator role where one is instantiated)
  int gkind = -1;
};
// hipLaunchKernelGGL, or the event-recording launch when the step's events are set
template <typename Kern, typename... Args>
inline void launch_timed(const hipEvent_t ev0, const hipEvent_t ev1, Kern kern, dim3 grid, dim3 block,
                         uint32_t lds, hipStream_t st, Args... args) {
  if (ev0) hipExtLaunchKernelGGL(kern, grid, block, lds, st, ev0, ev1, 0u, args...);
  else hipLaunchKernelGGL(kern, grid, block, lds, st, args...);
}
struct InitArgs {
  KParams p;
  int mode;
  const uint8_t* mask;
  hipStream_t stream;
};
struct ValArgs {
  KParams p;
  double* out;
  hipStream_t stream;
};

// a workgroup's LDS on gfx950 (the three-role kernel's n-step eligibility)
constexpr size_t kTrioLdsMax = 160 * 1024;

// the three-role kernel's two-slots-per-lane layout (launch_trio_m2): 9..16
// assets at the 256-lane layout (N x 16 >= 256 x 256 lanes), discrete
// actions, one-step rewards with a scalar shaper
inline bool trio_m2_ok(long long n_envs, int A, int nstep, int D, int in_kind) {
  return A > 8 && A <= 16 && n_envs * 16 >= 65536 && nstep == 1 && D == 1 &&
         in_kind == IN_DISCRETE;
}
void launch_trio_m2_a16(const StepArgs& a);
// the agent loop's three-role launches at APAD = 8 (the C3 headline), in units
// of their own: multi-step (mgn_launch_a8t.hip), one-step (mgn_launch_a8k1.hip)
void launch_trio_agent_a8(const StepArgs& a);
void launch_trio_agent_k1_a8(const StepArgs& a);
void launch_trio_agent_k1w_a8(const StepArgs& a);
// one-step launches at APAD 8 from this many envs on: the wide unit
// (mgn_launch_a8k1w.hip, four waves per SIMD)
constexpr int kTrioK1WideN = 65536;
// the n-step three-role launches, in units of their own
// (mgn_launch_a{2,4,8,16}nst.hip: built without machine LICM)
void launch_trio_nst_a2(const StepArgs& a);
void launch_trio_nst_a4(const StepArgs& a);
void launch_trio_nst_a8(const StepArgs& a);
void launch_trio_nst_a16(const StepArgs& a);
// the three-role kernel for one-asset envs (ONE: S = 2 lanes, the second a
// pad), in its own unit (mgn_launch_a1t.hip; the n-step handles in
// mgn_launch_a1tnst.hip): discrete steps (the agent loop)
void launch_trio_one(const StepArgs& a);
void launch_trio_one_nst(const StepArgs& a);

// smallest assets-per-lane with at most 16 lanes per env (DPP-only reductions)
constexpr int min_m(int apad) { return apad > 16 ? apad / 16 : 1; }

#define MGN_DECLARE_APAD(A)                          \
  void launch_duo_a##A(const StepArgs& a);           \
  void launch_trio_a##A(const StepArgs& a);          \
  size_t trio_nst_lds_a##A(long long n_envs, int nstep, bool win); \
  void launch_step_a##A(int m, const StepArgs& a);   \
  void launch_init_a##A(int m, const InitArgs& a);   \
  void launch_val_a##A(int m, const ValArgs& a);
MGN_DECLARE_APAD(1)
MGN_DECLARE_APAD(2)
MGN_DECLARE_APAD(4)
MGN_DECLARE_APAD(8)
MGN_DECLARE_APAD(16)
MGN_DECLARE_APAD(32)
MGN_DECLARE_APAD(64)
#undef MGN_DECLARE_APAD

}  // namespace mgn
