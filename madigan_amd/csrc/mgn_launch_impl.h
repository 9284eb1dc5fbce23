// mgn_launch_impl.h -- defines the launchers for one APAD (included once per
// mgn_launch_a<APAD>.hip).
#pragma once

#include <type_traits>

#include "mgn_launch.h"
#include "mgn_trio.h"

namespace mgn {

template <int M, int S>
struct StepL {
  static void run(const StepArgs& a) {
    const int epb = BLOCK / S;
    const int grid = (a.p.N + epb - 1) / epb;
    auto go = [&](auto kern) {
      launch_timed(a.ev0, a.ev1, kern, dim3(grid), dim3(BLOCK), 0, a.stream, a.p, a.out, a.in_kind,
                   a.units, a.aidx, a.act, a.K);
    };
    const bool nst = a.p.nstep > 1;
    if (a.p.reqm_one) {
      if (nst) go(k_step<M, S, true, true>);
      else go(k_step<M, S, true, false>);
    } else {
      if (nst) go(k_step<M, S, false, true>);
      else go(k_step<M, S, false, false>);
    }
  }
};
// two-role step kernel (mgn_duo.h): S = APAD lanes per env per role
template <int S>
void launch_duo(const StepArgs& a) {
  constexpr int epb = DUO_HALF / S;
  const int grid = (a.p.N + epb - 1) / epb;
  const bool nst = a.p.nstep > 1;
  // NST: the envs' n-step rings in dynamic LDS (duo_nst_lds_bytes)
  const size_t lds = nst ? (size_t)epb * a.p.nstep * (a.p.D + 1) * sizeof(double) : 0;
  auto go = [&](auto kern) {
    // a refused size is the caller's hipGetLastError (HIP records every call's status)
    if (lds && hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
                   hipSuccess)
      return;
    launch_timed(a.ev0, a.ev1, kern, dim3(grid), dim3(DUO_BLOCK), (uint32_t)lds, a.stream, a.p, a.out,
                 a.in_kind, a.units, a.aidx, a.act, a.K);
  };
  const bool disc = a.in_kind == IN_DISCRETE;
  const bool tou = a.gkind == MGN_SRC_TRENDOU;  // every asset TrendOU: the kind-specialized generator waves
  if (nst) {  // n-step buffers (generator sources; no ablation build)
    if (disc && tou) {
      if (a.p.reqm_one) go(k_step_duo<S, true, false, true, false, true, MGN_SRC_TRENDOU>);
      else go(k_step_duo<S, false, false, true, false, true, MGN_SRC_TRENDOU>);
    } else if (disc) {
      if (a.p.reqm_one) go(k_step_duo<S, true, false, true, false, true>);
      else go(k_step_duo<S, false, false, true, false, true>);
    } else {
      if (a.p.reqm_one) go(k_step_duo<S, true, false, false, false, true>);
      else go(k_step_duo<S, false, false, false, false, true>);
    }
  } else if (a.p.replay) {  // replay tapes (no ablation build)
    if (disc) {
      if (a.p.reqm_one) go(k_step_duo<S, true, false, true, true, false>);
      else go(k_step_duo<S, false, false, true, true, false>);
    } else {
      if (a.p.reqm_one) go(k_step_duo<S, true, false, false, true, false>);
      else go(k_step_duo<S, false, false, false, true, false>);
    }
#ifdef MGN_DIAG
  } else if (a.p.ablate) {  // diagnostic timing builds: discrete actions only
    if (a.p.reqm_one) go(k_step_duo<S, true, true, true, false, false>);
    else go(k_step_duo<S, false, true, true, false, false>);
#endif
  } else if (disc && tou) {
    if (a.p.reqm_one) go(k_step_duo<S, true, false, true, false, false, MGN_SRC_TRENDOU>);
    else go(k_step_duo<S, false, false, true, false, false, MGN_SRC_TRENDOU>);
  } else if (disc) {
    if (a.p.reqm_one) go(k_step_duo<S, true, false, true, false, false>);
    else go(k_step_duo<S, false, false, true, false, false>);
  } else {
    if (a.p.reqm_one) go(k_step_duo<S, true, false, false, false, false>);
    else go(k_step_duo<S, false, false, false, false, false>);
  }
}

// three-role kernel, two asset slots per lane (MM = 2): a 16-asset env on 8
// lanes per role, so the 256-lane layout holds 32 envs per workgroup (8192
// envs: 256 workgroups, one round over the CUs, where one slot per lane needs
// 512 in two rounds).  Discrete actions (the agent loop), one-step rewards
// with a scalar shaper (trio_m2_ok)
template <int S>
void launch_trio_m2(const StepArgs& a) {
  constexpr int epb = TRIO_W / S;
  const int grid = (a.p.N + epb - 1) / epb;
  auto go = [&](auto kern) {
    launch_timed(a.ev0, a.ev1, kern, dim3(grid), dim3(TRIO_BLOCK), 0, a.stream, a.p.L, a.p.mep, a.p.Bm, a.p.P,
                 a.p.cash, a.act, a.p, a.out, a.in_kind, a.units, a.aidx, a.K);
  };
  const bool win = a.p.W > 0;
  if (a.p.replay) {
    if (win) {
      if (a.p.reqm_one) go(k_step_trio<S, true, true, 0, true, TRIO_W, false, -1, true, 2>);
      else go(k_step_trio<S, false, true, 0, true, TRIO_W, false, -1, true, 2>);
    } else {
      if (a.p.reqm_one) go(k_step_trio<S, true, true, 0, false, TRIO_W, false, -1, true, 2>);
      else go(k_step_trio<S, false, true, 0, false, TRIO_W, false, -1, true, 2>);
    }
  } else if (win) {
    if (a.p.reqm_one) go(k_step_trio<S, true, true, 0, true, TRIO_W, false, -1, false, 2>);
    else go(k_step_trio<S, false, true, 0, true, TRIO_W, false, -1, false, 2>);
  } else if (a.gkind == MGN_SRC_TRENDOU && traj_mask(a.out) == O_STD) {
    if (a.p.reqm_one) go(k_step_trio<S, true, true, O_STD, false, TRIO_W, false, MGN_SRC_TRENDOU, false, 2>);
    else go(k_step_trio<S, false, true, O_STD, false, TRIO_W, false, MGN_SRC_TRENDOU, false, 2>);
  } else {
    if (a.p.reqm_one) go(k_step_trio<S, true, true, 0, false, TRIO_W, false, -1, false, 2>);
    else go(k_step_trio<S, false, true, 0, false, TRIO_W, false, -1, false, 2>);
  }
}

// the launch of a three-role instantiation: grid over the envs, the n-step
// rings (NST) in dynamic LDS
template <int S>
struct TrioGo {
  const StepArgs& a;
  bool small;
  template <typename Kern>
  void operator()(Kern kern, bool nst) const {
    const int epb = (small ? 64 : TRIO_W) / S;
    const int grid = (a.p.N + epb - 1) / epb;
    const size_t lds = nst ? trio_nst_dyn_lds(S, small ? 64 : TRIO_W, a.p.nstep) : 0;
    // a refused size is the caller's hipGetLastError (HIP records every
    // call's status); trio_eligible keeps static + dynamic LDS within 160 KiB
    if (lds && hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
                   hipSuccess)
      return;
    launch_timed(a.ev0, a.ev1, kern, dim3(grid), dim3(small ? 192 : TRIO_BLOCK), (uint32_t)lds, a.stream,
                 a.p.L, a.p.mep, a.p.Bm, a.p.P, a.p.cash, a.act, a.p, a.out, a.in_kind, a.units, a.aidx, a.K);
  }
};

// three-role pipelined step kernel (mgn_trio.h): S = APAD lanes per env per role
// NST: the finish role's NStepBuffer rings in dynamic LDS (D = 1), with a
// window for discrete steps (trio_launchable).  Instantiated only by the
// n-step units (mgn_launch_a{2,4,8,16}nst.hip, mgn_launch_a1tnst.hip), which
// are built without machine-level LICM (madigan_amd/build.py UNIT_FLAGS: with
// it, the loop-invariant constants hoisted out of the step loop spilled
// 87-195 VGPRs of the 256-lane n-step kernels)
template <int S, int NS>
void launch_trio_nst_k(const StepArgs& a) {
  const bool small = (long long)a.p.N * S < 256LL * TRIO_W;
  const bool disc = a.in_kind == IN_DISCRETE;
  const TrioGo<S> go{a, small};
  auto goN = [&](auto kern) { go(kern, true); };
  if (a.p.W > 0) {
    // windows: discrete steps only (trio_launchable), one wave per role at
    // every batch -- the finish role's window rows and n-step pops need more
    // than the 256-lane layout's 168 registers (it spilled 8)
    const TrioGo<S> go64{a, true};
    if (a.p.reqm_one) go64(k_step_trio<S, true, true, 0, true, 64, NS>, true);
    else go64(k_step_trio<S, false, true, 0, true, 64, NS>, true);
    return;
  }
  if (small) {
    if (disc) {
      if (a.p.reqm_one) goN(k_step_trio<S, true, true, 0, false, 64, NS>);
      else goN(k_step_trio<S, false, true, 0, false, 64, NS>);
    } else if constexpr (NS == 1) {
      if (a.p.reqm_one) goN(k_step_trio<S, true, false, 0, false, 64, NS>);
      else goN(k_step_trio<S, false, false, 0, false, 64, NS>);
    }
  } else if (disc && a.gkind == MGN_SRC_TRENDOU) {
    // the agent loop's output sets at compile time (O_STD, with the popped
    // counts O_STDN): with the finish role popping in full, n = 20 DDR 3.37
    // against 3.67 us/step (profiles/r05s_nst_ab.txt)
    auto pick = [&](auto omc) {
      constexpr uint32_t OM = decltype(omc)::value;
      if (a.p.reqm_one) goN(k_step_trio<S, true, true, OM, false, TRIO_W, NS, MGN_SRC_TRENDOU>);
      else goN(k_step_trio<S, false, true, OM, false, TRIO_W, NS, MGN_SRC_TRENDOU>);
    };
    const uint32_t om = traj_mask(a.out);
    if (om == O_STD) pick(std::integral_constant<uint32_t, O_STD>{});
    else if (om == O_STDN) pick(std::integral_constant<uint32_t, O_STDN>{});
    else pick(std::integral_constant<uint32_t, 0u>{});
  } else if (disc) {
    if (a.p.reqm_one) goN(k_step_trio<S, true, true, 0, false, TRIO_W, NS>);
    else goN(k_step_trio<S, false, true, 0, false, TRIO_W, NS>);
  } else if constexpr (NS == 1) {
    if (a.p.reqm_one) goN(k_step_trio<S, true, false, 0, false, TRIO_W, NS>);
    else goN(k_step_trio<S, false, false, 0, false, TRIO_W, NS>);
  }
}
// the running-sum pop (NS = 2, nrun_pop) where the host granted it
// (KParams::nst_run) and the steps are discrete (the agent loop); the exact
// pop (NS = 1) otherwise
template <int S>
void launch_trio_nst(const StepArgs& a) {
  // (sortino_shaperB's running form only at one wave per role: SBR)
  const bool wave64 = a.p.W > 0 || (long long)a.p.N * S < 256LL * TRIO_W;
  if (a.p.nst_run && a.in_kind == IN_DISCRETE && (a.p.shaper != MGN_SHAPER_SORTINO_B || wave64))
    launch_trio_nst_k<S, 2>(a);
  else
    launch_trio_nst_k<S, 1>(a);
}

// the one-asset envs (ONE, S = 2: the second lane of every env a pad; its
// sums are lane 0's one leaf), discrete steps (trio_launchable): window or
// not, n = 1 or n-step (generator sources, any source kind); window handles
// at one wave per role (the finish role's rows and pops need > 168 registers)
// (a template: instantiated only by mgn_launch_a1t.hip, NS = false, and by
// mgn_launch_a1tnst.hip, NS = true: the n-step handles)
template <int S = 2, bool NS_ = false>
void launch_trio_one_impl(const StepArgs& a) {
  static_assert(S == 2, "one asset on two lanes per role");
  const bool win = a.p.W > 0;
  const bool small = win || (long long)a.p.N * S < 256LL * TRIO_W;
  const TrioGo<S> go{a, small};
  auto pick = [&](auto rq1, auto winc, auto nstc) {
    constexpr bool R = decltype(rq1)::value, W = decltype(winc)::value;
    constexpr int NS = decltype(nstc)::value;
    if constexpr (W) {
      if constexpr (NS != 0) {
        // the reference's own experiment shape (one OU asset, a window,
        // n-step returns) with the bench's output set (O_WSTD) and the OU
        // generator at compile time: R1 8192 DDR 9.40e8 -> 9.57e8 env-steps/s
        // on one box (profiles/r05s_nst_ab.txt)
        if (a.gkind == MGN_SRC_OU && traj_mask(a.out) == O_WSTD) {
          go(k_step_trio<S, R, true, O_WSTD, W, 64, NS, MGN_SRC_OU, false, 1, true>, NS);
          return;
        }
      }
      go(k_step_trio<S, R, true, 0, W, 64, NS, -1, false, 1, true>, NS);
    } else {
      if (small) go(k_step_trio<S, R, true, 0, W, 64, NS, -1, false, 1, true>, NS);
      else go(k_step_trio<S, R, true, 0, W, TRIO_W, NS, -1, false, 1, true>, NS);
    }
  };
  using T = std::true_type;
  using F = std::false_type;
  // NS_: n-step handles, with the running-sum pop where the host granted it
  using N = std::integral_constant<int, NS_ ? 1 : 0>;
  using NR = std::integral_constant<int, NS_ ? 2 : 0>;
  if (NS_ && a.p.nst_run && (a.p.shaper != MGN_SHAPER_SORTINO_B || small)) {
    if (a.p.reqm_one) {
      win ? pick(T{}, T{}, NR{}) : pick(T{}, F{}, NR{});
    } else {
      win ? pick(F{}, T{}, NR{}) : pick(F{}, F{}, NR{});
    }
    return;
  }
  if (a.p.reqm_one) {
    win ? pick(T{}, T{}, N{}) : pick(T{}, F{}, N{});
  } else {
    win ? pick(F{}, T{}, N{}) : pick(F{}, F{}, N{});
  }
}

// the agent loop's output sets (O_STD / O_ALL) at the 256-lane layout,
// discrete actions, generator sources, one-step rewards: compile-time output
// masks.  One-step launches (the agent loop's K = 1, APAD <= 8) have their own
// instantiations (K1: an episode that ends at the launch's step is reset
// inside the launch, mgn_trio.h TAIL).  APAD 8 (the C3 headline) instantiates
// them in units of their own: the multi-step launches in mgn_launch_a8t.hip
// (built with machine LICM), the one-step launches in mgn_launch_a8k1.hip
// (without: with it they spilled 6 VGPRs and measured 7.3 against 6.9 us,
// profiles/r05e_licm1)
template <int S, bool K1_, int TWv = TRIO_W>
void launch_trio_agent_k(const StepArgs& a) {
  const int grid = (a.p.N + TWv / S - 1) / (TWv / S);
  auto go = [&](auto kern) {
    launch_timed(a.ev0, a.ev1, kern, dim3(grid), dim3(3 * TWv), 0, a.stream, a.p.L, a.p.mep, a.p.Bm, a.p.P,
                 a.p.cash, a.act, a.p, a.out, a.in_kind, a.units, a.aidx, a.K);
  };
  auto pick = [&](auto omc) {
    constexpr uint32_t OM = decltype(omc)::value;
    constexpr bool K1 = K1_ && S <= 8;
    if (a.gkind == MGN_SRC_TRENDOU) {
      if (a.p.reqm_one) go(k_step_trio<S, true, true, OM, false, TWv, 0, MGN_SRC_TRENDOU, false, 1, false, K1>);
      else go(k_step_trio<S, false, true, OM, false, TWv, 0, MGN_SRC_TRENDOU, false, 1, false, K1>);
    } else if (a.p.reqm_one) {
      go(k_step_trio<S, true, true, OM, false, TWv, 0, -1, false, 1, false, K1>);
    } else {
      go(k_step_trio<S, false, true, OM, false, TWv, 0, -1, false, 1, false, K1>);
    }
  };
  if (traj_mask(a.out) == O_STD) pick(std::integral_constant<uint32_t, O_STD>{});
  else pick(std::integral_constant<uint32_t, O_ALL>{});
}
template <int S>
void launch_trio_agent(const StepArgs& a) {
  if constexpr (S == 8) {
    if (a.K == 1 && a.p.N >= kTrioK1WideN) launch_trio_agent_k1w_a8(a);  // mgn_launch_a8k1w.hip
    else if (a.K == 1) launch_trio_agent_k1_a8(a);                       // mgn_launch_a8k1.hip
    else launch_trio_agent_a8(a);              // mgn_launch_a8t.hip
  } else {
    if (a.K == 1) launch_trio_agent_k<S, true>(a);
    else launch_trio_agent_k<S, false>(a);
  }
}

template <int S>
void launch_trio(const StepArgs& a) {
  if constexpr (S == 2) {
    if (a.p.A == 1) {
      launch_trio_one(a);  // mgn_launch_a1t.hip
      return;
    }
  }
  if constexpr (S == 16) {
    if (trio_m2_ok(a.p.N, a.p.A, a.p.nstep, a.p.D, a.in_kind)) {
      launch_trio_m2_a16(a);  // mgn_launch_a16m2.hip
      return;
    }
  }
  // one wave per role when 256 lanes per role would leave CUs idle
  const bool small = (long long)a.p.N * S < 256LL * TRIO_W;
  const int epb = (small ? 64 : TRIO_W) / S;
  const int grid = (a.p.N + epb - 1) / epb;
  auto go = [&](auto kern) {
    launch_timed(a.ev0, a.ev1, kern, dim3(grid), dim3(small ? 192 : TRIO_BLOCK), 0, a.stream, a.p.L, a.p.mep,
                 a.p.Bm, a.p.P, a.p.cash, a.act, a.p, a.out, a.in_kind, a.units, a.aidx, a.K);
  };
  const bool disc = a.in_kind == IN_DISCRETE;
  const uint32_t om = traj_mask(a.out);
  if (a.p.replay) {  // RP: replay tapes at 16 assets, the 256-lane layout (trio_eligible)
    if constexpr (S == 16) {
      if (a.p.W > 0) {
        if (disc) {
          if (a.p.reqm_one) go(k_step_trio<S, true, true, 0, true, TRIO_W, false, -1, true>);
          else go(k_step_trio<S, false, true, 0, true, TRIO_W, false, -1, true>);
        } else {
          if (a.p.reqm_one) go(k_step_trio<S, true, false, 0, true, TRIO_W, false, -1, true>);
          else go(k_step_trio<S, false, false, 0, true, TRIO_W, false, -1, true>);
        }
      } else if (disc) {
        if (a.p.reqm_one) go(k_step_trio<S, true, true, 0, false, TRIO_W, false, -1, true>);
        else go(k_step_trio<S, false, true, 0, false, TRIO_W, false, -1, true>);
      } else {
        if (a.p.reqm_one) go(k_step_trio<S, true, false, 0, false, TRIO_W, false, -1, true>);
        else go(k_step_trio<S, false, false, 0, false, TRIO_W, false, -1, true>);
      }
    }
    return;
  }
  if (a.p.nstep > 1) {
    // the n-step instantiations live in units of their own
    // (mgn_launch_a{2,4,8,16}nst.hip, built without machine LICM)
    if constexpr (S == 2) launch_trio_nst_a2(a);
    else if constexpr (S == 4) launch_trio_nst_a4(a);
    else if constexpr (S == 8) launch_trio_nst_a8(a);
    else if constexpr (S == 16) launch_trio_nst_a16(a);
    return;
  }
  if (small) {  // runtime output mask, window or not
    if (a.p.W > 0) {
      if (disc && a.gkind == MGN_SRC_OU) {  // C2: OU windows
        if (a.p.reqm_one) go(k_step_trio<S, true, true, 0, true, 64, false, MGN_SRC_OU>);
        else go(k_step_trio<S, false, true, 0, true, 64, false, MGN_SRC_OU>);
      } else if (disc) {
        if (a.p.reqm_one) go(k_step_trio<S, true, true, 0, true, 64>);
        else go(k_step_trio<S, false, true, 0, true, 64>);
      } else {
        if (a.p.reqm_one) go(k_step_trio<S, true, false, 0, true, 64>);
        else go(k_step_trio<S, false, false, 0, true, 64>);
      }
    } else if (disc) {
      if (a.p.reqm_one) go(k_step_trio<S, true, true, 0, false, 64>);
      else go(k_step_trio<S, false, true, 0, false, 64>);
    } else {
      if (a.p.reqm_one) go(k_step_trio<S, true, false, 0, false, 64>);
      else go(k_step_trio<S, false, false, 0, false, 64>);
    }
  } else if (a.p.W > 0) {  // window handles: the ring / history pushes (runtime output mask)
    if (disc) {
      if (a.p.reqm_one) go(k_step_trio<S, true, true, 0, true>);
      else go(k_step_trio<S, false, true, 0, true>);
    } else {
      if (a.p.reqm_one) go(k_step_trio<S, true, false, 0, true>);
      else go(k_step_trio<S, false, false, 0, true>);
    }
  } else if (disc && (om == O_STD || om == O_ALL)) {  // the agent loop's output sets
    launch_trio_agent<S>(a);
  } else if (disc) {
    if (a.p.reqm_one) go(k_step_trio<S, true, true>);
    else go(k_step_trio<S, false, true>);
  } else {
    if (a.p.reqm_one) go(k_step_trio<S, true, false>);
    else go(k_step_trio<S, false, false>);
  }
}

template <int M, int S>
struct InitL {
  static void run(const InitArgs& a) {
    const int epb = BLOCK / S;
    const int grid = (a.p.N + epb - 1) / epb;
    hipLaunchKernelGGL((k_init_reset<M, S>), dim3(grid), dim3(BLOCK), 0, a.stream, a.p, a.mode,
                       a.mask);
  }
};
template <int M, int S>
struct ValL {
  static void run(const ValArgs& a) {
    const int epb = BLOCK / S;
    const int grid = (a.p.N + epb - 1) / epb;
    hipLaunchKernelGGL((k_valuation<M, S>), dim3(grid), dim3(BLOCK), 0, a.stream, a.p, a.out);
  }
};

// M in {1,2,4,8} clamped to [min_m(APAD), APAD]; S = APAD / M <= 16
template <template <int, int> class F, int APAD, typename Arg>
void dispatch_m(int m, const Arg& a) {
  if constexpr (APAD >= 8) {
    if (m >= 8) { F<8, APAD / 8>::run(a); return; }
  }
  if constexpr (APAD >= 4 && min_m(APAD) <= 4) {
    if (m >= 4 || min_m(APAD) == 4) { F<4, APAD / 4>::run(a); return; }
  }
  if constexpr (APAD >= 2 && min_m(APAD) <= 2) {
    if (m >= 2 || min_m(APAD) == 2) { F<2, APAD / 2>::run(a); return; }
  }
  if constexpr (min_m(APAD) == 1) F<1, APAD>::run(a);
}

}  // namespace mgn

#define MGN_DEFINE_APAD(A)                                                                   \
  namespace mgn {                                                                            \
  void launch_duo_a##A(const StepArgs& a) {                                                  \
    if constexpr (A >= 2 && A <= 16) launch_duo<A>(a);                                       \
  }                                                                                          \
  void launch_trio_a##A(const StepArgs& a) {                                                 \
    if constexpr (A >= 2 && A <= 16) launch_trio<A>(a);                                       \
  }                                                                                          \
  size_t trio_nst_lds_a##A(long long n_envs, int nstep, bool win) {                          \
    if constexpr (A >= 2 && A <= 16) {                                                       \
      const bool small = win || n_envs * A < 256LL * TRIO_W;                                 \
      return (small ? trio_static_lds<A, 64, true>() : trio_static_lds<A, TRIO_W, true>()) +   \
             trio_nst_dyn_lds(A, small ? 64 : TRIO_W, nstep);                               \
    }                                                                                        \
    return ~(size_t)0;                                                                       \
  }                                                                                          \
  void launch_step_a##A(int m, const StepArgs& a) { dispatch_m<StepL, A>(m, a); }            \
  void launch_init_a##A(int m, const InitArgs& a) { dispatch_m<InitL, A>(m, a); }            \
  void launch_val_a##A(int m, const ValArgs& a) { dispatch_m<ValL, A>(m, a); }               \
  }
