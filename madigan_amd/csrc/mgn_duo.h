// mgn_duo.h -- the fused step kernel with two wave roles (generator / ledger).
//
// At the headline batch (8192 envs x 8 assets) one lane per (env, asset)
// gives 1024 waves: one per SIMD, so k_step runs single-wave-issue bound
// (MI355X_MICROARCH.md: one wave alone issues a VALU op every 4 cycles where
// two waves share the SIMD at 2).  Only part of an Env step is on the serial
// path from one step to the next: the Broker orders need the previous step's
// ledger, cash and prices, and the next step needs this step's `done` (auto
// reset).  The generator tick (DataSource::getData) depends only on the source
// state, and the step's outputs (log reward, State.portfolio, the shaper, the
// episode statistics, the window row) feed nothing but the outputs.  So this
// kernel gives each (env, asset) TWO lanes in two waves of a 512-thread
// workgroup (waves w and w + 4 share a SIMD):
//
//   ledger waves (4-7): actions, Broker rounds (Broker.cpp:124-178), the
//     post-tick sums, equity and `done` (Env.h:206-223); they publish a step
//     record (ledger, responses, equities, cash) to LDS;
//   generator waves (0-3): per iteration the source reset if one is pending
//     and the tick (gen_tick), whose prices go to LDS; then the previous
//     step's record -> reward, ledgerNormedFull, agent reward, shaper,
//     episode statistics, window row and every output store.
//
// Iteration j: [gen: tick j || ledger: orders of step j] barrier [gen: step
// j-1's record -> outputs || ledger: prices of tick j -> sums, done, record j
// (records double-buffered by iteration parity)] barrier.  Each value is
// the same expression of the same operands as in k_step, so every output is
// bit-identical to k_step (and to the oracle); only the computing lane differs.
// Scope: M = 1, APAD = S in {2, 4, 8}, n-step 1, no replay tape, no multi-component
// sources (those run k_step).
// Diagnostic ablation bits (mgn_set_ablation): 1 Broker rounds, 2 generator
// ticks, 4 the generator side's step finish (outputs).
#pragma once

#include "mgn_kernels.h"

namespace mgn {

constexpr int DUO_BLOCK = 512;

#ifdef MGN_STAMPS
// diagnostic build only: per role, cycles of [work 1, wait A, work 2, wait B]
// summed over one wave per role and block, then the iteration count
__device__ unsigned long long g_duo_stamps[16];
#define MGN_T(v) v = __builtin_amdgcn_s_memtime()
#else
#define MGN_T(v)
#endif
constexpr int DUO_HALF = DUO_BLOCK / 2;

enum { REC_STEP = 1, REC_TICK = 2, REC_DONE = 4, REC_MCALL = 8 };

// step record of lane / env (ledger -> generator waves)
template <int S>
struct DuoRec {
  static constexpr int EPB = DUO_HALF / S;
  double rL[DUO_HALF], rPrev[DUO_HALF], rTp[DUO_HALF], rTu[DUO_HALF], rTc[DUO_HALF];
  int32_t rRk[DUO_HALF];
  double rPrevEq[EPB], rCurEq[EPB], rCash[EPB], rLp[EPB], rB[EPB], rRew[EPB];
  int32_t rK[EPB], rFlags[EPB];
};

template <int S>
struct DuoShared {
  static constexpr int EPB = DUO_HALF / S;
  double price[DUO_HALF];  // tick prices, lane (env_local * S + slot)
  DuoRec<S> rec[2];        // record of iteration j in rec[j & 1]
  int32_t tick[EPB];   // env ticks this iteration
  int32_t reset[EPB];  // apply the source reset before the tick
  int32_t more[3];     // some env ticks next iteration, slot j % 3 (a slot is
                       // cleared two barriers after its last read)
};

// Output pointers live in VGPR pairs (in_vgpr: the compiler cannot move them
// back into SGPRs) and their null tests in one uniform bit mask: with every
// pointer of KParams and mgn_traj in SGPRs the kernel spilled SGPRs to VGPR
// lanes and reloaded them with v_readlane inside the step loop.
enum : uint32_t { O_REW = 1u, O_AREW = 2u, O_SHP = 4u, O_DONE = 8u, O_OPR = 16u, O_OPT = 32u,
                  O_TS = 64u, O_TP = 128u, O_TU = 256u, O_TC = 512u, O_RISK = 1024u,
                  O_MC = 2048u, O_NSH = 4096u, O_DEND = 8192u };
__device__ __forceinline__ uint32_t traj_mask(const mgn_traj& o) {
  return (o.reward ? O_REW : 0u) | (o.agent_reward ? O_AREW : 0u) | (o.shaped ? O_SHP : 0u) |
         (o.done ? O_DONE : 0u) | (o.obs_price ? O_OPR : 0u) | (o.obs_port ? O_OPT : 0u) |
         (o.timestamp ? O_TS : 0u) | (o.tprice ? O_TP : 0u) | (o.tunits ? O_TU : 0u) |
         (o.tcost ? O_TC : 0u) | (o.risk ? O_RISK : 0u) | (o.margin_call ? O_MC : 0u) |
         (o.n_shaped ? O_NSH : 0u) | (o.data_end ? O_DEND : 0u);
}
template <typename T>
__device__ __forceinline__ T* vptr(T* q) {
  return reinterpret_cast<T*>(in_vgpr(reinterpret_cast<uintptr_t>(q)));
}
__device__ __forceinline__ mgn_traj traj_vgpr(const mgn_traj& o) {
  mgn_traj v;
  v.reward = vptr(o.reward);
  v.agent_reward = vptr(o.agent_reward);
  v.shaped = vptr(o.shaped);
  v.done = vptr(o.done);
  v.obs_price = vptr(o.obs_price);
  v.obs_port = vptr(o.obs_port);
  v.timestamp = vptr(o.timestamp);
  v.tprice = vptr(o.tprice);
  v.tunits = vptr(o.tunits);
  v.tcost = vptr(o.tcost);
  v.risk = vptr(o.risk);
  v.margin_call = vptr(o.margin_call);
  v.n_shaped = vptr(o.n_shaped);
  v.data_end = vptr(o.data_end);
  return v;
}

// The generator lane's half of an Env step: everything downstream of the
// record (Env.h:211-229, Portfolio.cpp:150-155, offpolicy_q.py:152-164,
// nstep_buffer.py n = 1, preprocessor.py:172-175)
struct GenOut {
  double shA, shB, ep_ret, ep_len, cos_qn;
  DdrPre ddr;  // DDR's reward-independent operands, from the current A, B
  int32_t head, len;
  int32_t hcnt, klast;  // launch history: next row, the step its rows belong to
};

// P, ts: the State's price and timestamp (the tick the record belongs to)
template <int S>
__device__ __forceinline__ void duo_finish(const DuoRec<S>& sh, const Lane<1>& s, const KParams& p,
                                           const mgn_traj& out, uint32_t om, int in_kind, int env,
                                           int el, int l, int ls, double P, uint64_t ts,
                                           bool need_ar, GenOut& g) {
  constexpr int M = 1;
  const int flags = sh.rFlags[el];
  if (flags == 0) return;
  const int A = p.A;
  const int D = p.D;
  const double cash = sh.rCash[el];
  const double Lc = sh.rL[l];
  const bool valid = s.valid[0];
  if (flags & REC_STEP) {
    const int k = sh.rK[el];
    const size_t oN = (size_t)k * p.N, oNA = (size_t)k * p.N * A;
    const double prevEq = sh.rPrevEq[el];
    const double curEq = sh.rCurEq[el];
    const double qb = sh.rB[el];
    const double tp = sh.rTp[l], tu = sh.rTu[l], tc = sh.rTc[l];
    const bool done = (flags & REC_DONE) != 0;
    const double reward = sh.rRew[el];  // the ledger side's log(max(curEq / prevEq, clamp))
    double ar[M];
    ar[0] = 0.;
    if (valid && need_ar) {
      double v = (((Lc * P) - sh.rPrev[l]) - (tu * tp + tc)) / prevEq;
      v += 1;
      v = (v < .35) ? .35 : v;
      ar[0] = log_ratio(v);
    }
    double cos_term = 0.;
    if (p.shaper == MGN_SHAPER_PPC) {
      const double port0 = (cash - qb) / curEq;
      const double portA = (Lc * P) / curEq;
      double pp[M], pq[M];
      const double qv = valid ? p.target[1 + s.asset[0]] : 0.;
      const double pv = valid ? portA : 0.;
      pp[0] = pv * pv;
      pq[0] = pv * qv;
      const double np_ = sqrt(port0 * port0 + canon<M, S>(pp));
      const double dot = port0 * p.target[0] + canon<M, S>(pq);
      cos_term = p.cos_temp * (dot / (np_ * g.cos_qn));
    }
    double shaped_s = 0., rin_s = 0., shaped_v = 0.;
    if (D == 1) {
      rin_s = (p.reward_mode == MGN_REWARD_AGENT_SUM) ? canon<M, S>(ar) : reward;
      if (p.shaper == MGN_SHAPER_DDR) {  // shape() for DDR (nstep_buffer.py:128-162) on g.ddr
        const double r = rin_s;
        shaped_s = clip1((0.0 + 1.0 * ddr_one_pre(r, g.shA, g.shB, g.ddr)) / 1);
        double m = r < 0. ? r : 0.;
        if (r != r) m = r;
        g.shA += p.eta * (r - g.shA);
        g.shB += p.eta * (m * m - g.shB);
      } else {
        shaped_s = shape(p.shaper, rin_s, g.shA, g.shB, p.eta, cos_term, p.sexp);
      }
    } else {
      shaped_v = valid ? shape(p.shaper, ar[0], g.shA, g.shB, p.eta, cos_term, p.sexp) : 0.;
    }
    if (valid && D != 1) {
      const size_t i = oNA + (size_t)env * A + s.asset[0];
      if (om & O_AREW) out.agent_reward[i] = ar[0];
      if (om & O_SHP) out.shaped[i] = shaped_v;
    }
    if (ls == 0) {
      if (om & O_DEND) out.data_end[oN + env] = 0;
      if (om & O_REW) out.reward[oN + env] = reward;
      if (om & O_TS) out.timestamp[oN + env] = ts;
      if (om & O_NSH) out.n_shaped[oN + env] = 1;
      if (D == 1) {
        if (om & O_AREW) out.agent_reward[oN + env] = rin_s;
        if (om & O_SHP) out.shaped[oN + env] = shaped_s;
      }
    }
    g.ep_ret += reward;
    g.ep_len += 1;
    if (done) {
      if (ls == 0) {
        double* st = p.epstats + (size_t)env * 4;
        st[0] = g.ep_ret;
        st[1] = g.ep_len;
        st[2] = curEq;
        st[3] = st[3] + 1;
      }
      g.ep_ret = 0;
      g.ep_len = 0;
    }
  }
  if (p.W > 0) {
    // StackerDiscrete.stream_state of the State (preprocessor.py:172-175),
    // the values ring_push computes from the same sums
    const double eq = (cash + sh.rLp[el]) - sh.rB[el];
    g.head = (g.head + 1) % p.W;
    if (g.len < p.W) g.len += 1;
    const int R = p.F + p.A + 1;
    double* row = p.ring + ((size_t)env * p.W + g.head) * R;
    double* hrow = p.hist ? p.hist + ((size_t)env * p.hrows + g.hcnt) * R : nullptr;
    if (valid) {
      const double pv = p.ring_log ? log_norm(P) : P;
      const double lv = (Lc * P) / eq;
      row[s.asset[0]] = pv;
      row[p.F + 1 + s.asset[0]] = lv;
      if (hrow) {
        hrow[s.asset[0]] = pv;
        hrow[p.F + 1 + s.asset[0]] = lv;
      }
    }
    if (ls == 0) {
      const double cv = (cash - sh.rB[el]) / eq;
      row[p.F] = cv;
      p.ring_ts[(size_t)env * p.W + g.head] = ts;
      if (hrow) {
        hrow[p.F] = cv;
        p.hist_ts[(size_t)env * p.hrows + g.hcnt] = ts;
      }
    }
    if (hrow) {
      // a reset's refill rows belong to the step that ended the episode
      if (flags & REC_STEP) g.klast = sh.rK[el];
      hist_mark(p, env, ls, g.hcnt, g.len, g.klast);
    }
    // a reset empties the window before the refill ticks (Env.h:181-187 +
    // initialize_history); the ledger side flags it on the step that ends
    if ((flags & REC_DONE) && p.auto_reset) {
      g.len = 0;
      g.head = p.W - 1;
    }
  }
}

#ifndef MGN_DUO_VAR
#define MGN_DUO_VAR 0
#endif

// Broker::handleTransaction(units) for a segment of S lanes, one asset per
// lane, resolved speculatively.  The serial dependency between orders (each
// risk check sees the cash and portfolio sums the earlier orders left,
// Broker.cpp:149-155) is only a dependency on which earlier orders executed.
// Guess that every nonzero order executes; then each lane checks ITS order
// against the state the guess implies -- the cash chain c_i over the earlier
// executed orders (the same (((c + X1) - y) - Z) sequence as the serial form)
// and the canonical trees over the leaves (executed earlier orders: post-order
// leaves, the rest: pre-order) -- all lanes in parallel.  The checks up to the
// first order whose outcome contradicts the guess are exact; that order's
// outcome is taken from its check, later ones are re-guessed, repeat.  Every
// check that is kept was evaluated on exactly the operands the serial form
// uses, so the ledger, responses and sums are bit-identical to XRounds; an
// unrefused batch (the common case) costs one pass instead of S dependent
// rounds.
template <int S, bool RQ1>
__device__ __forceinline__ void broker_spec(Lane<1>& s, const KParams& p, EnvRecs<S>& er,
                                            double& cash, const double (&uc)[1], double (&tp)[1],
                                            double (&tu)[1], double (&tc)[1], int (&rk)[1], int ls,
                                            Sums& after, int& any_mc) {
  double cu2[1], me2[1], bm3[1], tpr[1], tco[1];
  order_prep<1, S>(s, p, er, uc, ls, cu2, me2, bm3, tpr, tco);
  const OrderRec& own = er.r[ls];
  const int act = uc[0] != 0. ? 1 : 0;
  const uint32_t act_bits = (uint32_t)seg_or<S>(act << ls);
  uint32_t go_bits = act_bits;  // the guess
  const double cash0 = cash;
  int go = 0, mc = 0, insuff = 0;
  double cend = cash0;
  double lv[4][S];  // this lane's leaves of the last (consistent) pass
  for (int it = 0; it <= S; ++it) {
    // cash before this lane's order, and after the last order, under the guess
    double c = cash0, c_own = cash0;
#pragma unroll
    for (int i = 0; i < S; ++i) {
      if (i == ls) c_own = c;
      const d2 xz = *reinterpret_cast<const d2*>(&er.r[i].aPX);  // {aPX, X1}
      const d2 yz = *reinterpret_cast<const d2*>(&er.r[i].y);    // {y, Z}
      const double ci = ((c + xz.y) - yz.x) - yz.y;
      c = ((go_bits >> i) & 1) ? ci : c;
    }
    cend = c;
    // canonical sums before this lane's order: leaves of executed earlier
    // orders after the order, the others before
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const bool post = (j < ls) && ((go_bits >> j) & 1);
      const d2* rv = reinterpret_cast<const d2*>(&er.r[j]) + (post ? 2 : 0);
      const d2 a = rv[0], b = rv[1];
      lv[0][j] = a.x;
      lv[1][j] = a.y;
      lv[2][j] = b.x;
      lv[3][j] = b.y;
    }
    const double r0 = tree<S>(lv[0]), r1 = tree<S>(lv[1]), r2 = tree<S>(lv[2]), r3 = tree<S>(lv[3]);
    // Portfolio::checkRisk(i, u), Portfolio.cpp:254-279 (as XRounds)
    const double pnl = r0 - r1;
    const double balance = c_own + r2;
    const double bp = balance + pnl;
    const double availM = RQ1 ? bp : bp / p.reqM;
    const double equity = (c_own + r0) - r3;
    const double mr = p.mainM * pnl;
    mc = (own.need_mc != 0) & ((equity <= -mr) | (bp <= -mr));
    insuff = (own.need_insuff != 0) & ((availM <= own.aPX) | (balance <= 0.));
    go = act & !mc & !insuff;
    const uint32_t bad = (uint32_t)seg_or<S>((go != (int)((go_bits >> ls) & 1)) ? (1 << ls) : 0);
    if (bad == 0) break;
    const int i0 = __builtin_ctz(bad);
    const uint32_t go_now = (uint32_t)seg_or<S>(go << ls);
    const uint32_t below = (1u << i0) - 1u;
    go_bits = (go_bits & below) | (go_now & (1u << i0)) | (act_bits & ~(below | (1u << i0)));
  }
  cash = cend;
  any_mc = seg_or<S>(act & mc) != 0;
  rk[0] = act ? (mc ? MGN_MARGIN_CALL : (insuff ? MGN_INSUFF_MARGIN : MGN_GREEN)) : rk[0];
  const bool go_own[1] = {go != 0};
  // the post-transaction sums: the last lane's leaves are final but its own;
  // settle that one and broadcast its trees to the segment
  if (ls == S - 1 && go) {
    const d2* rv = reinterpret_cast<const d2*>(&er.r[S - 1]) + 2;
    const d2 a = rv[0], b = rv[1];
    lv[0][S - 1] = a.x;
    lv[1][S - 1] = a.y;
    lv[2][S - 1] = b.x;
    lv[3][S - 1] = b.y;
  }
  after.lp = seg_bcast<S, S - 1>(tree<S>(lv[0]));
  after.ml = seg_bcast<S, S - 1>(tree<S>(lv[1]));
  after.sh = seg_bcast<S, S - 1>(tree<S>(lv[2]));
  after.b = seg_bcast<S, S - 1>(tree<S>(lv[3]));
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  apply_orders<1>(s, go_own, cu2, me2, bm3, tpr, tco, uc, tp, tu, tc);
}

// ABL: the diagnostic ablation build (mgn_set_ablation != 0); the product
// instantiation carries no ablation branches
template <int S, bool RQ1, bool ABL>
__global__ __launch_bounds__(DUO_BLOCK) void k_step_duo(KParams p, mgn_traj out, int in_kind,
                                                        const double* __restrict__ units_in,
                                                        const int32_t* __restrict__ aidx_in,
                                                        const int8_t* __restrict__ act_in, int K) {
  constexpr int M = 1;
  constexpr int EPB = DUO_HALF / S;  // envs per block
  constexpr int APADK = S;
  __shared__ DuoShared<S> sh;
  __shared__ EnvRecs<S> recs[EPB];
  __shared__ mgn_asset_source s_src[APADK];  // p.A <= APADK assets
  __shared__ double s_tgt[MGN_MAX_ASSETS + 1];
  {
    const double* g = reinterpret_cast<const double*>(p.src);
    double* d = reinterpret_cast<double*>(s_src);
    const int n = p.A * (int)(sizeof(mgn_asset_source) / sizeof(double));
    for (int i = threadIdx.x; i < n; i += DUO_BLOCK) d[i] = g[i];
    if (p.target)
      for (int i = threadIdx.x; i <= p.A; i += DUO_BLOCK) s_tgt[i] = p.target[i];
    p.src = s_src;
    if (p.target) p.target = s_tgt;
  }
  const bool gen_role = threadIdx.x < DUO_HALF;
  const int l = threadIdx.x % DUO_HALF;
  const int el = l / S;
  const int ls = l % S;
  const int env = blockIdx.x * EPB + el;
  const bool live = env < p.N;
  const int envc = live ? env : 0;  // clamped index for the dead tail (never stored)
  const int A = p.A;
  if (!gen_role && ls == 0) {
    sh.tick[el] = (live && K > 0) ? 1 : 0;
    sh.reset[el] = 0;
    sh.rec[0].rFlags[el] = 0;
    sh.rec[1].rFlags[el] = 0;
  }
  if (threadIdx.x == 0) {
    sh.more[0] = 0;
    sh.more[1] = 0;
    sh.more[2] = 0;
  }
  __syncthreads();

  if (gen_role) {
    // ---------------- generator waves
    p.eta = in_vgpr(p.eta);
    p.cos_temp = in_vgpr(p.cos_temp);
    Lane<M> s;
    load_lane<M>(s, p, envc, ls);
    if (!live) s.valid[0] = false;
    uint64_t ts = p.ts[envc];
    const int D = p.D;
    GenOut g;
    if (D == 1) {
      g.shA = p.sA[envc];
      g.shB = p.sB[envc];
    } else {
      g.shA = s.valid[0] ? p.sA[(size_t)envc * A + s.asset[0]] : 0.;
      g.shB = s.valid[0] ? p.sB[(size_t)envc * A + s.asset[0]] : 0.;
    }
    g.ep_ret = p.ep[(size_t)envc * 2];
    g.ep_len = p.ep[(size_t)envc * 2 + 1];
    g.head = 0;
    g.len = 0;
    g.hcnt = p.W;
    g.klast = 0;
    if (p.W > 0) {
      g.head = p.rhead[envc];
      g.len = p.rlen[envc];
    }
    g.cos_qn = 0.;
    if (p.shaper == MGN_SHAPER_PPC) {
      double qq[M];
      const double q = s.valid[0] ? p.target[1 + s.asset[0]] : 0.;
      qq[0] = q * q;
      g.cos_qn = sqrt(p.target[0] * p.target[0] + canon<M, S>(qq));
    }
    const bool need_ar = (p.reward_mode != MGN_REWARD_ENV_LOG) || (out.agent_reward != nullptr);
    const uint32_t om = traj_mask(out);
    const mgn_traj ov = traj_vgpr(out);
    // the Philox key schedule (seed + r * W, r < 10) is loop-invariant: from a
    // VGPR seed it stays in VGPRs instead of 20 spilled SGPRs
    p.seed = in_vgpr(p.seed);
    p.env_offset = in_vgpr(p.env_offset);
    p.epstats = vptr(p.epstats);
    p.ring = vptr(p.ring);
    p.ring_ts = vptr(p.ring_ts);
    int j = 0;
#ifdef MGN_STAMPS
    unsigned long long T0 = 0, T1 = 0, T2 = 0, T3 = 0, T4 = 0, acc[4] = {0, 0, 0, 0};
#endif
    for (;; ++j) {
      MGN_T(T0);
      // issue priority to the role on the critical path of the phase: the
      // ledger's orders in phase 1, the generator's step finish in phase 2
      // (VALU issue between the two waves of a SIMD goes by priority, then age)
      __builtin_amdgcn_s_setprio(0);
      // phase 1: tick j
      const double P_prev = s.P[0];
      const uint64_t ts_prev = ts;
      if (live && sh.tick[el]) {
        if (sh.reset[el]) src_reset<M, false>(s, p, env, ts);  // Env::reset -> dataSource->reset (Env.h:183)
        if (!(ABL && (p.ablate & 2))) gen_tick<M, false, false>(s, p, env, ts);
        ts = ts + 1;
        sh.price[l] = s.P[0];
      }
      if (D == 1 && p.shaper == MGN_SHAPER_DDR) g.ddr = ddr_pre(g.shA, g.shB);
      if (threadIdx.x == 0) sh.more[(j + 1) % 3] = 0;
      MGN_T(T1);
      __syncthreads();  // A: prices of tick j published
      MGN_T(T2);
      __builtin_amdgcn_s_setprio(2);
      // phase 2: finish step j-1 (its State: the price and time before tick j)
      if (live && j > 0 && !(ABL && (p.ablate & 4)))
        duo_finish<S>(sh.rec[(j - 1) & 1], s, p, ov, om, in_kind, env, el, l, ls, P_prev, ts_prev,
                      need_ar, g);
      MGN_T(T3);
      __syncthreads();  // B: record j published
      MGN_T(T4);
#ifdef MGN_STAMPS
      acc[0] += T1 - T0; acc[1] += T2 - T1; acc[2] += T3 - T2; acc[3] += T4 - T3;
#endif
      if (!sh.more[j % 3]) break;
    }
#ifdef MGN_STAMPS
    if (threadIdx.x == 0) {
      for (int i = 0; i < 4; ++i) atomicAdd(&g_duo_stamps[i], acc[i]);
      atomicAdd(&g_duo_stamps[8], (unsigned long long)j);
    }
#endif
    if (!live) return;
    if (D == 1 && p.shaper == MGN_SHAPER_DDR) g.ddr = ddr_pre(g.shA, g.shB);
    duo_finish<S>(sh.rec[j & 1], s, p, ov, om, in_kind, env, el, l, ls, s.P[0], ts, need_ar, g);
    if (s.valid[0]) {
      const size_t i = (size_t)env * A + s.asset[0];
      p.P[i] = s.P[0];
      p.sx[i] = s.sx[0];
      p.oum[i] = s.oum[0];
      p.dy[i] = s.dy[0];
      p.tlen[i] = s.tlen[0];
      p.tfl[i] = s.tfl[0];
    }
    if (ls == 0) {
      p.ts[env] = ts;
      p.ep[(size_t)env * 2] = g.ep_ret;
      p.ep[(size_t)env * 2 + 1] = g.ep_len;
      if (p.W > 0) {
        p.rhead[env] = g.head;
        p.rlen[env] = g.len;
      }
      if (D == 1) {
        p.sA[env] = g.shA;
        p.sB[env] = g.shB;
      }
    }
    if (D != 1 && s.valid[0]) {
      p.sA[(size_t)env * A + s.asset[0]] = g.shA;
      p.sB[(size_t)env * A + s.asset[0]] = g.shB;
    }
    return;
  }

  // ---------------- ledger waves
  const uint32_t om = traj_mask(out);
  const mgn_traj ov = traj_vgpr(out);
  act_in = vptr(act_in);
  units_in = vptr(units_in);
  aidx_in = vptr(aidx_in);
  p.init_cash = in_vgpr(p.init_cash);
  p.mainM = in_vgpr(p.mainM);
  p.unit_size = in_vgpr(p.unit_size);
  Lane<M> s;
  load_lane<M>(s, p, envc, ls);
  if (!live) s.valid[0] = false;
  double cash = p.cash[envc];
  Sums s0 = port_sums<M, S>(s.L, s.mep, s.Bm, s.P);
  int8_t act_next[M] = {0};
  if (in_kind == IN_DISCRETE && s.valid[0]) act_next[0] = act_in[(size_t)env * A + s.asset[0]];

  int k = 0;
  int pending = 0;
#ifdef MGN_STAMPS
  unsigned long long T0 = 0, T1 = 0, T2 = 0, T3 = 0, T4 = 0, acc[4] = {0, 0, 0, 0};
  unsigned long long Ta = 0, Tb = 0, accb[2] = {0, 0};
  int jn = 0;
#endif
  for (int j = 0;; ++j) {
    MGN_T(T0);
#ifdef MGN_STAMPS
    jn = j;
#endif
    __builtin_amdgcn_s_setprio(2);
    const bool stepping = live && (pending == 0) && (k < K);
    const bool ticking = live && (stepping || (pending > 0));
    const size_t oN = (size_t)k * p.N, oNA = (size_t)k * p.N * A;
    double uc[M], tp[M], tu[M], tc[M];
    int rk[M];
    double prevEq = 0., prevVal = 0.;
    int mcall = 0;
    Sums sa = s0;
    int any_mc = 0;
    tp[0] = 0.;
    tu[0] = 0.;
    tc[0] = 0.;
    rk[0] = MGN_GREEN;
    uc[0] = 0.;
    if (stepping) {
      prevEq = (cash + s0.lp) - s0.b;  // Env.h:208
      if (in_kind == IN_DISCRETE) {     // dqn.py:160-179
        const double bp = (cash + s0.sh) + (s0.lp - s0.ml);
        const double avM = RQ1 ? bp : bp / p.reqM;
        const int half = p.atoms / 2;
        const int a = act_next[0];
        if (k + 1 < K && s.valid[0])
          act_next[0] = act_in[oNA + (size_t)p.N * A + (size_t)env * A + s.asset[0]];
        if (s.valid[0]) {
          const double u = p.unit_size * avM / s.P[0];
          uc[0] = (double)(a - half) * u;
          if (a == 0) uc[0] = (s.L[0] != 0) ? -s.L[0] : 0.;
        }
      } else if (in_kind == IN_UNITS) {
        uc[0] = s.valid[0] ? units_in[oNA + (size_t)env * A + s.asset[0]] : 0.;
      } else if (in_kind == IN_SINGLE) {
        const int ai = aidx_in[env];
        const double u = units_in[oN + env];
        uc[0] = (s.valid[0] && s.asset[0] == ai) ? u : 0.;
      }
      prevVal = s.L[0] * s.P[0];
      MGN_T(Ta);
      if (in_kind != IN_NONE && !(ABL && (p.ablate & 1))) {
        broker_spec<S, RQ1>(s, p, recs[el], cash, uc, tp, tu, tc, rk, ls, sa, any_mc);
        mcall = margin_call(sa, cash, p.mainM) ? 1 : 0;  // Broker.cpp:156-157
      }
      MGN_T(Tb);
#ifdef MGN_STAMPS
      accb[0] += Ta - T0;
      accb[1] += Tb - Ta;
#endif
    }
    MGN_T(T1);
    __syncthreads();  // A: the prices of tick j are in LDS
    MGN_T(T2);
    __builtin_amdgcn_s_setprio(0);
    bool reset_now = false;
    int flags = 0;
    DuoRec<S>& rc = sh.rec[j & 1];
    if (ticking && s.valid[0]) s.P[0] = sh.price[l];
    if (stepping) {
      // post-tick sums, equity, done (Env.h:211-223): only L*P sees the new prices
      Sums q = sa;
      {
        double tlp[M];
        tlp[0] = s.L[0] * s.P[0];
        q.lp = canon<M, S>(tlp);
      }
      const double curEq = (cash + q.lp) - q.b;
      // Env.h:211-212 (0.01 clamp for step(i, u), Env.h:238); on this side, whose
      // phase 2 has slack, for the generator side's step finish
      const double ratio = curEq / prevEq;
      const double clampv = (in_kind == IN_SINGLE) ? 0.01 : 0.3;
      const double reward = log_ratio((ratio < clampv) ? clampv : ratio);
      const bool done = any_mc || margin_call(q, cash, p.mainM) || (curEq < 0.1 * p.init_cash);
      rc.rL[l] = s.L[0];
      rc.rPrev[l] = prevVal;
      rc.rTp[l] = tp[0];
      rc.rTu[l] = tu[0];
      rc.rTc[l] = tc[0];
      rc.rRk[l] = rk[0];
      flags = REC_STEP | (done ? REC_DONE : 0) | (mcall ? REC_MCALL : 0);
      // the step's ledger-side outputs: BrokerResponse, State.portfolio =
      // ledgerNormedFull (Portfolio.cpp:150-155), State.price, done, marginCall
      if (s.valid[0]) {
        const size_t i = oNA + (size_t)env * A + s.asset[0];
        if (om & O_TP) ov.tprice[i] = tp[0];
        if (om & O_TU) ov.tunits[i] = tu[0];
        if (om & O_TC) ov.tcost[i] = tc[0];
        if (om & O_RISK) ov.risk[i] = (uint8_t)rk[0];
        if (om & O_OPT)
          ov.obs_port[(size_t)k * p.N * (A + 1) + (size_t)env * (A + 1) + 1 + s.asset[0]] =
              (s.L[0] * s.P[0]) / curEq;
        if (om & O_OPR) ov.obs_price[(oN + env) * (size_t)p.F + s.asset[0]] = s.P[0];
      }
      if (ls == 0) {
        if (om & O_OPT) ov.obs_port[(size_t)k * p.N * (A + 1) + (size_t)env * (A + 1)] = (cash - q.b) / curEq;
        if (om & O_DONE) ov.done[oN + env] = done ? 1 : 0;
        if (om & O_MC) ov.margin_call[oN + env] = (uint8_t)mcall;
      }
      if (ls == 0) {
        rc.rPrevEq[el] = prevEq;
        rc.rCurEq[el] = curEq;
        rc.rRew[el] = reward;
        rc.rCash[el] = cash;
        rc.rLp[el] = q.lp;
        rc.rB[el] = q.b;
        rc.rK[el] = k;
      }
      s0 = q;
      k += 1;
      if (done && p.auto_reset) {
        // Env::reset (Env.h:181-187): fresh Broker here; the source reset
        // runs on the generator side before its next tick
        s.L[0] = 0.;
        s.mep[0] = 0.;
        s.Bm[0] = 0.;
        cash = p.init_cash;
        pending = p.W > 0 ? p.W : 1;
        reset_now = true;
      }
    } else if (ticking && pending > 0) {
      // a reset tick: its State only streams into the window
      pending -= 1;
      const Sums q = port_sums<M, S>(s.L, s.mep, s.Bm, s.P);
      if (pending == 0) s0 = q;
      rc.rL[l] = s.L[0];
      flags = REC_TICK;
      if (ls == 0) {
        rc.rCash[el] = cash;
        rc.rLp[el] = q.lp;
        rc.rB[el] = q.b;
      }
    }
    const bool next_tick = live && ((pending > 0) || (k < K));
    if (ls == 0) {
      rc.rFlags[el] = flags;
      sh.tick[el] = next_tick ? 1 : 0;
      sh.reset[el] = reset_now ? 1 : 0;
    }
    if (next_tick) sh.more[j % 3] = 1;
    MGN_T(T3);
    __syncthreads();  // B: record j published
    MGN_T(T4);
#ifdef MGN_STAMPS
    acc[0] += T1 - T0; acc[1] += T2 - T1; acc[2] += T3 - T2; acc[3] += T4 - T3;
#endif
    if (!sh.more[j % 3]) break;
  }
#ifdef MGN_STAMPS
  if (threadIdx.x == DUO_HALF) {
    for (int i = 0; i < 4; ++i) atomicAdd(&g_duo_stamps[4 + i], acc[i]);
    atomicAdd(&g_duo_stamps[9], (unsigned long long)jn);
    atomicAdd(&g_duo_stamps[10], 1ull);
    atomicAdd(&g_duo_stamps[11], accb[0]);
    atomicAdd(&g_duo_stamps[12], accb[1]);
  }
#endif

  if (!live) return;
  if (s.valid[0]) {
    const size_t i = (size_t)env * A + s.asset[0];
    p.L[i] = s.L[0];
    p.mep[i] = s.mep[0];
    p.Bm[i] = s.Bm[0];
  }
  if (ls == 0) p.cash[env] = cash;
}

}  // namespace mgn
