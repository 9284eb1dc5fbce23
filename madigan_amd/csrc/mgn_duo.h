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
//   generator waves (0-3): per iteration, first the previous step's record
//     -> reward, ledgerNormedFull, agent reward, shaper, episode statistics,
//     window row and every output store; then the source reset if one is
//     pending and the tick (gen_tick), whose prices go to LDS.
//
// Iteration j: [gen: record j-1 + tick j || ledger: orders of step j] barrier
// [ledger: prices of tick j -> sums, done, record j] barrier.  Each value is
// the same expression of the same operands as in k_step, so every output is
// bit-identical to k_step (and to the oracle); only the computing lane differs.
// Scope: M = 1, APAD = S in {2, 4, 8}, n-step 1, no replay tape (those run k_step).
#pragma once

#include "mgn_kernels.h"

namespace mgn {

constexpr int DUO_BLOCK = 512;
constexpr int DUO_HALF = DUO_BLOCK / 2;

enum { REC_STEP = 1, REC_TICK = 2, REC_DONE = 4, REC_MCALL = 8 };

template <int S>
struct DuoShared {
  static constexpr int EPB = DUO_HALF / S;
  double price[DUO_HALF];  // tick prices, lane (env_local * S + slot)
  // step record of lane / env (ledger -> generator waves)
  double rL[DUO_HALF], rPrev[DUO_HALF], rTp[DUO_HALF], rTu[DUO_HALF], rTc[DUO_HALF];
  int32_t rRk[DUO_HALF];
  double rPrevEq[EPB], rCurEq[EPB], rCash[EPB], rLp[EPB], rB[EPB];
  int32_t rK[EPB], rFlags[EPB];
  int32_t tick[EPB];   // env ticks this iteration
  int32_t reset[EPB];  // apply the source reset before the tick
  int32_t more[3];     // some env ticks next iteration, slot j % 3 (a slot is
                       // cleared two barriers after its last read)
};

// The generator lane's half of an Env step: everything downstream of the
// record (Env.h:211-229, Portfolio.cpp:150-155, offpolicy_q.py:152-164,
// nstep_buffer.py n = 1, preprocessor.py:172-175)
struct GenOut {
  double shA, shB, ep_ret, ep_len, cos_qn;
  int32_t head, len;
};

template <int S>
__device__ __forceinline__ void duo_finish(const DuoShared<S>& sh, const Lane<1>& s, const KParams& p,
                                           const mgn_traj& out, int in_kind, int env, int el, int l,
                                           int ls, uint64_t ts, bool need_ar, GenOut& g) {
  constexpr int M = 1;
  const int flags = sh.rFlags[el];
  if (flags == 0) return;
  const int A = p.A;
  const int D = p.D;
  const double cash = sh.rCash[el];
  const double Lc = sh.rL[l];
  const double P = s.P[0];
  const bool valid = s.valid[0];
  if (flags & REC_STEP) {
    const int k = sh.rK[el];
    const size_t oN = (size_t)k * p.N, oNA = (size_t)k * p.N * A;
    const double prevEq = sh.rPrevEq[el];
    const double curEq = sh.rCurEq[el];
    const double qb = sh.rB[el];
    const double tp = sh.rTp[l], tu = sh.rTu[l], tc = sh.rTc[l];
    const bool done = (flags & REC_DONE) != 0;
    const double ratio = curEq / prevEq;
    const double clampv = (in_kind == IN_SINGLE) ? 0.01 : 0.3;
    const double reward = log((ratio < clampv) ? clampv : ratio);
    const double port0 = (cash - qb) / curEq;
    const double portA = (Lc * P) / curEq;
    double ar[M];
    ar[0] = 0.;
    if (valid && need_ar) {
      double v = (((Lc * P) - sh.rPrev[l]) - (tu * tp + tc)) / prevEq;
      v += 1;
      v = (v < .35) ? .35 : v;
      ar[0] = log(v);
    }
    double cos_term = 0.;
    if (p.shaper == MGN_SHAPER_PPC) {
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
      shaped_s = shape(p.shaper, rin_s, g.shA, g.shB, p.eta, cos_term, p.sexp);
    } else {
      shaped_v = valid ? shape(p.shaper, ar[0], g.shA, g.shB, p.eta, cos_term, p.sexp) : 0.;
    }
    if (valid) {
      const size_t i = oNA + (size_t)env * A + s.asset[0];
      if (out.tprice) out.tprice[i] = tp;
      if (out.tunits) out.tunits[i] = tu;
      if (out.tcost) out.tcost[i] = tc;
      if (out.risk) out.risk[i] = (uint8_t)sh.rRk[l];
      if (out.obs_port) out.obs_port[(size_t)k * p.N * (A + 1) + (size_t)env * (A + 1) + 1 + s.asset[0]] = portA;
      if (out.obs_price) out.obs_price[(oN + env) * (size_t)p.F + s.asset[0]] = P;
      if (D != 1) {
        if (out.agent_reward) out.agent_reward[i] = ar[0];
        if (out.shaped) out.shaped[i] = shaped_v;
      }
    }
    if (ls == 0) {
      if (out.data_end) out.data_end[oN + env] = 0;
      if (out.reward) out.reward[oN + env] = reward;
      if (out.done) out.done[oN + env] = done ? 1 : 0;
      if (out.timestamp) out.timestamp[oN + env] = ts;
      if (out.margin_call) out.margin_call[oN + env] = (flags & REC_MCALL) ? 1 : 0;
      if (out.n_shaped) out.n_shaped[oN + env] = 1;
      if (out.obs_port) out.obs_port[(size_t)k * p.N * (A + 1) + (size_t)env * (A + 1)] = port0;
      if (D == 1) {
        if (out.agent_reward) out.agent_reward[oN + env] = rin_s;
        if (out.shaped) out.shaped[oN + env] = shaped_s;
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
    if (valid) {
      row[s.asset[0]] = p.ring_log ? log_norm(P) : P;
      row[p.F + 1 + s.asset[0]] = (Lc * P) / eq;
    }
    if (ls == 0) {
      row[p.F] = (cash - sh.rB[el]) / eq;
      p.ring_ts[(size_t)env * p.W + g.head] = ts;
    }
    // a reset empties the window before the refill ticks (Env.h:181-187 +
    // initialize_history); the ledger side flags it on the step that ends
    if ((flags & REC_DONE) && p.auto_reset) {
      g.len = 0;
      g.head = p.W - 1;
    }
  }
}

template <int S, bool RQ1>
__global__ __launch_bounds__(DUO_BLOCK) void k_step_duo(KParams p, mgn_traj out, int in_kind,
                                                        const double* __restrict__ units_in,
                                                        const int32_t* __restrict__ aidx_in,
                                                        const int8_t* __restrict__ act_in, int K) {
  constexpr int M = 1;
  constexpr int EPB = DUO_HALF / S;  // envs per block
  __shared__ DuoShared<S> sh;
  __shared__ EnvRecs<S> recs[EPB];
  __shared__ mgn_asset_source s_src[MGN_MAX_ASSETS];
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
    sh.rFlags[el] = 0;
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
    for (int j = 0;; ++j) {
      if (live) {
        duo_finish<S>(sh, s, p, out, in_kind, env, el, l, ls, ts, need_ar, g);
        if (sh.tick[el]) {
          if (sh.reset[el]) src_reset<M>(s, p);  // Env::reset -> dataSource->reset (Env.h:183)
          gen_tick<M>(s, p, env, ts);
          ts = ts + 1;
          sh.price[l] = s.P[0];
        }
      }
      if (threadIdx.x == 0) sh.more[(j + 1) % 3] = 0;
      __syncthreads();  // A: prices of tick j published; record j-1 consumed
      __syncthreads();  // B: record j published
      if (!sh.more[j % 3]) break;
    }
    if (!live) return;
    duo_finish<S>(sh, s, p, out, in_kind, env, el, l, ls, ts, need_ar, g);
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
  for (int j = 0;; ++j) {
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
      if (in_kind != IN_NONE) {
        broker_x<M, S, RQ1>(s, p, recs[el], cash, s0, uc, tp, tu, tc, rk, ls, sa, any_mc);
        mcall = margin_call(sa, cash, p.mainM) ? 1 : 0;  // Broker.cpp:156-157
      }
    }
    __syncthreads();  // A: the prices of tick j are in LDS
    bool reset_now = false;
    int flags = 0;
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
      const bool done = any_mc || margin_call(q, cash, p.mainM) || (curEq < 0.1 * p.init_cash);
      sh.rL[l] = s.L[0];
      sh.rPrev[l] = prevVal;
      sh.rTp[l] = tp[0];
      sh.rTu[l] = tu[0];
      sh.rTc[l] = tc[0];
      sh.rRk[l] = rk[0];
      flags = REC_STEP | (done ? REC_DONE : 0) | (mcall ? REC_MCALL : 0);
      if (ls == 0) {
        sh.rPrevEq[el] = prevEq;
        sh.rCurEq[el] = curEq;
        sh.rCash[el] = cash;
        sh.rLp[el] = q.lp;
        sh.rB[el] = q.b;
        sh.rK[el] = k;
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
      sh.rL[l] = s.L[0];
      flags = REC_TICK;
      if (ls == 0) {
        sh.rCash[el] = cash;
        sh.rLp[el] = q.lp;
        sh.rB[el] = q.b;
      }
    }
    const bool next_tick = live && ((pending > 0) || (k < K));
    if (ls == 0) {
      sh.rFlags[el] = flags;
      sh.tick[el] = next_tick ? 1 : 0;
      sh.reset[el] = reset_now ? 1 : 0;
    }
    if (next_tick) sh.more[j % 3] = 1;
    __syncthreads();  // B: record j published
    if (!sh.more[j % 3]) break;
  }

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
