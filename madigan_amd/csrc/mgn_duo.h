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

constexpr int DUO_HALF = DUO_BLOCK / 2;

enum { REC_STEP = 1, REC_TICK = 2, REC_DONE = 4, REC_MCALL = 8 };

// step record of lane / env (ledger -> generator waves)
template <int S>
struct DuoRec {
  static constexpr int EPB = DUO_HALF / S;
  // per lane: ledger, responses, agent reward, per-asset shaped reward
  double rL[DUO_HALF], rTp[DUO_HALF], rTu[DUO_HALF], rTc[DUO_HALF];
  double rAr[DUO_HALF], rShv[DUO_HALF];
  int32_t rRk[DUO_HALF];
  // per env: equity (post-tick, also of a refill tick), cash, borrowed
  // margin, log reward, the shaper's input and output (D == 1)
  double rCurEq[EPB], rCash[EPB], rB[EPB], rRew[EPB], rRin[EPB], rShaped[EPB];
  double rCos[EPB];  // PPC's cos term (n-step: added to the column at add time)
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
// lanes and reloaded them with v_readlane inside the step loop.  The VGPR
// pointers are typed address_space(1) (global): a pointer whose provenance
// the compiler cannot see is otherwise generic, its accesses become FLAT
// instructions, and FLAT counts on lgkmcnt as well as vmcnt -- every LDS
// wait and every barrier of the step loop then waited for the previous
// stores (and the next action's load) to complete in memory.
enum : uint32_t { O_REW = 1u, O_AREW = 2u, O_SHP = 4u, O_DONE = 8u, O_OPR = 16u, O_OPT = 32u,
                  O_TS = 64u, O_TP = 128u, O_TU = 256u, O_TC = 512u, O_RISK = 1024u,
                  O_MC = 2048u, O_NSH = 4096u, O_DEND = 8192u };
__host__ __device__ __forceinline__ uint32_t traj_mask(const mgn_traj& o) {
  return (o.reward ? O_REW : 0u) | (o.agent_reward ? O_AREW : 0u) | (o.shaped ? O_SHP : 0u) |
         (o.done ? O_DONE : 0u) | (o.obs_price ? O_OPR : 0u) | (o.obs_port ? O_OPT : 0u) |
         (o.timestamp ? O_TS : 0u) | (o.tprice ? O_TP : 0u) | (o.tunits ? O_TU : 0u) |
         (o.tcost ? O_TC : 0u) | (o.risk ? O_RISK : 0u) | (o.margin_call ? O_MC : 0u) |
         (o.n_shaped ? O_NSH : 0u) | (o.data_end ? O_DEND : 0u);
}
#define MGN_G __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ MGN_G T* vptr(T* q) {
  return (MGN_G T*)in_vgpr(reinterpret_cast<uintptr_t>(q));
}
template <typename T>
__device__ __forceinline__ const MGN_G T* vptr(const T* q) {
  return (const MGN_G T*)in_vgpr(reinterpret_cast<uintptr_t>(q));
}
struct GTraj {
  MGN_G double *reward, *agent_reward, *shaped;
  MGN_G uint8_t* done;
  MGN_G double *obs_price, *obs_port;
  MGN_G uint64_t* timestamp;
  MGN_G double *tprice, *tunits, *tcost;
  MGN_G uint8_t *risk, *margin_call, *n_shaped, *data_end;
};
// OMC != 0: the output set is known at compile time; the pointers of the
// fields outside it are never loaded
template <uint32_t OMC = 0>
__device__ __forceinline__ GTraj traj_vgpr(const mgn_traj& o) {
  constexpr uint32_t M = OMC ? OMC : ~0u;
  GTraj v = {};
  if (M & O_REW) v.reward = vptr(o.reward);
  if (M & O_AREW) v.agent_reward = vptr(o.agent_reward);
  if (M & O_SHP) v.shaped = vptr(o.shaped);
  if (M & O_DONE) v.done = vptr(o.done);
  if (M & O_OPR) v.obs_price = vptr(o.obs_price);
  if (M & O_OPT) v.obs_port = vptr(o.obs_port);
  if (M & O_TS) v.timestamp = vptr(o.timestamp);
  if (M & O_TP) v.tprice = vptr(o.tprice);
  if (M & O_TU) v.tunits = vptr(o.tunits);
  if (M & O_TC) v.tcost = vptr(o.tcost);
  if (M & O_RISK) v.risk = vptr(o.risk);
  if (M & O_MC) v.margin_call = vptr(o.margin_call);
  if (M & O_NSH) v.n_shaped = vptr(o.n_shaped);
  if (M & O_DEND) v.data_end = vptr(o.data_end);
  return v;
}
// the output sets with their own trio instantiations: every field, and the
// agent loop's State + EnvInfo + reward + shaped reward (no agent reward,
// n_shaped or data_end)
constexpr uint32_t O_ALL = 16383u;
constexpr uint32_t O_STD = O_REW | O_SHP | O_DONE | O_OPR | O_OPT | O_TS | O_TP | O_TU | O_TC | O_RISK | O_MC;
// an n-step agent loop's: O_STD and the popped-value counts
constexpr uint32_t O_STDN = O_STD | O_NSH;
// a windowed n-step agent loop's (bench.py windowed()): O_STDN and data_end
constexpr uint32_t O_WSTD = O_STD | O_DEND | O_NSH;
// element index k * stride + base as one 32 x 32 + 64 multiply-add (the
// host checks that every stride fits 32 bits)
__device__ __forceinline__ size_t kidx(int k, uint32_t stride, size_t base) {
  return (size_t)(uint32_t)k * stride + base;
}
// output stores (written once per launch, read after it)
template <typename T>
__device__ __forceinline__ void ost(MGN_G T* q, T v) {
#if defined(MGN_ABL_NOSTORE)  // diagnostic timing build: outputs not stored
  (void)q; (void)v;
#else
  *q = v;
#endif
}
// the generator side's per-env state outputs, global VGPR pointers
struct GState {
  MGN_G double *epstats, *ring, *hist;
  MGN_G uint64_t *ring_ts, *hist_ts;
};

// One-step shaping (DSR / DDR / PPC / naive, n = 1) runs on the ledger side,
// right after the step's reward (on the generator side it measured slower at
// C3, 2.79 -> 2.95 us per step at 256-step launches, round 1).

// The step finish is split between the roles.  The ledger lanes evaluate it
// (ledger_finish: Env.h:211-229 reward, Portfolio.cpp:150-155
// ledgerNormedFull, offpolicy_q.py:152-164 agent reward, nstep_buffer.py
// n = 1 shaping) right after the step's post-tick sums and publish it in the
// step record; the generator lanes store the record's outputs one iteration
// later (duo_store) and keep the episode statistics and the window ring
// (preprocessor.py:172-175).  Each value is the same expression
// of the same operands as in k_step, so every output stays bit-identical.
struct GenOut {
  double ep_ret, ep_len, n_done;
  int32_t head, len;
  int32_t hcnt, klast;  // launch history: next row, the step its rows belong to
};
// the ledger side's shaper state (nstep_buffer.py:38-60) and PPC constants
struct LedOut {
  double shA, shB, cos_qn;
};

// the finish of step k on the ledger side (its post-tick quantities in
// registers); writes the record's output fields
template <int S, bool NST>
__device__ __forceinline__ void ledger_finish(DuoRec<S>& rc, const Lane<1>& s, const KParams& p,
                                              const double* s_tgt, int el, int l, int ls,
                                              double cash, double qb, double prevEq, double curEq,
                                              double reward, double prevVal, double tp, double tu,
                                              double tc, bool need_ar, LedOut& g) {
  constexpr int M = 1;
  const bool valid = s.valid[0];
  const int D = p.D;
  const double Lc = s.L[0], P = s.P[0];
  double ar[M];
  ar[0] = 0.;
  if (valid && need_ar) {
    double v = (((Lc * P) - prevVal) - (tu * tp + tc)) / prevEq;
    v += 1;
    v = (v < .35) ? .35 : v;
    ar[0] = log_ratio(v);
  }
  double cos_term = 0.;
  if (p.shaper == MGN_SHAPER_PPC) {
    const double port0 = (cash - qb) / curEq;
    const double portA = (Lc * P) / curEq;
    double pp[M], pq[M];
    const double qv = valid ? s_tgt[1 + s.asset[0]] : 0.;
    const double pv = valid ? portA : 0.;
    pp[0] = pv * pv;
    pq[0] = pv * qv;
    const double np_ = sqrt(port0 * port0 + canon<M, S>(pp));
    const double dot = port0 * s_tgt[0] + canon<M, S>(pq);
    cos_term = p.cos_temp * (dot / (np_ * g.cos_qn));
  }
  double shaped_s = 0., rin_s = 0., shaped_v = 0.;
  if constexpr (NST) {
    // the generator side adds the column value to the NStepBuffer
    if (D == 1) rin_s = (p.reward_mode == MGN_REWARD_AGENT_SUM) ? canon<M, S>(ar) : reward;
  } else if (D == 1) {
    rin_s = (p.reward_mode == MGN_REWARD_AGENT_SUM) ? canon<M, S>(ar) : reward;
    if (p.shaper == MGN_SHAPER_DDR) {  // shape() for DDR (nstep_buffer.py:128-162)
      const double r = rin_s;
      shaped_s = clip1((0.0 + 1.0 * ddr_one_pre(r, g.shA, g.shB, ddr_pre(g.shA, g.shB))) / 1);
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
  rc.rAr[l] = ar[0];
  rc.rShv[l] = shaped_v;
  if (ls == 0) {
    rc.rRin[el] = rin_s;
    rc.rShaped[el] = shaped_s;
    rc.rCos[el] = cos_term;
  }
}

// replay (RP): the State's tape row, this lane's feature value and the row's
// dataEnd flag (HDFSourceSingle, DataSource.cpp:391-398)
struct RpCur {
  double curF;
  int64_t row;
  uint32_t dend;
};

// State.price of the record's State into dst (put_feats): the tape's feature
// row for replay (one column per lane when F <= S, else read back per column),
// else the generator price of the lane's asset; lg: StackerDiscrete's log
template <int S, bool RP>
__device__ __forceinline__ void duo_feats(const Lane<1>& s, const KParams& p, int ls, double P,
                                          const RpCur& rp, MGN_G double* dst, bool lg) {
  if constexpr (RP) {
    if (s.fcol >= 0) {
      if (s.fcol < p.F) ost(dst + s.fcol, lg ? log_norm(rp.curF) : rp.curF);
    } else {
      for (int f = ls; f < p.F; f += S) {
        const double v = p.rp_feat[(size_t)rp.row * p.F + f];
        ost(dst + f, lg ? log_norm(v) : v);
      }
    }
  } else if (s.valid[0]) {
    ost(dst + s.asset[0], lg ? log_norm(P) : P);
  }
}

// n > 1 (NST): the NStepBuffer of one env on the generator side -- fill count
// and oldest index (tracked by every lane of the env), the shaper state of
// the lane's column (D == 1: the env's, held by lane 0), and the env's (n, D)
// ring in LDS (nstep_buffer.py:315-356 as replay_buffer.py:68-80 drives it)
struct NstState {
  int32_t len, head;
  double A, B;
  double* ring;     // (n, D)
  double* scratch;  // (n): one pop's summands (D == 1)
};

// the generator side's half: the record's stores, episode statistics and
// window row.  P, ts, rp: the State's price, timestamp and tape row (the tick
// the record belongs to)
template <int S, bool RP, bool NST>
__device__ __forceinline__ void duo_store(const DuoRec<S>& sh, const Lane<1>& s, const KParams& p,
                                          const GTraj& out, const GState& gs, uint32_t om, int env,
                                          int el, int l, int ls, double P, uint64_t ts, const RpCur& rp,
                                          GenOut& g, NstState& ns) {
  const int flags = sh.rFlags[el];
  if (flags == 0) return;
  const int A = p.A;
  const int D = p.D;
  const bool valid = s.valid[0];
  // ledgerNormedFull (Portfolio.cpp:150-155) of the record's State: these
  // two divisions are off the ledger's step chain here
  const double eq = sh.rCurEq[el];
  const double portA = (sh.rL[l] * P) / eq;
  const double port0 = (sh.rCash[el] - sh.rB[el]) / eq;
  if (flags & REC_STEP) {
    const int k = sh.rK[el];
    const size_t oN = (size_t)k * p.N, oNA = (size_t)k * p.N * A;
    const double curEq = sh.rCurEq[el];
    const bool done = (flags & REC_DONE) != 0;
    const double reward = sh.rRew[el];
    // BrokerResponse, State.portfolio = ledgerNormedFull, State.price, done, marginCall
    if (valid) {
      const size_t i = oNA + (size_t)env * A + s.asset[0];
      if (om & O_TP) ost(out.tprice + (i), sh.rTp[l]);
      if (om & O_TU) ost(out.tunits + (i), sh.rTu[l]);
      if (om & O_TC) ost(out.tcost + (i), sh.rTc[l]);
      if (om & O_RISK) ost(out.risk + (i), (uint8_t)sh.rRk[l]);
      if (om & O_OPT) ost(out.obs_port + ((size_t)k * p.N * (A + 1) + (size_t)env * (A + 1) + 1 + s.asset[0]), portA);
      if (D != 1) {
        if (om & O_AREW) ost(out.agent_reward + (i), sh.rAr[l]);
        if (!NST && (om & O_SHP)) {
          ost(out.shaped + (i), sh.rShv[l]);
        }
      }
    }
    if (om & O_OPR) duo_feats<S, RP>(s, p, ls, P, rp, out.obs_price + (oN + env) * (size_t)p.F, false);
    if (ls == 0) {
      if (om & O_OPT) ost(out.obs_port + ((size_t)k * p.N * (A + 1) + (size_t)env * (A + 1)), port0);
      if (om & O_DONE) ost(out.done + (oN + env), (uint8_t)(done ? 1 : 0));
      if (om & O_MC) ost(out.margin_call + (oN + env), (uint8_t)((flags & REC_MCALL) ? 1 : 0));
      if (om & O_DEND) ost(out.data_end + (oN + env), (uint8_t)(RP ? rp.dend : 0u));
      if (om & O_REW) ost(out.reward + (oN + env), reward);
      if (om & O_TS) ost(out.timestamp + (oN + env), (uint64_t)(ts));
      if (!NST && (om & O_NSH)) ost(out.n_shaped + (oN + env), (uint8_t)(1));
      if (D == 1) {
        if (om & O_AREW) ost(out.agent_reward + (oN + env), sh.rRin[el]);
        if (!NST && (om & O_SHP)) ost(out.shaped + (oN + env), sh.rShaped[el]);
      }
    }
    if constexpr (NST) {
      // NStepBuffer add + pops (as k_step): append the column value; pop once
      // if full, every entry on done; the popped aggregates are row k's
      const int n = p.nstep;
      const int L1 = ns.len + 1;
      const int pops = done ? L1 : (L1 >= n ? 1 : 0);
      const bool ppc = p.shaper == MGN_SHAPER_PPC;
      const double cosv = sh.rCos[el];
      MGN_G double* row = (om & O_SHP) ? out.shaped + (oN + env) * (size_t)n * D : nullptr;
      const bool naive = p.shaper >= MGN_SHAPER_SHARPE;
      if (D == 1 && !done && L1 >= n && !naive) {
        // the common case, one pop of a full buffer: the env's S lanes
        // evaluate the L1 summands (term k on lane k mod S) into LDS, lane 0
        // sums them in k order -- nstep_column's operations, in its order
        const double rin = sh.rRin[el];
        const int tail = (ns.head + ns.len) % n;
        if (ls == 0) ns.ring[tail] = ppc ? rin + cosv : rin;
        const double A0 = seg_bcast<S, 0>(ns.A), B0 = seg_bcast<S, 0>(ns.B);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const PopPre c = pop_pre(p.shaper, A0, B0);
        double* scr = ns.scratch;
        for (int kk = ls; kk < L1; kk += S) {
          const int idx = (ns.head + kk < n) ? ns.head + kk : ns.head + kk - n;
          scr[kk] = pop_term(p.shaper, ns.ring[idx], A0, B0, c, p.disc[kk]);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (ls == 0) {
          double acc = 0.0;
          for (int kk = 0; kk < L1; ++kk) acc += scr[kk];
          double res = acc;
          if (p.shaper == MGN_SHAPER_DSR || p.shaper == MGN_SHAPER_DDR) {
            res = clip1(acc / L1);
            const double r0 = ns.ring[ns.head];
            ns.A += p.eta * (r0 - ns.A);
            if (p.shaper == MGN_SHAPER_DSR) {
              ns.B += p.eta * (r0 * r0 - ns.B);
            } else {
              double m = r0 < 0. ? r0 : 0.;
              if (r0 != r0) m = r0;
              ns.B += p.eta * (m * m - ns.B);
            }
          }
          if (row) ost(row, res);
        }
        if (row)
          for (int jj = 1 + ls; jj < n; jj += S) ost(row + jj, 0.);
      } else if (D == 1) {
        if (ls == 0) {
          const double rin = sh.rRin[el];
          nstep_column(p, ns.ring, row, 0, 1, ppc ? rin + cosv : rin, done, ns.len, ns.head, ns.A, ns.B);
        }
      } else if (valid) {
        const double a = sh.rAr[l];
        nstep_column(p, ns.ring, row, s.asset[0], D, ppc ? a + cosv : a, done, ns.len, ns.head, ns.A,
                     ns.B);
      }
      if (ls == 0 && (om & O_NSH)) ost(out.n_shaped + (oN + env), (uint8_t)pops);
      ns.head = (ns.head + pops) % n;
      ns.len = L1 - pops;
    }
    g.ep_ret += reward;
    g.ep_len += 1;
    if (done) {
      if (ls == 0) {
        MGN_G double* st = gs.epstats + (size_t)env * 4;
        st[0] = g.ep_ret;
        st[1] = g.ep_len;
        st[2] = curEq;
        g.n_done = g.n_done + 1;
        st[3] = g.n_done;
      }
      g.ep_ret = 0;
      g.ep_len = 0;
    }
  }
  if (p.W > 0) {
    // StackerDiscrete.stream_state of the State (preprocessor.py:172-175):
    // (L * P) / equity and (cash - borrowed) / equity, the values ring_push
    // computes from the same sums
    g.head = (g.head + 1 == p.W) ? 0 : g.head + 1;
    if (g.len < p.W) g.len += 1;
    const int R = p.F + p.A + 1;
    MGN_G double* row = gs.ring + ((size_t)env * p.W + g.head) * R;
    MGN_G double* hrow = p.hist ? gs.hist + ((size_t)env * p.hrows + g.hcnt) * R : nullptr;
    duo_feats<S, RP>(s, p, ls, P, rp, row, p.ring_log != 0);
    if (hrow) duo_feats<S, RP>(s, p, ls, P, rp, hrow, p.ring_log != 0);
    if (valid) {
      row[p.F + 1 + s.asset[0]] = portA;
      if (hrow) hrow[p.F + 1 + s.asset[0]] = portA;
    }
    if (ls == 0) {
      row[p.F] = port0;
      gs.ring_ts[(size_t)env * p.W + g.head] = ts;
      if (hrow) {
        hrow[p.F] = port0;
        gs.hist_ts[(size_t)env * p.hrows + g.hcnt] = ts;
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

// The cash chain of one pass of broker_spec under its guess (Broker.cpp:
// 128-135: cash becomes ((cash + X1) - y) - Z when an order executes), systolic over
// DPP (row_shr:1 -- a segment of S <= 16 lanes lies in one 16-lane row): lane
// i holds order i's terms, masked once per pass to the additions' identities
// where the guess skips the order ((c + -0.0) - 0.0 - 0.0 == c, bit for bit,
// -0.0 and NaN included); in every step each lane applies its order to the
// cash it holds and hands the result to lane i + 1, while the segment's first
// lane keeps cash0.  After step t the lanes 0..t + 1 hold their final values
// (lane i: the serial c_i = step(c_(i-1), order i-1), one chain_step per
// order as the serial form), so S - 1 steps leave every lane its cash before
// its own order, with no LDS round trip (the first lane's walk over the
// records in LDS, round 4, cost ~1450 cycles per iteration at C3) and no
// per-step select of the executing orders (masking the terms was 2-5 %
// slower on round 4's one-lane walk, profiles/r04_ab_chain_mask.txt, where it
// replaced one select per order).  M orders per lane (two-slot
// layout): the lane's orders in slot order within its step.  c_own[m]: the
// cash before the lane's order m; cend: after the last order (the segment's
// last lane's)
template <int S, int M>
__device__ __forceinline__ void dpp_chain(double cash0, const OwnChk (&own)[M], const bool (&gown)[M], int ls,
                                          double (&c_own)[M], double& cend) {
  double X1[M], y[M], Z[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    X1[m] = gown[m] ? own[m].X1 : -0.0;
    y[m] = gown[m] ? own[m].y : 0.0;
    Z[m] = gown[m] ? own[m].Z : 0.0;
  }
  auto apply = [&](double c, double (&mid)[M]) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      mid[m] = c;
      c = ((c + X1[m]) - y[m]) - Z[m];
    }
    return c;
  };
  double v = cash0, mid[M];
#pragma unroll
  for (int t = 0; t + 1 < S; ++t) {
    const double sh = dpp_f64<0x111>(apply(v, mid));  // row_shr:1
    v = (ls == 0) ? cash0 : sh;
  }
  cend = seg_bcast<S, S - 1>(apply(v, mid));
#pragma unroll
  for (int m = 0; m < M; ++m) c_own[m] = mid[m];
}

// The canonical trees of broker_spec in registers: every lane
// holds its own order's four leaves before (pre) and after (post) the order;
// the tree of lane ls's check has post leaves for the executed orders j < ls
// and pre leaves elsewhere.  Level by level, a lane takes its sibling
// subtree's two versions over DPP -- P (post leaves where executed) and Q
// (all pre) -- and adds the one its check needs to its own path (the sibling
// lies left: P, right: Q), while P and Q of the joined subtree are formed
// for the next level (row_half_mirror / row_mirror reach the sibling half of
// 8 / 16 lanes: its lanes all hold the same subtree values by then).  Each
// node is the sum of the same two children as the heap tree's (IEEE addition
// commutes), so the sums are bit-identical to the LDS form; the root of P is
// the sums after every executed order.
// ONE (a one-asset env on S = 2 lanes): the tree is lane 0's one leaf; every
// lane of the segment takes lane 0's root (its path is only read by lane 0,
// whose order is the only one)
template <int S, bool ONE = false>
__device__ __forceinline__ void dpp_tree4(const double (&pre)[4], const double (&post)[4], bool go_own, int ls,
                                          double (&path)[4], double (&rootP)[4]) {
  double nP[4], nQ[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    path[q] = pre[q];
    nQ[q] = pre[q];
    nP[q] = go_own ? post[q] : pre[q];
  }
  if constexpr (ONE) {
#pragma unroll
    for (int q = 0; q < 4; ++q) rootP[q] = seg_bcast<S, 0>(nP[q]);
    return;
  }
  auto level = [&](auto sibP, auto sibQ, bool right) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const double sp = sibP(nP[q]), sq = sibQ(nQ[q]);
      path[q] = path[q] + (right ? sp : sq);
      nP[q] = nP[q] + sp;
      nQ[q] = nQ[q] + sq;
    }
  };
  if constexpr (S >= 2)
    level([](double v) { return dpp_f64<0xB1>(v); }, [](double v) { return dpp_f64<0xB1>(v); }, (ls & 1) != 0);
  if constexpr (S >= 4)
    level([](double v) { return dpp_f64<0x4E>(v); }, [](double v) { return dpp_f64<0x4E>(v); }, (ls & 2) != 0);
  if constexpr (S >= 8)
    level([](double v) { return dpp_f64<0x141>(v); }, [](double v) { return dpp_f64<0x141>(v); }, (ls & 4) != 0);
  if constexpr (S >= 16)
    level([](double v) { return dpp_f64<0x140>(v); }, [](double v) { return dpp_f64<0x140>(v); }, (ls & 8) != 0);
#pragma unroll
  for (int q = 0; q < 4; ++q) rootP[q] = nP[q];
}

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
template <int S, bool RQ1, bool ONE>
__device__ __forceinline__ void broker_spec(Lane<1>& s, const KParams& p, EnvRecs<S>& er,
                                            double& cash, const double (&uc)[1], double (&tp)[1],
                                            double (&tu)[1], double (&tc)[1], int (&rk)[1], int ls,
                                            Sums& after, int& any_mc) {
  double cu2[1], me2[1], bm3[1], tpr[1], tco[1];
#ifdef MGN_STAMPS
  const unsigned long long t_a = __builtin_amdgcn_s_memtime();
#endif
  double lf_pre[4], lf_post[4];  // the own leaves and check operands, in registers
  OwnChk oc[1];
  order_prep<1, S, false>(s, p, er, uc, ls, cu2, me2, bm3, tpr, tco, lf_pre, lf_post, oc);
#ifdef MGN_STAMPS
  const unsigned long long t_b = __builtin_amdgcn_s_memtime();
#endif
  const OwnChk& own = oc[0];
  const int act = uc[0] != 0. ? 1 : 0;
  const uint32_t act_bits = (uint32_t)seg_or<S>(act << ls);
  uint32_t go_bits = act_bits;  // the guess
  const double cash0 = cash;
  int go = 0, mc = 0, insuff = 0;
  double cend = cash0;
  double rootP[4];  // the sums after the orders the pass took
#ifdef MGN_STAMPS
  unsigned long long t_tr = 0, t_ch = 0;
#endif
  for (int it = 0; it <= S; ++it) {
    // canonical sums before this lane's order: leaves of executed earlier
    // orders after the order, the others before
    double r[4];
    dpp_tree4<S, ONE>(lf_pre, lf_post, ((go_bits >> ls) & 1) != 0, ls, r, rootP);
#ifdef MGN_STAMPS
    if (it == 0) t_tr = __builtin_amdgcn_s_memtime();
#endif
    // cash before this lane's order, and after the last order, under the
    // guess (dpp_chain)
    double cown1[1];
    {
      const bool g1[1] = {((go_bits >> ls) & 1) != 0};
      dpp_chain<S, 1>(cash0, oc, g1, ls, cown1, cend);
    }
    const double c_own = cown1[0];
#ifdef MGN_STAMPS
    if (it == 0) t_ch = __builtin_amdgcn_s_memtime();
#endif
    // Portfolio::checkRisk(i, u), Portfolio.cpp:254-279 (as XRounds)
    const double pnl = r[0] - r[1];
    const double balance = c_own + r[2];
    const double bp = balance + pnl;
    const double availM = RQ1 ? bp : bp / p.reqM;
    const double equity = (c_own + r[0]) - r[3];
    const double mr = p.mainM * pnl;
    mc = (own.need_mc != 0) & ((equity <= -mr) | (bp <= -mr));
    insuff = (own.need_insuff != 0) & ((availM <= own.aPX) | (balance <= 0.));
    go = act & !mc & !insuff;
    const uint32_t bad = (uint32_t)seg_or<S>((go != (int)((go_bits >> ls) & 1)) ? (1 << ls) : 0);
#ifdef MGN_STAMPS
    if (threadIdx.x == DUO_HALF) s_duo_sub[6] += 1;  // passes of the wave
#endif
    if (bad == 0) break;
    const int i0 = __builtin_ctz(bad);
    const uint32_t go_now = (uint32_t)seg_or<S>(go << ls);
    const uint32_t below = (1u << i0) - 1u;
    go_bits = (go_bits & below) | (go_now & (1u << i0)) | (act_bits & ~(below | (1u << i0)));
  }
  cash = cend;
#ifdef MGN_STAMPS
  const unsigned long long t_c = __builtin_amdgcn_s_memtime();
#endif
  any_mc = seg_or<S>(act & mc) != 0;
  rk[0] = act ? (mc ? MGN_MARGIN_CALL : (insuff ? MGN_INSUFF_MARGIN : MGN_GREEN)) : rk[0];
  const bool go_own[1] = {go != 0};
  // the post-transaction sums: the root of the last pass's P tree (its guess
  // held for every order)
  after.lp = rootP[0];
  after.ml = rootP[1];
  after.sh = rootP[2];
  after.b = rootP[3];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  apply_orders<1>(s, go_own, cu2, me2, bm3, tpr, tco, uc, tp, tu, tc);
#ifdef MGN_STAMPS
  const unsigned long long t_d = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == DUO_HALF) {
    s_duo_sub[0] += t_b - t_a;
    s_duo_sub[1] += t_c - t_b;
    s_duo_sub[2] += t_d - t_c;
    s_duo_sub[3] += t_tr - t_b;   // first pass: the DPP trees
    s_duo_sub[4] += t_ch - t_tr;  // first pass: the cash chain, published and read back
    s_duo_sub[7] += t_c - t_ch;   // the checks and the remaining passes
    s_duo_sub[5] += 1;  // broker calls
  }
#endif
}

// broker_spec with two orders per lane (slots 2 ls, 2 ls + 1 of a 2 S-asset
// env: the three-role kernel's 16-asset layout on 8 lanes).  The canonical
// tree's first level is the lane's own pair, formed in registers: the check
// of slot 0 reads the pair pre + pre, slot 1 (post of slot 0 where it
// executes) + pre, and the pair's P / Q versions go on to dpp_tree4's
// cross-lane levels, which add the same sibling to both slots' paths.  The
// cash chain is dpp_chain's with the lane's two orders per step; the fix-up
// of a wrong guess is broker_spec's
// (the first order whose check disagrees decides, the later ones are guessed
// again), so the result is the sequential Broker's.
template <int S, bool RQ1>
__device__ __forceinline__ void broker_spec_m2(Lane<2>& s, const KParams& p, EnvRecs<2 * S>& er, double& cash,
                                               const double (&uc)[2], double (&tp)[2], double (&tu)[2],
                                               double (&tc)[2], int (&rk)[2], int ls, Sums& after, int& any_mc) {
  constexpr int M = 2, APAD = 2 * S;
  double cu2[M], me2[M], bm3[M], tpr[M], tco[M];
  double lf_pre[4 * M], lf_post[4 * M];
  OwnChk oc[M];
  order_prep<M, S, false>(s, p, er, uc, ls, cu2, me2, bm3, tpr, tco, lf_pre, lf_post, oc);
  // the leaves are re-formed in every pass from the slot state the lane
  // holds anyway (ledger, price, and the order's outcome): the same products
  // (order_prep's), so the same bits, without 16 leaf registers live across
  // the passes (the 168-register budget)
  auto leaves = [&](int m, double (&pr)[4], double (&po)[4]) {
    double L0 = s.L[m], me0 = s.mep[m], bm0 = s.Bm[m], P = s.P[m], c2 = cu2[m], e2 = me2[m], b2 = bm3[m];
    asm volatile("" : "+v"(L0), "+v"(me0), "+v"(bm0), "+v"(P), "+v"(c2), "+v"(e2), "+v"(b2));
    const double mk0 = (L0 < 0.) ? 1.0 : 0.0;
    const double mk1 = (c2 < 0.) ? 1.0 : 0.0;
    pr[0] = L0 * P;
    pr[1] = me0 * L0;
    pr[2] = L0 * (me0 * mk0);
    pr[3] = bm0;
    po[0] = c2 * P;
    po[1] = e2 * c2;
    po[2] = c2 * (e2 * mk1);
    po[3] = b2;
  };
  const int sh0 = ls * M;
  int act[M];
  act[0] = uc[0] != 0. ? 1 : 0;
  act[1] = uc[1] != 0. ? 1 : 0;
  const uint32_t act_bits = (uint32_t)seg_or<S>((act[0] << sh0) | (act[1] << (sh0 + 1)));
  uint32_t go_bits = act_bits;  // the guess
  const double cash0 = cash;
  int go[M] = {0, 0}, mc[M] = {0, 0}, insuff[M] = {0, 0};
  double cend = cash0;
  double rootP[4];
  for (int it = 0; it <= APAD; ++it) {
    const bool g0 = ((go_bits >> sh0) & 1) != 0, g1 = ((go_bits >> (sh0 + 1)) & 1) != 0;
    double path0[4], path1[4];
    {
      double nP[4], nQ[4], pr0[4], po0[4], pr1[4], po1[4];
      leaves(0, pr0, po0);
      leaves(1, pr1, po1);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double a0 = pr0[q], a1 = pr1[q];
        const double b0 = g0 ? po0[q] : a0;
        nQ[q] = a0 + a1;
        path0[q] = nQ[q];
        path1[q] = b0 + a1;
        nP[q] = b0 + (g1 ? po1[q] : a1);
      }
      auto level = [&](auto sib, bool right) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const double sp = sib(nP[q]), sq = sib(nQ[q]);
          const double add = right ? sp : sq;
          path0[q] = path0[q] + add;
          path1[q] = path1[q] + add;
          nP[q] = nP[q] + sp;
          nQ[q] = nQ[q] + sq;
        }
      };
      if constexpr (S >= 2) level([](double v) { return dpp_f64<0xB1>(v); }, (ls & 1) != 0);
      if constexpr (S >= 4) level([](double v) { return dpp_f64<0x4E>(v); }, (ls & 2) != 0);
      if constexpr (S >= 8) level([](double v) { return dpp_f64<0x141>(v); }, (ls & 4) != 0);
      if constexpr (S >= 16) level([](double v) { return dpp_f64<0x140>(v); }, (ls & 8) != 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) rootP[q] = nP[q];
    }
    double cownm[M];
    {
      const bool gm[M] = {g0, g1};
      dpp_chain<S, M>(cash0, oc, gm, ls, cownm, cend);
    }
    uint32_t badm = 0, gom = 0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const double* r = m == 0 ? path0 : path1;
      const double c_own = cownm[m];
      // Portfolio::checkRisk(i, u), Portfolio.cpp:254-279 (as XRounds)
      const double pnl = r[0] - r[1];
      const double balance = c_own + r[2];
      const double bp = balance + pnl;
      const double availM = RQ1 ? bp : bp / p.reqM;
      const double equity = (c_own + r[0]) - r[3];
      const double mr = p.mainM * pnl;
      mc[m] = (oc[m].need_mc != 0) & ((equity <= -mr) | (bp <= -mr));
      insuff[m] = (oc[m].need_insuff != 0) & ((availM <= oc[m].aPX) | (balance <= 0.));
      go[m] = act[m] & !mc[m] & !insuff[m];
      badm |= (go[m] != (int)((go_bits >> (sh0 + m)) & 1)) ? (1u << (sh0 + m)) : 0u;
      gom |= (uint32_t)go[m] << (sh0 + m);
    }
    const uint32_t bad = (uint32_t)seg_or<S>((int)badm);
#ifdef MGN_STAMPS
    if (threadIdx.x == DUO_HALF) s_duo_sub[6] += 1;  // passes of the wave
#endif
    if (bad == 0) break;
    const int i0 = __builtin_ctz(bad);
    const uint32_t go_now = (uint32_t)seg_or<S>((int)gom);
    const uint32_t below = (1u << i0) - 1u;
    go_bits = (go_bits & below) | (go_now & (1u << i0)) | (act_bits & ~(below | (1u << i0)));
  }
  cash = cend;
  any_mc = seg_or<S>((act[0] & mc[0]) | (act[1] & mc[1])) != 0;
#pragma unroll
  for (int m = 0; m < M; ++m)
    rk[m] = act[m] ? (mc[m] ? MGN_MARGIN_CALL : (insuff[m] ? MGN_INSUFF_MARGIN : MGN_GREEN)) : rk[m];
  const bool go_own[M] = {go[0] != 0, go[1] != 0};
  after.lp = rootP[0];
  after.ml = rootP[1];
  after.sh = rootP[2];
  after.b = rootP[3];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  apply_orders<M>(s, go_own, cu2, me2, bm3, tpr, tco, uc, tp, tu, tc);
#ifdef MGN_STAMPS
  if (threadIdx.x == DUO_HALF) s_duo_sub[5] += 1;  // broker calls
#endif
}

// The kernel arguments (KParams + mgn_traj, ~640 bytes) are read through the
// scalar cache in chunks the register allocator interleaves with their uses,
// each chunk a dependent miss on a cold cache at launch (~1.7 us of the
// prologue measured).  One scalar load per 64-byte line, all in flight
// together, warms every line for the cost of one miss.
template <int BYTES>
__device__ __forceinline__ void warm_kernargs() {
  static_assert(BYTES <= 12 * 64, "one operand per line below");
  const __attribute__((address_space(4))) uint32_t* ka =
      (const __attribute__((address_space(4))) uint32_t*)__builtin_amdgcn_kernarg_segment_ptr();
  constexpr int L = (BYTES + 63) / 64;
  uint32_t x[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) x[i] = ka[(i < L ? i : L - 1) * 16];
  // one consumer of every line: the loads issue together, one wait
  asm volatile("" ::"s"(x[0]), "s"(x[1]), "s"(x[2]), "s"(x[3]), "s"(x[4]), "s"(x[5]), "s"(x[6]),
               "s"(x[7]), "s"(x[8]), "s"(x[9]), "s"(x[10]), "s"(x[11]));
}

// HDFSourceSingle::getData on the tape (gen_tick's replay branch): the row
// iterCache / loadData would serve, then advance (wrap = the reference's
// rewind to boundsIdx_.first, DataSource.cpp:368-371, :397-399).  The next
// row's price, feature, timestamp and dataEnd flag are loaded here for the
// next tick, so a tick's tape reads leave the step's dependency chain.
struct RpNext {
  double P, F;
  uint64_t ts;
  uint32_t dend;
};
__device__ __forceinline__ void duo_replay_tick(Lane<1>& s, const KParams& p, uint64_t& ts,
                                                RpCur& cur, RpNext& nx) {
  const int64_t row = s.rcur;
  const bool fown = s.fcol >= 0 && s.fcol < p.F;
  if (s.pf_ok) {
    if (s.valid[0]) s.P[0] = nx.P;
    if (fown) cur.curF = nx.F;
    ts = nx.ts;
    cur.dend = nx.dend;
  } else {
    if (s.valid[0]) s.P[0] = p.rp_price[(size_t)row * p.A + s.asset[0]];
    if (fown) cur.curF = p.rp_feat[(size_t)row * p.F + s.fcol];
    ts = p.rp_ts[row];
    cur.dend = p.rp_end[row];
  }
  cur.row = row;
  s.row = row;
  s.rcur = (row + 1 == p.rp_rows) ? 0 : row + 1;
  if (s.valid[0]) nx.P = p.rp_price[(size_t)s.rcur * p.A + s.asset[0]];
  if (fown) nx.F = p.rp_feat[(size_t)s.rcur * p.F + s.fcol];
  nx.ts = p.rp_ts[s.rcur];
  nx.dend = p.rp_end[s.rcur];
  s.pf_ok = true;
}

// ABL: the diagnostic ablation build (mgn_set_ablation != 0); the product
// instantiation carries no ablation branches.  DISC: discrete actions
// (mgn_rollout) compiled in alone; otherwise in_kind selects Env::step() /
// step(units) / step(assetIdx, units) at run time.  (With every input kind in
// one body the paths merge before the Broker, and the wait the units load
// needs there also stalled the discrete path on its action prefetch.)  RP:
// every asset from the replay tape (mgn_attach_replay): the generator lanes
// read the tape, one row ahead, instead of ticking a generator.  NST: n-step
// aggregation (nstep > 1) on the generator side, each env's (n, D) ring and
// an n-entry pop scratch in dynamic LDS (launch_duo sizes it: envs per block
// x n x (D + 1) doubles).
// the exit test after barrier B of iteration j: the ledger runs at most one
// step per iteration, so every iteration j < K - 1 is followed by another and
// the shared `more` flag (an LDS round trip on both roles' paths) is read only
// from iteration K - 1 on
template <int S, bool RQ1, bool ABL, bool DISC, bool RP, bool NST, int GK = -1>
__global__ __launch_bounds__(DUO_BLOCK) void k_step_duo(KParams p, mgn_traj out, int in_kind_rt,
                                                        const double* __restrict__ units_in,
                                                        const int32_t* __restrict__ aidx_in,
                                                        const int8_t* __restrict__ act_in, int K) {
  // the argument segment: KParams, mgn_traj, in_kind_rt (padded to 8),
  // units_in, aidx_in, act_in, K
  warm_kernargs<(int)(sizeof(KParams) + sizeof(mgn_traj) + 8 + 24 + 4)>();
  const int in_kind = DISC ? IN_DISCRETE : in_kind_rt;
  MGN_WALL(threadIdx.x < DUO_HALF ? 0 : 1);
#if defined(MGN_STAMPS) || defined(MGN_WALLX)
  if (threadIdx.x == 0 && blockIdx.x < 2048) {  // HW_ID (CU / SE) and XCC_ID of the block
    g_duo_wall[blockIdx.x * 32 + 8] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    g_duo_wall[blockIdx.x * 32 + 9] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
  }
#endif
  constexpr int M = 1;
  constexpr int EPB = DUO_HALF / S;  // envs per block
  constexpr int APADK = S;
  __shared__ DuoShared<S> sh;
  __shared__ EnvRecs<S> recs[EPB];
  __shared__ mgn_asset_source s_src[APADK];  // p.A <= APADK assets
  __shared__ double s_tgt[MGN_MAX_ASSETS + 1];
  __shared__ double s_disc[NST ? MGN_MAX_NSTEP : 1];
  extern __shared__ __attribute__((aligned(16))) double s_nring[];  // NST: (EPB, n, D)
  const bool gen_role = threadIdx.x < DUO_HALF;
  const int l = threadIdx.x % DUO_HALF;
  const int el = l / S;
  const int ls = l % S;
  const int env = blockIdx.x * EPB + el;
  const bool live = env < p.N;
  const int envc = live ? env : 0;  // clamped index for the dead tail (never stored)
  const int A = p.A;
  // Prologue: each role's state loads are issued first, then the parameter
  // staging loads, so the launch pays one memory round trip before the loop
  // (the staging's wait covers both) instead of two.
  Lane<M> s;
  s.asset[0] = ls;
  s.valid[0] = live && ls < A;
  s.rcur = 0;
  s.row = 0;
  s.pf_ok = false;
  s.fcol = -1;
  const size_t li = (size_t)envc * A + (s.valid[0] ? ls : 0);
  s.P[0] = s.valid[0] ? p.P[li] : 0.;
  s.L[0] = s.mep[0] = s.Bm[0] = s.sx[0] = s.oum[0] = s.dy[0] = 0.;
  s.tlen[0] = 0;
  s.tfl[0] = 0;
  // generator role: the source state, timestamp, episode accumulators, window
  uint64_t ts = 0;
  double ep_ret = 0., ep_len = 0., n_done = 0.;
  int32_t rhead = 0, rlen = 0;
  // ledger role: the ledger, cash, shaper state, the first action
  double cash = 0., shA = 0., shB = 0.;
  int act_cur = 0;
  const MGN_G int8_t* act_lane = vptr(act_in) + li;
  // NST (generator role): the env's NStepBuffer
  NstState nst{0, 0, 0., 0., NST ? s_nring + (size_t)el * p.nstep * p.D : nullptr,
               NST ? s_nring + (size_t)EPB * p.nstep * p.D + (size_t)el * p.nstep : nullptr};
  if (gen_role) {
    if constexpr (RP) {
      s.rcur = p.rcur[envc];
      if (p.F <= S) s.fcol = ls;  // one feature column per lane: prefetched
    }
    if (s.valid[0]) {
      s.sx[0] = p.sx[li];
      s.oum[0] = p.oum[li];
      s.dy[0] = p.dy[li];
      s.tlen[0] = p.tlen[li];
      s.tfl[0] = p.tfl[li];
    }
    if constexpr (NST) {  // the generator side owns the shaper state
      if (p.D == 1) {
        nst.A = p.sA[envc];
        nst.B = p.sB[envc];
      } else if (s.valid[0]) {
        nst.A = p.sA[li];
        nst.B = p.sB[li];
      }
    }
    if constexpr (NST) {
      nst.len = p.nlen[envc];
      nst.head = p.nhead[envc];
      // the env's ring into LDS (every lane of the env copies a share)
      const int nD = p.nstep * p.D;
      for (int i = ls; i < nD; i += S) nst.ring[i] = p.nring[(size_t)envc * nD + i];
    }
    ts = p.ts[envc];
    s.dskip = p.dskip[envc];
    ep_ret = p.ep[(size_t)envc * 2];
    ep_len = p.ep[(size_t)envc * 2 + 1];
    n_done = p.epstats[(size_t)envc * 4 + 3];
    if (p.W > 0) {
      rhead = p.rhead[envc];
      rlen = p.rlen[envc];
    }
  } else {
    if (s.valid[0]) {
      s.L[0] = p.L[li];
      s.mep[0] = p.mep[li];
      s.Bm[0] = p.Bm[li];
    }
    cash = p.cash[envc];
    if (p.D == 1) {
      shA = p.sA[envc];
      shB = p.sB[envc];
    } else if (s.valid[0]) {
      shA = p.sA[li];
      shB = p.sB[li];
    }
    if (in_kind == IN_DISCRETE && K > 0) act_cur = act_lane[0];
  }
  MGN_WALL(gen_role ? 16 : 17);
  {
    const double* g = reinterpret_cast<const double*>(p.src);
    double* d = reinterpret_cast<double*>(s_src);
    const int n = p.A * (int)(sizeof(mgn_asset_source) / sizeof(double));
    for (int i = threadIdx.x; i < n; i += DUO_BLOCK) d[i] = g[i];
    if (p.target)
      for (int i = threadIdx.x; i <= p.A; i += DUO_BLOCK) s_tgt[i] = p.target[i];
    if constexpr (NST)
      for (int i = threadIdx.x; i < p.nstep; i += DUO_BLOCK) s_disc[i] = p.disc[i];
    p.src = s_src;
    if (p.target) p.target = s_tgt;
    if constexpr (NST) p.disc = s_disc;
  }
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
#ifdef MGN_STAMPS
  if (threadIdx.x < 8) s_duo_sub[threadIdx.x] = 0;
#endif
  __syncthreads();
  MGN_WALL(gen_role ? 18 : 19);
  s.kind[0] = s.valid[0] ? s_src[ls].kind : -1;

  if (gen_role) {
    // ---------------- generator waves
    GenOut g;
    g.ep_ret = ep_ret;
    g.ep_len = ep_len;
    g.n_done = n_done;
    g.head = rhead;
    g.len = rlen;
    g.hcnt = p.W;
    g.klast = 0;
    const uint32_t om = traj_mask(out);
    const GTraj ov = traj_vgpr(out);
    GState gs;
    gs.epstats = vptr(p.epstats);
    gs.ring = vptr(p.ring);
    gs.ring_ts = vptr(p.ring_ts);
    gs.hist = vptr(p.hist);
    gs.hist_ts = vptr(p.hist_ts);
    // the Philox key schedule (seed + r * W, r < 10) is loop-invariant: from a
    // VGPR seed it stays in VGPRs instead of 20 spilled SGPRs
    p.seed = in_vgpr(p.seed);
    p.env_offset = in_vgpr(p.env_offset);
    // drain the prologue's loads here: otherwise the wait-count pass cannot
    // tell them from the loop's stores and waits for every store (vmcnt(0))
    // where a prologue value is first used inside the loop
    drain_vmem();
    MGN_WALL(20);
    int j = 0;
#ifdef MGN_STAMPS
    unsigned long long T0 = 0, T1 = 0, T2 = 0, T3 = 0, T4 = 0, acc[4] = {0, 0, 0, 0};
#endif
    // fin: the ledger waves have left after their last barrier B; one more
    // pass stores the last record through the loop's own (already fetched)
    // store code, with no tick and no barrier
    bool fin = false;
    RpCur rp{0., 0, 0u};  // replay: the current State's tape row
    RpNext rnx{0., 0., 0, 0u};
#ifdef MGN_WALLX
    unsigned long long R1 = 0, R2 = 0, rmax = 0, rj = 0;
#endif
    for (;; ++j) {
      MGN_T(T0);
      // phase 1: the ledger's broker is the critical path, its VALU issue goes
      // first on the shared SIMD (priority, then age); phase 2: the stores
      // and the ledger's finish end at the same barrier, equal priority
      // (measured: 2.83 -> 2.71 us per step at 256 steps, 3.39 -> 3.19 at 20)
      __builtin_amdgcn_s_setprio(0);
      // phase 1: tick j
      const double P_prev = s.P[0];
      const uint64_t ts_prev = ts;
      const RpCur rp_prev = rp;
      if (!fin) {
        if (live && sh.tick[el]) {
          if constexpr (RP) {
            // the replay source carries on through a reset (DataSource.cpp:200-206)
            if (sh.reset[el]) s.dskip += 1;  // Env::reset counts (the draw index)
            duo_replay_tick(s, p, ts, rp, rnx);
          } else {
            if (sh.reset[el]) src_reset<M, false, GK>(s, p, env, ts);  // Env::reset -> dataSource->reset (Env.h:183)
            if (!(ABL && (p.ablate & 2))) gen_tick<M, false, false, GK, true>(s, p, env, ts);
            ts = ts + 1;
          }
          sh.price[l] = s.P[0];
        }
        if (threadIdx.x == 0) sh.more[(j + 1) % 3] = 0;
        MGN_T(T1);
        __syncthreads();  // A: prices of tick j published
        MGN_T(T2);
      }
      MGN_RT(R1);
      __builtin_amdgcn_s_setprio(2);
      // phase 2: store step j-1 (its State: the price and time before tick j)
      if (live && j > 0 && !(ABL && (p.ablate & 4)))
        duo_store<S, RP, NST>(sh.rec[(j - 1) & 1], s, p, ov, gs, om, env, el, l, ls, P_prev, ts_prev,
                              rp_prev, g, nst);
      MGN_RT(R2);
#ifdef MGN_WALLX
      if (R2 - R1 > rmax) {
        rmax = R2 - R1;
        rj = j;
      }
#endif
      if (fin) break;
      MGN_T(T3);
      __syncthreads();  // B: record j published
      MGN_T(T4);
#ifdef MGN_STAMPS
      acc[0] += T1 - T0; acc[1] += T2 - T1; acc[2] += T3 - T2; acc[3] += T4 - T3;
#endif
      // a wave-uniform (scalar) exit test: the fin pass skips a barrier
      if (j + 1 >= K && !__builtin_amdgcn_readfirstlane(sh.more[j % 3])) {
        fin = true;
        MGN_WALL(4);
      }
    }
    MGN_WALL(5);
    MGN_WALLV(12, rmax);
    MGN_WALLV(13, rj);
#ifdef MGN_STAMPS
    if (threadIdx.x == 0) {
      for (int i = 0; i < 4; ++i) atomicAdd(&g_duo_stamps[i], acc[i]);
      atomicAdd(&g_duo_stamps[8], (unsigned long long)(j - 1));
    }
#endif
    if (!live) return;
    if (s.valid[0]) {
      const size_t i = (size_t)env * A + s.asset[0];
      p.P[i] = s.P[0];
      p.sx[i] = s.sx[0];
      p.oum[i] = s.oum[0];
      p.dy[i] = s.dy[0];
      p.tlen[i] = s.tlen[0];
      p.tfl[i] = s.tfl[0];
    }
    if constexpr (NST) {
      const int nD = p.nstep * p.D;
      for (int i = ls; i < nD; i += S) p.nring[(size_t)env * nD + i] = nst.ring[i];
      if (ls == 0) {
        p.nlen[env] = nst.len;
        p.nhead[env] = nst.head;
      }
    }
    if constexpr (NST) {
      if (p.D == 1) {
        if (ls == 0) {
          p.sA[env] = nst.A;
          p.sB[env] = nst.B;
        }
      } else if (s.valid[0]) {
        p.sA[(size_t)env * A + s.asset[0]] = nst.A;
        p.sB[(size_t)env * A + s.asset[0]] = nst.B;
      }
    }
    if (ls == 0) {
      p.ts[env] = ts;
      p.dskip[env] = s.dskip;
      if (RP) p.rcur[env] = s.rcur;
      p.ep[(size_t)env * 2] = g.ep_ret;
      p.ep[(size_t)env * 2 + 1] = g.ep_len;
      if (p.W > 0) {
        p.rhead[env] = g.head;
        p.rlen[env] = g.len;
      }
    }
    MGN_WALL(10);
    return;
  }

  // ---------------- ledger waves
  const MGN_G double* gunits = vptr(units_in);
  const MGN_G int32_t* gaidx = vptr(aidx_in);
  p.init_cash = in_vgpr(p.init_cash);
  p.mainM = in_vgpr(p.mainM);
  p.unit_size = in_vgpr(p.unit_size);
  p.eta = in_vgpr(p.eta);
  p.cos_temp = in_vgpr(p.cos_temp);
  const int D = p.D;
  LedOut g;
  g.shA = shA;
  g.shB = shB;
  g.cos_qn = 0.;
  if (p.shaper == MGN_SHAPER_PPC) {
    double qq[M];
    const double q = s.valid[0] ? s_tgt[1 + s.asset[0]] : 0.;
    qq[0] = q * q;
    g.cos_qn = sqrt(s_tgt[0] * s_tgt[0] + canon<M, S>(qq));
  }
  const bool need_ar = (p.reward_mode != MGN_REWARD_ENV_LOG) || (out.agent_reward != nullptr);
  Sums s0 = port_sums<M, S>(s.L, s.mep, s.Bm, s.P);
  // the discrete action of lane (env, asset) at step k lives at act + k * N * A
  // (act_lane: this lane's step-0 action, loaded in the prologue); one load per
  // iteration, unconditional (clamped address), one step ahead: no merge copy
  // of a pending load, so the wait lands at the next iteration's use
  const size_t act_step = (size_t)p.N * A;
  drain_vmem();
  MGN_WALL(21);

  __builtin_amdgcn_s_setprio(2);  // the critical path of both phases
  MGN_WALL(2);
  int k = 0;
  int pending = 0;
#ifdef MGN_STAMPS
  unsigned long long T0 = 0, T1 = 0, T2 = 0, T3 = 0, T4 = 0, acc[4] = {0, 0, 0, 0};
  unsigned long long Ta = 0, Tb = 0, accb[2] = {0, 0};
  int jn = 0;
#endif
#ifdef MGN_WALLX
  unsigned long long R0 = 0, R1 = 0, rmax = 0, rj = 0;
#endif
  for (int j = 0;; ++j) {
    MGN_T(T0);
    MGN_RT(R0);
#ifdef MGN_STAMPS
    jn = j;
#endif
    const bool stepping = live && (pending == 0) && (k < K);
    const bool ticking = live && (stepping || (pending > 0));
    // this iteration's action, and the load of the next iteration's (step k + 1
    // if this one steps, else step k again)
    const int act_now = act_cur;
    if (in_kind == IN_DISCRETE) {
      const int kn = k + (stepping ? 1 : 0);
      act_cur = act_lane[(size_t)(kn < K ? kn : K - 1) * act_step];
    }
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
        const int a = act_now;
        if (s.valid[0]) {
          const double u = p.unit_size * avM / s.P[0];
          uc[0] = (double)(a - half) * u;
          if (a == 0) uc[0] = (s.L[0] != 0) ? -s.L[0] : 0.;
        }
      } else if (in_kind == IN_UNITS) {
        uc[0] = s.valid[0] ? gunits[oNA + (size_t)env * A + s.asset[0]] : 0.;
      } else if (in_kind == IN_SINGLE) {
        const int ai = gaidx[env];
        const double u = gunits[oN + env];
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
    MGN_RT(R1);
#ifdef MGN_WALLX
    if (R1 - R0 > rmax) {
      rmax = R1 - R0;
      rj = j;
    }
#endif
    __syncthreads();  // A: the prices of tick j are in LDS
    MGN_T(T2);
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
      // Env.h:211-212 (0.01 clamp for step(i, u), Env.h:238)
      const double ratio = curEq / prevEq;
      const double clampv = (in_kind == IN_SINGLE) ? 0.01 : 0.3;
      const double reward = log_ratio((ratio < clampv) ? clampv : ratio);
      const bool done = any_mc || margin_call(q, cash, p.mainM) || (curEq < 0.1 * p.init_cash);
#ifdef MGN_STAMPS
      const unsigned long long t_p2a = __builtin_amdgcn_s_memtime();
#endif
      rc.rL[l] = s.L[0];
      rc.rTp[l] = tp[0];
      rc.rTu[l] = tu[0];
      rc.rTc[l] = tc[0];
      rc.rRk[l] = rk[0];
      flags = REC_STEP | (done ? REC_DONE : 0) | (mcall ? REC_MCALL : 0);
      // the step finish (ledgerNormedFull, agent reward, shaper) into the
      // record; the generator side stores the step's outputs from it one
      // iteration later, so the ledger waves issue no stores and their only
      // vector-memory wait is on the action load
      if (!(ABL && (p.ablate & 4)))
        ledger_finish<S, NST>(rc, s, p, s_tgt, el, l, ls, cash, q.b, prevEq, curEq, reward, prevVal, tp[0],
                         tu[0], tc[0], need_ar, g);
#ifdef MGN_STAMPS
      const unsigned long long t_p2b = __builtin_amdgcn_s_memtime();
      if (threadIdx.x == DUO_HALF) {
        s_duo_sub[3] += t_p2a - T2;
        s_duo_sub[4] += t_p2b - t_p2a;
      }
#endif
      if (ls == 0) {
        rc.rCurEq[el] = curEq;
        rc.rCash[el] = cash;
        rc.rB[el] = q.b;
        rc.rRew[el] = reward;
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
      flags = REC_TICK;
      rc.rL[l] = s.L[0];
      if (ls == 0) {  // the window row's equity (ring_push's sums)
        rc.rCurEq[el] = (cash + q.lp) - q.b;
        rc.rCash[el] = cash;
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
    if (j == 0) MGN_WALL(6);
    if (j == 2) MGN_WALL(7);
#endif
    if (j + 1 >= K && !__builtin_amdgcn_readfirstlane(sh.more[j % 3])) break;
  }
  MGN_WALL(3);
  MGN_WALLV(14, rmax);
  MGN_WALLV(15, rj);
#ifdef MGN_STAMPS
  if (threadIdx.x == DUO_HALF) {
    for (int i = 0; i < 4; ++i) atomicAdd(&g_duo_stamps[4 + i], acc[i]);
    atomicAdd(&g_duo_stamps[9], (unsigned long long)jn);
    atomicAdd(&g_duo_stamps[10], 1ull);
    atomicAdd(&g_duo_stamps[11], accb[0]);
    atomicAdd(&g_duo_stamps[12], accb[1]);
    for (int i = 0; i < 5; ++i) atomicAdd(&g_duo_stamps[13 + i], s_duo_sub[i]);
  }
#endif

  if (!live) return;
  if (s.valid[0]) {
    const size_t i = (size_t)env * A + s.asset[0];
    p.L[i] = s.L[0];
    p.mep[i] = s.mep[0];
    p.Bm[i] = s.Bm[0];
  }
  if (ls == 0) {
    p.cash[env] = cash;
    if (!(NST) && D == 1) {  // else the generator side owns the shaper state
      p.sA[env] = g.shA;
      p.sB[env] = g.shB;
    }
  }
  if (!(NST) && D != 1 && s.valid[0]) {
    p.sA[(size_t)env * A + s.asset[0]] = g.shA;
    p.sB[(size_t)env * A + s.asset[0]] = g.shB;
  }
  MGN_WALL(11);
}

}  // namespace mgn
