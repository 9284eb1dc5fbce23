// mgn_trio.h -- the fused step kernel with three wave roles, pipelined.
//
// k_step_duo splits an Env step between a generator role and a ledger role
// but keeps the step's own order: orders, then the tick, then the post-tick
// sums, done and reward -- two barriers per step, and each role idles for
// part of both phases.  The step's dependencies allow a pipeline instead:
//   * the Broker orders of step k (Broker.cpp:124-178) need the ledger after
//     step k-1, the prices of tick k-1 and whether step k-1 ended the
//     episode (Env::reset before step k, Env.h:181-187);
//   * the tick of step k (DataSource::getData) needs the source state after
//     tick k-1 (and the same reset);
//   * step k-1's post-tick sums, equity, reward, done, ledgerNormedFull,
//     agent reward, shaper and episode statistics (Env.h:211-223) need the
//     ledger after the orders of step k-1 and the prices of tick k-1, and
//     feed nothing but `done`.
// So a 768-thread workgroup holds 32 envs three times (waves w, w + 4, w + 8
// share a SIMD): in iteration j the ledger waves (L) run step j's orders, the
// generator waves (G) run step j's tick, and the finish waves (F) evaluate
// step j-1 -- one barrier per iteration, records double-buffered by
// iteration parity.  `done` of step j-1 is known only at the end of
// iteration j, after L and G have speculatively run step j on the assumption
// that the episode goes on.  When F finds done (auto-reset), iteration j+1
// rolls step j back: L resets the ledger (a fresh Broker), G restores the
// source state saved before tick j, applies the source reset and ticks
// (Env::reset's getData), and step j is run again from the fresh episode in
// iteration j+2 at the same step index, overwriting the outputs the
// speculative run stored.  Episodes end rarely, so almost every speculation
// stands.  Every value is the same expression of the same operands as in
// k_step, so every output is bit-identical to k_step / k_step_duo (and the
// oracle).
// Stores: F stores every output of the steps it confirms (the BrokerResponse
// arrays stored by L, or State.price and the timestamp by G, measured
// slower, round 2); G and L write their state back at exit.
// Scope: one asset slot per lane at APAD = S in {2, 4, 8, 16}, or two (MM = 2)
// at S = 8 for 9..16 assets, or a one-asset env on S = 2 lanes (ONE: its sums
// are lane 0's one leaf); generator sources or (16 assets) a replay tape;
// n = 1 or n-step of a scalar reward (NST: DSR / DDR / PPC / none, and the
// naive shapers), with or without a window (WIN: the finish role pushes the
// ring / launch-history row of every step it confirms, and the refill rows
// after an auto-reset); k_step_duo / k_step run the rest.
#pragma once

#include "mgn_duo.h"

namespace mgn {

constexpr int TRIO_BLOCK = 768;
constexpr int TRIO_W = 256;  // lanes per role
// TW = 64 (one wave per role, 192-thread workgroups): small batches, whose
// 256-lane workgroups would leave CUs idle (C2: 4096 envs x 4 assets fill 64
// of 256 CUs at 256 lanes per role, all of them at 64)

// the roles' issue priorities (s_setprio; the ledger's orders are the
// critical path -- equal priorities measured slower, round 2)
constexpr int kPrioG = 0, kPrioL = 2, kPrioF = 1;

// one-step launches (the agent loop): an auto-reset after the step absorbed
// in the iteration that finds it (no window, generator sources): the
// generator role, idle once its tick is done, forms the reset tick's state
// beside the finish role's evaluation, and the generator / ledger roles adopt
// it (or drop it) after the loop, where the reset took another iteration --
// in about half of the one-step launches at C3 some workgroup has one.
// Measured: K = 1 7.30-7.40 -> 7.20-7.23 us; at 16- and 20-step launches the
// candidate tick under the finish role's last iteration cost 1-2 %, so longer
// launches run the reset in an iteration of its own
// (profiles/r04_ab_tail_reset.txt)
//
// WIN with a log window: the generator role forms the window rows' log
// prices (the finish role reads them from LDS; GLOG below)
//
// NST: rounds of a pop's summands evaluated together (the terms' chains
// interleave; rounds past the buffer's are computed and dropped)
constexpr int kNstU = 3;

// NST: the finish role pops in full, after its reward chain.  (Forming a
// pop's prefix -- its summands over the entries already in the ring, and
// their ordered sum -- ahead of the pop in another role measured neutral in
// the pop's own iteration, round 4, profiles/r04_ab_nst_prefix.txt, and
// slower one or two iterations ahead, round 5: n = 20 DDR 3.37 against 3.67
// us/step with the prefix one iteration ahead by the generator role,
// profiles/r05s_nst_ab.txt.)

// the loop's exit test after iteration j's barrier: iterations 0..K always
// run (the K steps, one iteration behind for the finish role), so the shared
// `more` flag -- an LDS read on every role's path out of the barrier -- is
// consulted only from iteration K on (rollbacks and refill ticks raise it)
__device__ __forceinline__ bool trio_exit(int j, int K, const int32_t& more) {
  if (j < K) return false;
  return !__builtin_amdgcn_readfirstlane(more);
}

// The done test of the step L ran in the previous iteration (Env.h:216-218),
// on the records -- the ledger after the orders, the tick's prices, cash, the
// price-independent sums and the refused-order flag.  The ONE definition:
// the finish role's own test, and (one-step launches, TAIL_EXACT) the
// generator's and the ledger's copies of it, which must agree with the
// finish role's reset flag -- a term added here reaches all three.  q and
// curEq: the post-tick sums and equity (the finish role's reward reads them)
template <int M, int S, bool ONE>
__device__ __forceinline__ bool rec_done(const double (&Lr)[M], const double (&P)[M], double cashv, double ml,
                                         double shv, double b, bool any_mc, const KParams& p, Sums& q,
                                         double& curEq) {
  double tlp[M];
#pragma unroll
  for (int m = 0; m < M; ++m) tlp[m] = Lr[m] * P[m];
  q.lp = canon<M, S, ONE>(tlp);
  q.ml = ml;
  q.sh = shv;
  q.b = b;
  curEq = (cashv + q.lp) - q.b;
  return any_mc || margin_call(q, cashv, p.mainM) || (curEq < 0.1 * p.init_cash);
}

// TR_REFILL (WIN): the iteration's tick was an auto-reset refill tick
// (initialize_history's env.step(), preprocessor.py:191-194): F pushes its
// window row, nothing else
enum { TR_STEP = 1, TR_ANYMC = 2, TR_MCALL = 4, TR_REFILL = 8 };

// NST: per env, the ring and the pop's summands in slots of nst_pad(n, S)
// doubles: n rounded up to a multiple of max(8, S) -- a pop writes whole
// rounds of S summands (R S slots, R = ceil(len / S)) and the ordered sum
// reads R S / 2 pairs, so at S = 16 a multiple of 8 would run into the next
// env's ring; 64-B aligned
__host__ __device__ constexpr int nst_pad(int n, int S) {
  return (n + (S > 8 ? S : 8) - 1) / (S > 8 ? S : 8) * (S > 8 ? S : 8);
}

// per asset slot (M per lane: slot (env, asset) at el APAD + ls M + m)
template <int S, int TW = TRIO_W, int M = 1>
struct TrioShared {
  static constexpr int TRIO_W = TW;
  static constexpr int EPB = TRIO_W / S;
  static constexpr int NSL = TRIO_W * M;  // asset slots of the block
  // prices after the iteration's tick (G -> L, F) and their refined
  // reciprocals (G -> L: the unit size's division, rcp_refined)
  double price[2][NSL], prcp[2][NSL];
  // the orders L ran (L -> F): ledger after the orders, responses, L*P before
  double rL[2][NSL], rTp[2][NSL], rTu[2][NSL], rTc[2][NSL], rPv[2][NSL];
  int32_t rRk[2][NSL];
  // per env: cash and the three price-independent sums after the orders,
  // equity before the step, the step index and TR_* flags
  double rCash[2][EPB], rMl[2][EPB], rSh[2][EPB], rB[2][EPB], rPrevEq[2][EPB];
  double rLpA[2][EPB];  // the sum L*P after the orders at the step's pre-tick prices (F: marginCall)
  int32_t rK[2][EPB], rFlags[2][EPB];
  // F -> G, L: the step F evaluated ended its episode and the env resets
  int32_t reset[2][EPB];
  uint64_t ts[2][EPB];  // timestamp after the tick (G -> F when F stores it)
  int32_t more[3];
  // RP (replay tape): the tick's tape row and dataEnd flag per env, the
  // lane's feature column value (F <= S) -- G -> F for State.price / windows
  int64_t row[2][EPB];
  uint32_t dend[2][EPB];
  double feat[2][NSL];
  // WIN with a log window: the tick's log-normalised prices, formed by the
  // generator role for the finish role's window rows
  double lprice[2][NSL];
};

// LDS of k_step_trio<S, ..., TW, NST, ..., M>: its static arrays (an upper
// bound of the compiler's layout) plus, for NST, the rings in dynamic LDS; the
// launcher's eligibility test keeps the sum within a workgroup's 160 KiB
// (kTrioLdsMax, mgn_launch.h)
template <int S, int TW, bool NST, int M = 1>
constexpr size_t trio_static_lds() {
  return sizeof(TrioShared<S, TW, M>) + (size_t)(TW / S) * sizeof(EnvRecs<S * M>) +
         S * M * sizeof(mgn_asset_source) + (MGN_MAX_ASSETS + 1) * sizeof(double) +
         (NST ? 2 * MGN_MAX_NSTEP : 1) * sizeof(double) + 256;  // s_disc (+ s_disc2 of the running pop)
}

// The replay tape's tick for the lane's M slots (duo_replay_tick's, per slot:
// feature column fcol + m when the row's features are spread one per slot)
template <int M>
struct RpCurM {
  double curF[M];
  int64_t row;
  uint32_t dend;
};
template <int M>
struct RpNextM {
  double P[M], F[M];
  uint64_t ts;
  uint32_t dend;
};
template <int M>
__device__ __forceinline__ void trio_replay_tick(Lane<M>& s, const KParams& p, uint64_t& ts, RpCurM<M>& cur,
                                                 RpNextM<M>& nx) {
  const int64_t row = s.rcur;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const bool fown = s.fcol >= 0 && s.fcol + m < p.F;
    if (s.pf_ok) {
      if (s.valid[m]) s.P[m] = nx.P[m];
      if (fown) cur.curF[m] = nx.F[m];
    } else {
      if (s.valid[m]) s.P[m] = p.rp_price[(size_t)row * p.A + s.asset[m]];
      if (fown) cur.curF[m] = p.rp_feat[(size_t)row * p.F + s.fcol + m];
    }
  }
  if (s.pf_ok) {
    ts = nx.ts;
    cur.dend = nx.dend;
  } else {
    ts = p.rp_ts[row];
    cur.dend = p.rp_end[row];
  }
  cur.row = row;
  s.row = row;
  s.rcur = (row + 1 == p.rp_rows) ? 0 : row + 1;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    if (s.valid[m]) nx.P[m] = p.rp_price[(size_t)s.rcur * p.A + s.asset[m]];
    if (s.fcol >= 0 && s.fcol + m < p.F) nx.F[m] = p.rp_feat[(size_t)s.rcur * p.F + s.fcol + m];
  }
  nx.ts = p.rp_ts[s.rcur];
  nx.dend = p.rp_end[s.rcur];
  s.pf_ok = true;
}
// per env: the ring and the finish role's pop summands
inline size_t trio_nst_dyn_lds(int S, int TW, int nstep) {
  return (size_t)(TW / S) * 2 * nst_pad(nstep, S) * sizeof(double);
}

// OMC: the output set when known at compile time (O_ALL, O_STD), else 0.
// WIN: the handle keeps a window (StackerDiscrete ring, and the launch
// history under mgn_rollout_hist).  The window rows are pushed by F, which
// only ever sees confirmed steps, so a rolled-back speculative step leaves no
// row; an auto-reset refills the window with W ticks (the rollback
// iteration's reset tick and W - 1 more) during which L does not step and F
// pushes one refill row per tick -- the rows, order and history marks of
// k_step_duo / k_step.
// NST: n-step aggregation (nstep > 1, scalar reward D = 1) in the finish
// role: the env's NStepBuffer ring and one pop's summands in dynamic LDS
// (launch_trio sizes it: envs per block x 2 nst_pad(n, S) doubles), the discounts staged
// in LDS, so a pop is n LDS reads issued together, not n dependent loads.
// GK >= 0: every asset's source is of kind GK (the generator role's per-lane
// kind dispatch folds away: TrendOU at C3).
// RP: every asset from the replay tape (HDFSourceSingle, DataSource.cpp:
// 391-398): G reads the tape one row ahead instead of ticking (duo_replay_tick)
// and publishes the row, its dataEnd flag and the lane's feature value; F
// writes State.price and the window rows from the tape's feature row.  The
// replay source carries on through a reset (DataSource.cpp:200-206), so the
// reset's getData reads the row the voided speculative tick read: a rollback
// keeps the tick's state as the reset tick's.
// the generator state of a lane's slots (what src_reset / gen_tick change),
// field by field: a whole-struct copy of Lane went through scratch memory.
// The variate cache (zc, ztag) is not state: an entry is the draw its tag
// names whichever tick cached it, so a dropped candidate's entry stays valid
template <int M>
__device__ __forceinline__ void gen_state_copy(Lane<M>& d, const Lane<M>& s) {
#pragma unroll
  for (int m = 0; m < M; ++m) {
    d.P[m] = s.P[m];
    d.sx[m] = s.sx[m];
    d.oum[m] = s.oum[m];
    d.dy[m] = s.dy[m];
    d.tlen[m] = s.tlen[m];
    d.tfl[m] = s.tfl[m];
  }
  d.dskip = s.dskip;
}

// MM: asset slots per lane (2: a 16-asset env on 8 lanes per role, so 8192
// envs fit one workgroup per CU; slots ls MM + m in the canonical order, the
// ledger's broker_spec_m2; one-step rewards with a scalar shaper, D = 1)
template <int S, bool RQ1, bool DISC, uint32_t OMC = 0, bool WIN = false, int TW = TRIO_W, int NST = 0,
          int GK = -1, bool RP = false, int MM = 1, bool ONE = false, bool K1 = false>
// The leading pointer arguments are the ledger role's state and actions:
// built with -amdgpu-kernarg-preload-count (madigan_amd/build.py) they arrive
// in SGPRs with the wave, so the orders' loads issue without waiting for the
// kernel-argument segment (a one-step launch is one dependent chain)
#ifdef MGN_TRIO_WPE4
// (mgn_launch_a8k1w.hip defines it: the one-step launches of large batches,
// one wave per role at four waves per SIMD -- 128 VGPRs, five 192-thread
// workgroups per CU, each an independent serial chain)
__global__ __attribute__((amdgpu_flat_work_group_size(1, 3 * TW), amdgpu_waves_per_eu(4))) void k_step_trio(
#else
__global__ __launch_bounds__(3 * TW, 1) void k_step_trio(
#endif
                                                          const double* __restrict__ kL,
                                                          const double* __restrict__ kmep,
                                                          const double* __restrict__ kBm,
                                                          const double* __restrict__ kP,
                                                          const double* __restrict__ kcash,
                                                          const int8_t* __restrict__ act_in, KParams p,
                                                          mgn_traj out, int in_kind_rt,
                                                          const double* __restrict__ units_in,
                                                          const int32_t* __restrict__ aidx_in, int K) {
  MGN_IT(0, 0);
  // the argument segment: 6 leading pointers, KParams, mgn_traj, in_kind_rt
  // (padded to 8), units_in, aidx_in, K
  warm_kernargs<(int)(48 + sizeof(KParams) + sizeof(mgn_traj) + 8 + 16 + 4)>();
  MGN_IT(47, 0);
  const int in_kind = DISC ? IN_DISCRETE : in_kind_rt;
  constexpr int M = MM;
  // TAIL: one-step launches (K1, an instantiation of their own: the code
  // would cost the longer launches registers), one slot per lane
  constexpr bool TAIL = K1 && !RP && !WIN && MM == 1;
  constexpr bool GLOG = WIN && !RP;
  constexpr int NPADS = 2;  // NST: ring, pop summands
  // NST == 2: the running-sum pop (MGN_NSTEP_POP_RUNNING, nrun_pop; the host
  // routes only DSR / DDR / PPC / none here); NST == 1: the exact pop
  constexpr bool NRUN = NST == 2;
  // sortino_shaperB's running pop: the one-wave-per-role layouts only (the
  // windowed and small-batch handles, R1 among them); at 256 lanes its code
  // would spill the running kernels (the launcher runs the exact pop there)
  constexpr bool SBR = NRUN && TW == 64;
  static_assert(M == 1 || (M == 2 && !NST), "two slots per lane: one-step rewards");
  static_assert(!ONE || (S == 2 && M == 1), "a one-asset env on two lanes per role");
  constexpr int APAD = S * M;
  constexpr int TRIO_W = TW;
  constexpr int TRIO_BLOCK = 3 * TW;
  constexpr int EPB = TRIO_W / S;
  __shared__ TrioShared<S, TW, M> sh;
  __shared__ EnvRecs<APAD> recs[EPB];
  __shared__ mgn_asset_source s_src[APAD];
  __shared__ double s_tgt[MGN_MAX_ASSETS + 1];
  __shared__ double s_disc[NST ? MGN_MAX_NSTEP : 1];                     // NST: gamma^k
  __shared__ double s_disc2[SBR ? MGN_MAX_NSTEP : 1];                     // SBR: (gamma^k)^(1/exp)
  extern __shared__ __attribute__((aligned(16))) double s_nst[];          // NST: (EPB, NPADS nst_pad(n, S))
  const int role = threadIdx.x / TRIO_W;  // 0 generator, 1 ledger, 2 finish
  const int l = threadIdx.x % TRIO_W;
  // GSLOT: a handle whose assets are of several source kinds (a Composite)
  // gives its generator lanes slot-major: lane l ticks asset slot l / EPB of
  // env l % EPB, so a generator wave holds 64 / EPB asset slots of every env
  // of the block -- one or two source kinds -- instead of every slot of a
  // few envs, each kind's branch executed by the waves that hold it (the
  // Composite's Sine, OU and TrendOU branches no longer run in every
  // generator wave).  Records stay env-major: the lane publishes at el S + ls.
  constexpr bool GSLOT = GK < 0 && !RP && TW / S > 1 && M == 1;
  // TAIL_EXACT (one-step launches, env-major generator lanes): the generator
  // and the ledger evaluate the finish role's done test themselves in the
  // launch's last iteration (rec_done) -- the generator forms the reset tick
  // only for the envs that end (not as a candidate for every env), and both
  // write their final state back during that iteration instead of after it
  constexpr bool TAIL_EXACT = TAIL && !GSLOT;
  const int el = (GSLOT && role == 0) ? l % EPB : l / S;
  const int ls = (GSLOT && role == 0) ? l / EPB : l % S;
  const int lx = (el * S + ls) * M;  // the lane's first (env, asset) slot record index
  const int env = blockIdx.x * EPB + el;
  const bool live = env < p.N;
  const int envc = live ? env : 0;
  const int A = p.A;
  Lane<M> s;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    s.asset[m] = ls * M + m;
    s.valid[m] = live && ls * M + m < A;
  }
  s.rcur = 0;
  s.row = 0;
  s.pf_ok = false;
  s.fcol = (RP && p.F <= APAD) ? ls * M : -1;  // RP: one feature column per slot
  const size_t li = (size_t)envc * A + (s.valid[0] ? ls * M : 0);  // the lane's first slot (valid[m] => valid[0])
  // QREG: the handle's one source kind is known at compile time (GK), so the
  // generator lanes hold their asset's few parameters in registers, loaded
  // with the state (TrendOU: q[0..8], OU: q[0..2]) -- no LDS staging, and no
  // prologue barrier: every role starts its first iteration as soon as its
  // own state arrives (the one-step launch's prologue was two memory round
  // trips and a barrier before the orders could start)
  constexpr int NQ = (RP || M > 1) ? 0 : GK == MGN_SRC_TRENDOU ? 9 : GK == MGN_SRC_OU ? 3 : 0;
  constexpr bool QREG = NQ > 0;
  double qr[QREG ? NQ : 1];
  const double* const tgt_g = p.target;  // the PPC target in global memory (F's prologue)
#pragma unroll
  for (int m = 0; m < M; ++m) {
    // the finish role takes its prices from the generator's LDS records
    s.P[m] = kAblPro ? 5.0 : ((s.valid[m] && role != 2) ? kP[li + m] : 0.);
    s.L[m] = s.mep[m] = s.Bm[m] = s.sx[m] = s.oum[m] = s.dy[m] = 0.;
    s.tlen[m] = 0;
    s.tfl[m] = 0;
  }
  // role state, loaded before the parameter staging (one round trip)
  uint64_t ts = 0;                             // G
  double cash = 0.;                            // L
  int act_cur[M] = {};                         // L
  const MGN_G int8_t* act_lane = vptr(act_in) + li;
  double ep_ret = 0., ep_len = 0., n_done = 0.;  // F
  double shA = 0., shB = 0.;                     // F
  int32_t rhead = 0, rlen = 0;                   // F (WIN): the window ring
  int32_t nlen = 0, nhead = 0;                   // F (NST): NStepBuffer fill count / oldest index
  NstRun nrs{0., 0., 0., 0., 0., 0.};             // F (NRUN): the buffer's running sums, on every lane of the env
  int32_t nsl = 0;                               // F (NRUN): pops since the sums were last formed from the ring
  if (!kAblPro && role == 0) {
    // only the fields the kind reads (GK): TrendOU no sine phase, OU none
    constexpr bool r_sx = GK < 0 || GK == MGN_SRC_SINE || GK == MGN_SRC_SAWTOOTH || GK == MGN_SRC_TRIANGLE ||
                          GK == MGN_SRC_TRENDYOU;
    constexpr bool r_oum = GK < 0 || GK == MGN_SRC_TRENDOU || GK == MGN_SRC_TRENDYOU || GK == MGN_SRC_OUPAIR;
    constexpr bool r_trend = GK < 0 || GK == MGN_SRC_TRENDOU || GK == MGN_SRC_SIMPLETREND ||
                             GK == MGN_SRC_TRENDYOU;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      if (s.valid[m]) {
        if (r_sx) s.sx[m] = p.sx[li + m];
        if (r_oum) s.oum[m] = p.oum[li + m];
        if (r_trend) {
          s.dy[m] = p.dy[li + m];
          s.tlen[m] = p.tlen[li + m];
          s.tfl[m] = p.tfl[li + m];
        }
      }
    }
    if constexpr (QREG) {
      const double* q = p.src[s.valid[0] ? ls : 0].p;
#pragma unroll
      for (int i = 0; i < NQ; ++i) qr[i] = q[i];
    }
    ts = p.ts[envc];
    s.dskip = p.dskip[envc];
    if (RP) s.rcur = p.rcur[envc];
  } else if (role == 1) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      if (s.valid[m]) {
        s.L[m] = kL[li + m];
        s.mep[m] = kmep[li + m];
        s.Bm[m] = kBm[li + m];
      }
    }
    cash = kcash[envc];
    if (in_kind == IN_DISCRETE && K > 0) {
#pragma unroll
      for (int m = 0; m < M; ++m) act_cur[m] = (m == 0 || s.valid[m]) ? act_lane[m] : 0;
    }
  } else {
    ep_ret = p.ep[(size_t)envc * 2];
    ep_len = p.ep[(size_t)envc * 2 + 1];
    n_done = p.epstats[(size_t)envc * 4 + 3];
    if (WIN) {
      rhead = p.rhead[envc];
      rlen = p.rlen[envc];
    }
    if (M > 1 || p.D == 1) {  // M > 1: D = 1 (launch_trio)
      shA = p.sA[envc];
      shB = p.sB[envc];
    } else if (s.valid[0]) {
      shA = p.sA[li];
      shB = p.sB[li];
    }
    if constexpr (NST != 0) {
      nlen = p.nlen[envc];
      nhead = p.nhead[envc];
      // the env's ring into LDS (every lane of the env copies a share)
      double* ring = s_nst + (size_t)el * NPADS * nst_pad(p.nstep, S);
      for (int i = ls; i < p.nstep; i += S) {
        const double x = p.nring[(size_t)envc * p.nstep + i];
        ring[i] = x;
        if constexpr (NRUN) {  // the sums of the entries the lane copied (position k from the oldest)
          int k = i - nhead;
          k += (k < 0) ? p.nstep : 0;
          if (SBR && p.shaper == MGN_SHAPER_SORTINO_B) {
            // (each entry's root kept beside the ring, in the summands' slots)
            const double rt = (x < 0.) ? root_e(-x, p.sexp) : 0.;
            ring[nst_pad(p.nstep, S) + i] = rt;
            if (k < nlen) nrun_add_sb(nrs, x, rt, p.disc[k], p.disc2[k]);
          } else if (k < nlen) {
            nrun_add(nrs, x, p.disc[k]);
          }
        }
      }
      if constexpr (NRUN) nrun_allsum<S>(nrs);
    }
  }
  {
    if (!QREG) {
      const double* g = reinterpret_cast<const double*>(p.src);
      double* d = reinterpret_cast<double*>(s_src);
      const int n = p.A * (int)(sizeof(mgn_asset_source) / sizeof(double));
      for (int i = threadIdx.x; i < n; i += TRIO_BLOCK) d[i] = g[i];
    }
    // read by the finish role from iteration 1 on (after iteration 0's barrier)
    if (p.target)
      for (int i = threadIdx.x; i <= p.A; i += TRIO_BLOCK) s_tgt[i] = p.target[i];
    if (NST)
      for (int i = threadIdx.x; i < p.nstep; i += TRIO_BLOCK) {
        s_disc[i] = p.disc[i];
        if constexpr (SBR) s_disc2[i] = p.disc2[i];
      }
    p.src = s_src;
    if (p.target) p.target = s_tgt;
  }
  // iteration 0 reads no record of another role (no step before it, no reset
  // pending: the j > 0 tests below), and `more` is read from iteration K >= 1
  // on, after G zeroed its slot one iteration earlier
  if (threadIdx.x == 0) {
    sh.more[0] = 0;
    sh.more[1] = 0;
    sh.more[2] = 0;
  }
  MGN_ST(if (threadIdx.x < 8) s_duo_sub[threadIdx.x] = 0;)
  if (!QREG || K == 0) __syncthreads();
  MGN_IT(1, 0);
#pragma unroll
  for (int m = 0; m < M; ++m) s.kind[m] = s.valid[m] ? (QREG ? GK : s_src[s.asset[m]].kind) : -1;

  // NST: a pop's summands (nstep_column's operands: summand kk of the entries
  // [head, head + len) on lane kk mod S, kNstU rounds evaluated together
  // on clamped operands so their chains interleave, slots [len, R S) +0.0)
  // into scr, and their ordered sum in kk order (S per chunk, the next
  // chunk's reads issued before this chunk's adds; +0.0 slots leave it
  // unchanged: acc starts at +0.0 and is never -0.0).  The shaper's summand
  // is chosen once per pop, outside the rounds (a branch per summand kept the
  // rounds' chains from interleaving: n = 20 DDR 3.66 -> 3.80 us/step)
  const auto nst_rounds = [&](const double* ring, double* scr, int head, int len, auto term) {
    constexpr int U = kNstU;
    const int n = p.nstep;
    const int R = (len + S - 1) / S;
    for (int j = 0; j < R; j += U) {
      double rr[U], dd[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int kk = ls + (j + u) * S;
        int idx = head + kk;
        idx -= (idx >= n) ? n : 0;
        const bool ok = kk < len && j + u < R;
        rr[u] = ring[ok ? idx : 0];
        dd[u] = s_disc[ok ? kk : 0];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int kk = ls + (j + u) * S;
        const double t = kAblNstTerm ? rr[u] : term(rr[u], dd[u]);
        if (j + u < R) scr[kk] = (kk < len) ? t : 0.0;
      }
    }
  };
  const auto nst_summands = [&](const double* ring, double* scr, int head, int len, double A, double B,
                                const PopPre& c) {
    // (DDR / DSR: the denominators' reciprocals formed once per pop)
    if (p.shaper == MGN_SHAPER_DDR) {
      const DdrPreR cr{c.q, rt_rcp(c.q.dpos), rt_rcp(c.q.dneg)};
      nst_rounds(ring, scr, head, len, [&](double r, double d) { return d * ddr_one_r(r, A, B, cr); });
    } else if (p.shaper == MGN_SHAPER_DSR) {
      const double rden = rt_rcp(c.dden);
      nst_rounds(ring, scr, head, len, [&](double r, double d) { return d * dsr_one_r(r, A, B, c.dden, rden); });
    }
    else if (p.shaper == MGN_SHAPER_SORTINO_B)
      nst_rounds(ring, scr, head, len, [&](double r, double d) { return sortinoB_term(r, d, p.sexp); });
    else  // PPC / none: the stored value
      nst_rounds(ring, scr, head, len, [&](double r, double d) { return d * r; });
  };
  const auto nst_sum = [&](const double* scr, int len) {
    const int R = (len + S - 1) / S;
    if constexpr (kAblNstSum) return scr[0];
    double acc = 0.0;
    const d2* sc = reinterpret_cast<const d2*>(scr);
    d2 cur[S / 2];
#pragma unroll
    for (int u = 0; u < S / 2; ++u) cur[u] = sc[u];
    for (int j = 0; j < R; ++j) {
      d2 nxt[S / 2];
      const int jn = (j + 1 < R) ? j + 1 : j;
#pragma unroll
      for (int u = 0; u < S / 2; ++u) nxt[u] = sc[jn * (S / 2) + u];
#pragma unroll
      for (int u = 0; u < S / 2; ++u) {
        acc += cur[u].x;
        acc += cur[u].y;
      }
#pragma unroll
      for (int u = 0; u < S / 2; ++u) cur[u] = nxt[u];
    }
    return acc;
  };

  if (role == 0) {
    // ---------------- generator waves: tick of step j, State.price / timestamp
    p.seed = in_vgpr(p.seed);
    p.env_offset = in_vgpr(p.env_offset);
    drain_vmem();
    MGN_IT(54, 0);
    int k = 0;
    // the source state before the last speculative tick (restored when F
    // finds that the previous step ended the episode)
    // (only the fields the kind's source reset leaves as they are: with GK
    // known the others are overwritten by src_reset right after the restore)
    constexpr bool SV_P = GK < 0 || !(GK == MGN_SRC_TRENDOU || GK == MGN_SRC_SIMPLETREND ||
                                      GK == MGN_SRC_TRENDYOU || GK == MGN_SRC_OUPAIR);
    constexpr bool SV_SX = GK < 0 || GK != MGN_SRC_TRENDYOU;
    constexpr bool SV_OUM = GK < 0 || !(GK == MGN_SRC_TRENDOU || GK == MGN_SRC_TRENDYOU || GK == MGN_SRC_OUPAIR);
    constexpr bool SV_TLEN = GK < 0 || !(GK == MGN_SRC_TRENDOU || GK == MGN_SRC_SIMPLETREND || GK == MGN_SRC_TRENDYOU);
    constexpr bool SV_TFL = GK < 0 || GK != MGN_SRC_SIMPLETREND;
    double svP[M] = {}, svSx[M] = {}, svOum[M] = {}, svDy[M] = {};
    int32_t svTlen[M] = {};
    uint8_t svTfl[M] = {};
    uint64_t svTs = 0;
    // TAIL: the state before the tail reset candidate (s holds the candidate
    // while `shadow`), and the last iteration
    Lane<M> s2;
    gen_state_copy<M>(s2, s);
    uint64_t ts2 = 0;
    bool shadow = false, tail_it = false, stored = false;
    int jlast = 0;
    __builtin_amdgcn_s_setprio(kPrioG);
    MGN_ST(unsigned long long T0 = 0, T1 = 0, T2 = 0, acc0 = 0, acc1 = 0; int jn = 0;)
    int gpend = 0;  // WIN: refill ticks still to come after the reset tick
    RpCurM<M> rp{};  // RP: the current State's tape row, features, dataEnd
    RpNextM<M> rnx{};
    // one tick: the tape row (RP; its timestamp) or the generator and ++ts
    auto tick = [&]() {
      if constexpr (RP) {
        trio_replay_tick<M>(s, p, ts, rp, rnx);
      } else {
        gen_tick<M, false, false, GK, true, (M > 1)>(s, p, env, ts, QREG ? qr : nullptr);
        ts = ts + 1;
      }
    };
    // the source state write-back at exit; fields a kind never writes are
    // not stored (their value in HBM is the one loaded).  (Storing it in the
    // first idle iteration, under the finish role's last iteration, measured
    // 1-2.5 % slower per step: profiles/r03k_early_store_fast_rt_ab.txt.)
    auto g_store = [&]() {
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const int kd = GK >= 0 ? GK : s.kind[m];
        const bool w_sx =
            kd == MGN_SRC_SINE || kd == MGN_SRC_SAWTOOTH || kd == MGN_SRC_TRIANGLE || kd == MGN_SRC_TRENDYOU;
        const bool w_oum = kd == MGN_SRC_TRENDOU || kd == MGN_SRC_TRENDYOU || kd == MGN_SRC_OUPAIR;
        const bool w_trend = kd == MGN_SRC_TRENDOU || kd == MGN_SRC_SIMPLETREND || kd == MGN_SRC_TRENDYOU;
        if (s.valid[m]) {
          const size_t i = (size_t)env * A + s.asset[m];
          p.P[i] = s.P[m];
          if (w_sx) p.sx[i] = s.sx[m];
          if (w_oum) p.oum[i] = s.oum[m];
          if (w_trend) {
            p.dy[i] = s.dy[m];
            p.tlen[i] = s.tlen[m];
            p.tfl[i] = s.tfl[m];
          }
        }
      }
      if (ls == 0) {
        p.ts[env] = ts;
        p.dskip[env] = s.dskip;
      }
    };
    for (int j = 0;; ++j) {
      const int cur = j & 1, prv = cur ^ 1;
      MGN_T(T0);
      if (threadIdx.x == 0) sh.more[(j + 1) % 3] = 0;
      if (live) {
        if constexpr (TAIL) {
          // another iteration: the previous one's candidate is dropped (a
          // reset found there is run below as any other)
          if (shadow) {
            gen_state_copy<M>(s, s2);
            ts = ts2;
            shadow = false;
          }
        }
        const bool rst = j > 0 && sh.reset[prv][el] != 0;
        const bool prev_step = j > 0 && (sh.rFlags[prv][el] & TR_STEP) != 0;
        // every branch's tick is the one call below (one copy of the
        // generator's code: the kind dispatch of every slot, inlined once)
        bool tk = false;
        if (WIN && !rst && gpend > 0) {
          // a refill tick (not speculative: the reset is confirmed)
          tk = true;
          gpend -= 1;
        } else if (RP && rst) {
          // the replay source carries on: the reset's getData reads the row the
          // voided speculative tick read, whose state stands; after a step that
          // was not speculated (none ran in the previous iteration) it reads the next
          if (prev_step) k -= 1;
          else tk = true;
          s.dskip += 1;  // Env::reset counts (the draw index; no draws from a tape)
          if (WIN) gpend = p.W - 1;
        } else if (rst) {
          if (prev_step) {  // roll the speculative tick back
#pragma unroll
            for (int m = 0; m < M; ++m) {
              if (SV_P) s.P[m] = svP[m];
              if (SV_SX) s.sx[m] = svSx[m];
              if (SV_OUM) s.oum[m] = svOum[m];
              s.dy[m] = svDy[m];
              if (SV_TLEN) s.tlen[m] = svTlen[m];
              if (SV_TFL) s.tfl[m] = svTfl[m];
            }
            ts = svTs;
            k -= 1;
          }
          // Env::reset -> dataSource->reset + getData (Env.h:181-187)
          src_reset<M, false, GK>(s, p, env, ts, QREG ? qr : nullptr);
          tk = true;
          if (WIN) gpend = p.W - 1;
        } else if (k < K) {
          if (!RP) {
#pragma unroll
            for (int m = 0; m < M; ++m) {
              if (SV_P) svP[m] = s.P[m];
              if (SV_SX) svSx[m] = s.sx[m];
              if (SV_OUM) svOum[m] = s.oum[m];
              svDy[m] = s.dy[m];
              if (SV_TLEN) svTlen[m] = s.tlen[m];
              if (SV_TFL) svTfl[m] = s.tfl[m];
            }
            svTs = ts;
          }
          if constexpr (kAblG) ts = ts + 1;  // (prices frozen)
          else tk = true;
          k += 1;
        } else if (TAIL && K == 1) {
          // idle (the launch's ticks done, no reset pending): a reset the
          // finish role finds in this iteration -- Env::reset's source reset
          // and getData on the final state.  TAIL_EXACT: for the envs whose
          // step ends (rec_done, the finish role's own test); else a
          // candidate for every env, kept in s2 and adopted after the loop
          bool cand = true;
          if constexpr (TAIL_EXACT) {
            const int fl = sh.rFlags[prv][el];
            double Lr[M], Pr[M];
#pragma unroll
            for (int m = 0; m < M; ++m) {
              Lr[m] = sh.rL[prv][lx + m];
              Pr[m] = sh.price[prv][lx + m];
            }
            double eq;
            Sums qd;
            cand = p.auto_reset && (fl & TR_STEP) && !sh.reset[prv][el] &&
                   rec_done<M, S, ONE>(Lr, Pr, sh.rCash[prv][el], sh.rMl[prv][el], sh.rSh[prv][el],
                                       sh.rB[prv][el], (fl & TR_ANYMC) != 0, p, qd, eq);
            tail_it = true;
          }
          if (cand) {
            gen_state_copy<M>(s2, s);
            ts2 = ts;
            shadow = true;
            src_reset<M, false, GK>(s, p, env, ts, QREG ? qr : nullptr);
            tk = true;
          }
        }
        if (tk) tick();
        if constexpr (TAIL_EXACT) {
          // the final state, written back while the finish role evaluates
          if (tail_it) {
            g_store();
            stored = true;
          }
        }
      }
#pragma unroll
      for (int m = 0; m < M; ++m) {
        sh.price[cur][lx + m] = s.P[m];
        if (DISC) sh.prcp[cur][lx + m] = rcp_refined(s.P[m]);  // (the ledger's unit size)
      }
      if constexpr (GLOG) {
        // the window row's log price (StackerDiscrete's log normaliser,
        // preprocessor.py:79-81) off the finish role's chain
        if (p.ring_log != 0) {
#pragma unroll
          for (int m = 0; m < M; ++m) sh.lprice[cur][lx + m] = log_norm(s.P[m]);
        }
      }
      if (ls == 0) sh.ts[cur][el] = ts;
      if constexpr (RP) {
        if (ls == 0) {
          sh.row[cur][el] = rp.row;
          sh.dend[cur][el] = rp.dend;
        }
#pragma unroll
        for (int m = 0; m < M; ++m) sh.feat[cur][lx + m] = rp.curF[m];
      }
      if (j == 0) MGN_IT(48, 0);
      MGN_T(T1);
      __syncthreads();
      MGN_T(T2);
      MGN_IT(2 + (j < 40 ? j : 40), 0);
      MGN_ST(acc0 += T1 - T0; acc1 += T2 - T1; jn = j;)
      jlast = j;
      if (trio_exit(j, K, sh.more[j % 3])) break;
    }
    MGN_ST(if (threadIdx.x == 0) {
      atomicAdd(&g_duo_stamps[0], acc0);
      atomicAdd(&g_duo_stamps[1], acc1);
      atomicAdd(&g_duo_stamps[8], (unsigned long long)(jn + 1));
      atomicAdd(&g_duo_stamps[10], 1ull);
    })
    if constexpr (kAblEpi) return;
    if constexpr (TAIL) {
      // the last iteration's candidate stands where the finish role found the
      // episode's end there (a tail reset: it raised no further iteration)
      if (live && shadow && !sh.reset[jlast & 1][el]) {
        gen_state_copy<M>(s, s2);
        ts = ts2;
      }
    }
    if (live && !stored) {  // (TAIL_EXACT: written back in the last iteration)
      g_store();
      if (RP && ls == 0) p.rcur[env] = s.rcur;
    }
    MGN_IT_DRAIN();
    MGN_IT(44, 0);
    return;
  }

  if (role == 1) {
    // ---------------- ledger waves: Broker orders of step j
    const uint32_t om = OMC ? OMC : traj_mask(out);
    const MGN_G double* gunits = vptr(units_in);
    const MGN_G int32_t* gaidx = vptr(aidx_in);
    p.init_cash = in_vgpr(p.init_cash);
    p.mainM = in_vgpr(p.mainM);
    p.unit_size = in_vgpr(p.unit_size);
    const uint32_t act_step = (uint32_t)p.N * (uint32_t)A;
    const bool need_ar = (p.reward_mode != MGN_REWARD_ENV_LOG) || (om & O_AREW);  // as the finish role's
    // the Broker responses' outputs (per asset (k, env, asset), as the finish role's)
    struct {
      MGN_G double *tprice, *tunits, *tcost;
      MGN_G uint8_t* risk;
      MGN_G double *obs_price, *obs_port;  // TAIL_EXACT
    } ovl = {(om & O_TP) ? vptr(out.tprice) : nullptr, (om & O_TU) ? vptr(out.tunits) : nullptr,
             (om & O_TC) ? vptr(out.tcost) : nullptr, (om & O_RISK) ? vptr(out.risk) : nullptr,
             (TAIL_EXACT && (om & O_OPR)) ? vptr(out.obs_price) : nullptr,
             (TAIL_EXACT && (om & O_OPT)) ? vptr(out.obs_port) : nullptr};
    const uint32_t sNA = (uint32_t)p.N * (uint32_t)A, sNF = (uint32_t)p.N * (uint32_t)p.F,
                   sNA1 = (uint32_t)p.N * (uint32_t)(A + 1);
    const size_t bA = (size_t)env * A + s.asset[0], bP = (size_t)env * p.F + s.asset[0],
                 bO = (size_t)env * (A + 1);
    // sums of the ledger (canonical trees): ml, sh, b change only with the
    // orders, lp with the prices; `fresh` = recompute all four (start, reset)
    Sums sa = port_sums<M, S, ONE>(s.L, s.mep, s.Bm, s.P);
    drain_vmem();
    MGN_IT(51, TRIO_W);
    int k = 0;
    int lpend = 0;  // WIN: refill ticks still to come after the reset tick
    int jlast = 0;  // TAIL: the last iteration
    int lflags = 0;  // TAIL_EXACT: the flags of the last step run
    bool lstored = false;  // TAIL_EXACT: the ledger written back in the last iteration
    // the ledger write-back at exit
    auto l_store = [&]() {
#pragma unroll
      for (int m = 0; m < M; ++m) {
        if (s.valid[m]) {
          const size_t i = (size_t)env * A + s.asset[m];
          p.L[i] = s.L[m];
          p.mep[i] = s.mep[m];
          p.Bm[i] = s.Bm[m];
        }
      }
      if (ls == 0) p.cash[env] = cash;
    };
    __builtin_amdgcn_s_setprio(kPrioL);  // the orders are the critical path
    // (stamp builds: the ledger's phases -- prices + pre-order sums, units,
    // the Broker, the records)
    MGN_ST(unsigned long long T0 = 0, T1 = 0, T2 = 0, acc0 = 0, acc1 = 0;
           unsigned long long Lp1 = 0, Lp2 = 0, Lp3 = 0, lacc[4] = {0, 0, 0, 0};)
    for (int j = 0;; ++j) {
      const int cur = j & 1, prv = cur ^ 1;
      MGN_T(T0);
      MGN_ST(Lp1 = Lp2 = Lp3 = T0;)
      // one-step launches: in the last iteration the finish role's chain is
      // the critical path, this role's work (done test, State, write-back) not
      if (TAIL_EXACT && K == 1 && j == 1) __builtin_amdgcn_s_setprio(kPrioG);
      // the previous iteration's records -- reset, flags, the tick's prices
      // and their reciprocals -- read together ahead of the tests on them (a
      // compiler-only memory barrier keeps them from being sunk into the
      // branches; iteration 0 reads records no role wrote, and uses none)
      const int rs_rec = sh.reset[prv][el], fl_rec = sh.rFlags[prv][el];
      double p_rec[M], r_rec[M];
#pragma unroll
      for (int m = 0; m < M; ++m) {
        p_rec[m] = sh.price[prv][lx + m];
        r_rec[m] = DISC ? sh.prcp[prv][lx + m] : 0.;
      }
      asm volatile("" ::: "memory");
      const bool rst = live && j > 0 && rs_rec != 0;
      const bool prev_step = j > 0 && (fl_rec & TR_STEP) != 0;
      // WIN: this iteration's tick refills the window (the reset tick or one
      // of the W - 1 after it): no step
      const bool refill = WIN && live && (rst || lpend > 0);
      if (WIN && !rst && lpend > 0) lpend -= 1;
      // prices of the last tick (the step's pre-tick prices; iteration 0:
      // the handle's current prices)
#pragma unroll
      for (int m = 0; m < M; ++m)
        if (j > 0 && live && s.valid[m]) s.P[m] = p_rec[m];
      if (rst) {
        // the episode ended at the step F evaluated: the speculative step of
        // iteration j-1 is void; a fresh Broker (Env.h:181-187) waits for the
        // reset tick's prices
        if (prev_step) k -= 1;
#pragma unroll
        for (int m = 0; m < M; ++m) {
          s.L[m] = 0.;
          s.mep[m] = 0.;
          s.Bm[m] = 0.;
        }
        cash = p.init_cash;
        if (WIN) lpend = p.W - 1;
      }
      const bool stepping = live && !rst && !refill && k < K;
      int act_now[M];
#pragma unroll
      for (int m = 0; m < M; ++m) act_now[m] = act_cur[m];
      if (in_kind == IN_DISCRETE && K > 0) {
        // the action of the next step this lane runs (k + 1 if this one
        // steps; a rollback re-reads step k's, clamped in range)
        const int kn = k + (stepping ? 1 : 0);
        const MGN_G int8_t* ar = act_lane + kidx(kn < K ? kn : K - 1, act_step, 0);
#pragma unroll
        for (int m = 0; m < M; ++m) act_cur[m] = (m == 0 || s.valid[m]) ? ar[m] : 0;
      }
      int flags = 0;
      if (stepping) {
        const bool after_reset = prev_step ? false : true;
        Sums s0;
        if (after_reset && j > 0) {
          s0 = port_sums<M, S, ONE>(s.L, s.mep, s.Bm, s.P);  // after a reset tick
        } else if (j == 0) {
          s0 = sa;  // the prologue's sums of the handle's state and prices
        } else {
          double tlp[M];
#pragma unroll
          for (int m = 0; m < M; ++m) tlp[m] = s.L[m] * s.P[m];
          s0 = sa;
          s0.lp = canon<M, S, ONE>(tlp);
        }
        const double prevEq = (cash + s0.lp) - s0.b;  // Env.h:208
        if (j == 0) MGN_IT(58, TRIO_W);
        MGN_ST(Lp1 = __builtin_amdgcn_s_memtime();)
        double uc[M], tp[M], tu[M], tc[M], prevVal[M];
        int rk[M];
        const size_t oN = (size_t)k * p.N, oNA = (size_t)k * p.N * A;
#pragma unroll
        for (int m = 0; m < M; ++m) {
          tp[m] = 0.;
          tu[m] = 0.;
          tc[m] = 0.;
          rk[m] = MGN_GREEN;
          uc[m] = 0.;
          prevVal[m] = s.L[m] * s.P[m];
        }
        if (in_kind == IN_DISCRETE) {  // dqn.py:160-179
          const double bp = (cash + s0.sh) + (s0.lp - s0.ml);
          const double avM = RQ1 ? bp : bp / p.reqM;
          const int half = p.atoms / 2;
#pragma unroll
          for (int m = 0; m < M; ++m) {
            if (s.valid[m]) {
              // (unit_size avM) / P with the generator's reciprocal of P
              // (iteration 0 reads the handle's prices, not the generator's: no reciprocal)
              const double u = div_by_rcp(p.unit_size * avM, s.P[m], j > 0 ? r_rec[m] : 0.);
              uc[m] = (double)(act_now[m] - half) * u;
              if (act_now[m] == 0) uc[m] = (s.L[m] != 0) ? -s.L[m] : 0.;
            }
          }
        } else if (in_kind == IN_UNITS) {
#pragma unroll
          for (int m = 0; m < M; ++m) uc[m] = s.valid[m] ? gunits[oNA + (size_t)env * A + s.asset[m]] : 0.;
        } else if (in_kind == IN_SINGLE) {
          const int ai = gaidx[env];
          const double u = gunits[oN + env];
#pragma unroll
          for (int m = 0; m < M; ++m) uc[m] = (s.valid[m] && s.asset[m] == ai) ? u : 0.;
        }
        if constexpr (M > 1) {
          // published before the orders (not live across them: the
          // 168-register budget at two slots per lane)
#pragma unroll
          for (int m = 0; m < M; ++m)
            if (need_ar) sh.rPv[cur][lx + m] = prevVal[m];
          if (ls == 0) sh.rPrevEq[cur][el] = prevEq;
        }
        Sums after = s0;
        int any_mc = 0;
        MGN_ST(Lp2 = __builtin_amdgcn_s_memtime();)
        if (!kAblL && in_kind != IN_NONE) {
          if (j == 0) MGN_IT(52, TRIO_W);
          if constexpr (M == 1)
            broker_spec<S, RQ1, ONE>(s, p, recs[el], cash, uc, tp, tu, tc, rk, ls, after, any_mc);
          else
            broker_spec_m2<S, RQ1>(s, p, recs[el], cash, uc, tp, tu, tc, rk, ls, after, any_mc);
          if (j == 0) MGN_IT(53, TRIO_W);
        }
        MGN_ST(Lp3 = __builtin_amdgcn_s_memtime();)
        sa = after;
#pragma unroll
        for (int m = 0; m < M; ++m) {
          sh.rL[cur][lx + m] = s.L[m];
          if (need_ar) {  // the agent reward's operands: the orders' responses, L * P before them
            sh.rTp[cur][lx + m] = tp[m];
            sh.rTu[cur][lx + m] = tu[m];
            sh.rTc[cur][lx + m] = tc[m];
            if (M == 1) sh.rPv[cur][lx + m] = prevVal[m];
          }
          // the step's Broker responses (EnvInfo: transaction price / units /
          // cost, risk) are stored here rather than by the finish role: a
          // speculative step that F voids runs again under the same k, and
          // its stores overwrite these
          if (s.valid[m]) {
            const size_t i = kidx(k, sNA, bA) + m;
            if (om & O_TP) ost(ovl.tprice + i, tp[m]);
            if (om & O_TU) ost(ovl.tunits + i, tu[m]);
            if (om & O_TC) ost(ovl.tcost + i, tc[m]);
            if (om & O_RISK) ost(ovl.risk + i, (uint8_t)rk[m]);
          }
        }
        if (ls == 0) {
          sh.rCash[cur][el] = cash;
          sh.rMl[cur][el] = after.ml;
          sh.rSh[cur][el] = after.sh;
          sh.rB[cur][el] = after.b;
          if (M == 1) sh.rPrevEq[cur][el] = prevEq;
          sh.rLpA[cur][el] = after.lp;
          sh.rK[cur][el] = k;
        }
        // the Broker's post-order margin check (Broker.cpp:156-157) is the
        // finish role's (marginCall output), off this role's chain
        flags = TR_STEP | (any_mc ? TR_ANYMC : 0) | (in_kind != IN_NONE ? TR_MCALL : 0);
        lflags = flags;
        k += 1;
      }
      if constexpr (TAIL_EXACT) {
        // one-step launches, the last iteration: the finish role's done test
        // on this env's step (rec_done); an episode that ends leaves the fresh
        // Broker (Env.h:181-187).  The final ledger is written back here,
        // while the finish role evaluates the step.  The step's State (prices
        // and ledgerNormedFull, preprocessor-independent) is stored here too,
        // from the finish role's operands with its operations (the step of
        // iteration 0 is never voided: no reset is pending in iteration 1), so
        // the finish role's chain keeps only the reward, done and shaping
        if (K == 1 && j == 1 && live) {
          if (lflags & TR_STEP) {
            double curEq;
            Sums qd;
            const bool dn =
                rec_done<M, S, ONE>(s.L, s.P, cash, sa.ml, sa.sh, sa.b, (lflags & TR_ANYMC) != 0, p, qd, curEq);
            const int ks = k - 1;  // the step's index
#pragma unroll
            for (int m = 0; m < M; ++m) {
              if (s.valid[m]) {
                if (om & O_OPR) ost(ovl.obs_price + (kidx(ks, sNF, bP) + m), s.P[m]);
                if (om & O_OPT) ost(ovl.obs_port + (kidx(ks, sNA1, bO) + 1 + s.asset[m]), (s.L[m] * s.P[m]) / curEq);
              }
            }
            if (ls == 0 && (om & O_OPT)) ost(ovl.obs_port + kidx(ks, sNA1, bO), (cash - sa.b) / curEq);
            if (p.auto_reset && dn) {
#pragma unroll
              for (int m = 0; m < M; ++m) {
                s.L[m] = 0.;
                s.mep[m] = 0.;
                s.Bm[m] = 0.;
              }
              cash = p.init_cash;
            }
          }
          l_store();
          lstored = true;
        }
      }
      if (WIN && refill) {
        // the refill row's portfolio (the fresh Broker's): F evaluates it
#pragma unroll
        for (int m = 0; m < M; ++m) sh.rL[cur][lx + m] = s.L[m];
        if (ls == 0) {
          sh.rCash[cur][el] = cash;
          sh.rB[cur][el] = 0.;  // canonical sum of the fresh Broker's borrowed margins (+0)
        }
        flags = TR_REFILL;
      }
      if (ls == 0) sh.rFlags[cur][el] = flags;
      // another iteration: F evaluates this step, or steps remain (a reset
      // that voided nothing leaves none: its tick ran in this iteration;
      // WIN: its refill rows follow)
      if (live && (stepping || refill || k < K || (WIN && (rst || lpend > 0)))) sh.more[j % 3] = 1;
      jlast = j;
      if (j == 0) MGN_IT(49, TRIO_W);
      MGN_T(T1);
      __syncthreads();
      MGN_T(T2);
      MGN_ST(acc0 += T1 - T0; acc1 += T2 - T1;
             if (Lp3 != T0) {  // an iteration that stepped
               lacc[0] += Lp1 - T0;
               lacc[1] += Lp2 - Lp1;
               lacc[2] += Lp3 - Lp2;
               lacc[3] += T1 - Lp3;
             })
      if (trio_exit(j, K, sh.more[j % 3])) break;
    }
    MGN_ST(if (l == 0) {
      atomicAdd(&g_duo_stamps[4], acc0);
      atomicAdd(&g_duo_stamps[5], acc1);
      for (int i = 0; i < 3; ++i) atomicAdd(&g_duo_stamps[13 + i], s_duo_sub[i]);
      atomicAdd(&g_duo_stamps[18], s_duo_sub[5]);
      atomicAdd(&g_duo_stamps[19], s_duo_sub[6]);
      atomicAdd(&g_duo_stamps[2], s_duo_sub[3]);
      atomicAdd(&g_duo_stamps[3], s_duo_sub[4]);
      atomicAdd(&g_duo_stamps[6], s_duo_sub[7]);
      for (int i = 0; i < 4; ++i) atomicAdd(&g_duo_stamps[20 + i], lacc[i]);
    })
    if constexpr (kAblEpi) return;
    if constexpr (TAIL) {
      // a tail reset (the finish role found the episode's end in the last
      // iteration): the fresh Broker (Env.h:181-187)
      if (live && !lstored && sh.reset[jlast & 1][el]) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
          s.L[m] = 0.;
          s.mep[m] = 0.;
          s.Bm[m] = 0.;
        }
        cash = p.init_cash;
      }
    }
    if (live && !lstored) l_store();
    MGN_IT_DRAIN();
    MGN_IT(45, TRIO_W);
    return;
  }

  // ---------------- finish waves: step j-1's reward, done and outputs
  const uint32_t om = OMC ? OMC : traj_mask(out);
  const GTraj ov = traj_vgpr<OMC>(out);
  GState gs;
  gs.epstats = vptr(p.epstats);
  // WIN: the ring / launch-history pointers (global, as every store of the
  // loop) and the history cursor: next row, the step its rows belong to
  int hcnt = p.W, klast = 0;
  MGN_G int32_t *ghend = nullptr, *ghlen = nullptr;
  if (WIN) {
    gs.ring = vptr(p.ring);
    gs.ring_ts = vptr(p.ring_ts);
    gs.hist = vptr(p.hist);
    gs.hist_ts = vptr(p.hist_ts);
    ghend = vptr(p.hend);
    ghlen = vptr(p.hlen);
  }
  p.init_cash = in_vgpr(p.init_cash);
  p.mainM = in_vgpr(p.mainM);
  p.eta = in_vgpr(p.eta);
  p.cos_temp = in_vgpr(p.cos_temp);
  const int D = M > 1 ? 1 : p.D;
  LedOut g;
  g.shA = shA;
  g.shB = shB;
  g.cos_qn = 0.;
  if (p.shaper == MGN_SHAPER_PPC) {
    double qq[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const double q = s.valid[m] ? tgt_g[1 + s.asset[m]] : 0.;
      qq[m] = q * q;
    }
    g.cos_qn = sqrt(tgt_g[0] * tgt_g[0] + canon<M, S, ONE>(qq));
  }
  const bool need_ar = (p.reward_mode != MGN_REWARD_ENV_LOG) || (om & O_AREW);
  // one-step launches (TAIL_EXACT): the ledger role stores the step's State
  const bool lobs = TAIL_EXACT && K == 1;
  // output element strides per step (32-bit: checked on the host) and the
  // lane's bases: per asset (k, env, asset), State.price (k, env, feature),
  // State.portfolio (k, env, 0), per env (k, env)
  const uint32_t sN = (uint32_t)p.N, sNA = (uint32_t)p.N * (uint32_t)A, sNF = (uint32_t)p.N * (uint32_t)p.F,
                 sNA1 = (uint32_t)p.N * (uint32_t)(A + 1);
  const size_t bA = (size_t)env * A + s.asset[0], bP = (size_t)env * p.F + s.asset[0],
               bO = (size_t)env * (A + 1);  // slot m at + m
  // WIN: StackerDiscrete.stream_state of a State (preprocessor.py:172-175):
  // log-normalised (as the ring stores them) prices, ledgerNormedFull and the
  // timestamp into ring slot head + 1 and history row hcnt (ring_push's
  // values; duo_store's order)
  // State.price of the State G published at parity q into dst[0, F): the
  // lane's asset price, or (RP) the tape row's features (duo_feats' split:
  // one column per lane when F <= S, else read back per column); lg:
  // StackerDiscrete's log
  const auto put_price = [&](MGN_G double* dst, const double(&P)[M], bool lg, int q) {
    if constexpr (RP) {
      if (s.fcol >= 0) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
          if (s.fcol + m < p.F) {
            const double v = sh.feat[q][lx + m];
            ost(dst + (s.fcol + m), lg ? log_norm(v) : v);
          }
        }
      } else {
        const int64_t row = sh.row[q][el];
        for (int f = ls; f < p.F; f += S) {
          const double v = p.rp_feat[(size_t)row * p.F + f];
          ost(dst + f, lg ? log_norm(v) : v);
        }
      }
    } else {
#pragma unroll
      for (int m = 0; m < M; ++m)
        if (s.valid[m]) ost(dst + s.asset[m], lg ? log_norm(P[m]) : P[m]);
    }
  };
  const auto push_row = [&](const double(&P)[M], const double(&portA)[M], double port0, uint64_t tsv, int kmark,
                            int q) {
    rhead = (rhead + 1 == p.W) ? 0 : rhead + 1;  // (rhead in [0, W): no integer division)
    if (rlen < p.W) rlen += 1;
    const int R = p.F + A + 1;
    MGN_G double* row = gs.ring + ((size_t)env * p.W + rhead) * R;
    MGN_G double* hrow = p.hist ? gs.hist + ((size_t)env * p.hrows + hcnt) * R : nullptr;
    if constexpr (RP) {
      put_price(row, P, p.ring_log != 0, q);
      if (hrow) put_price(hrow, P, p.ring_log != 0, q);
    } else {
#pragma unroll
      for (int m = 0; m < M; ++m) {
        if (s.valid[m]) {
          // the slot's price column, normalised once for the ring and the history row
          const double pv = p.ring_log == 0 ? P[m] : (GLOG ? sh.lprice[q][lx + m] : log_norm(P[m]));
          ost(row + s.asset[m], pv);
          if (hrow) ost(hrow + s.asset[m], pv);
        }
      }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      if (s.valid[m]) {
        ost(row + (p.F + 1 + s.asset[m]), portA[m]);
        if (hrow) ost(hrow + (p.F + 1 + s.asset[m]), portA[m]);
      }
    }
    if (ls == 0) {
      ost(row + p.F, port0);
      ost(gs.ring_ts + ((size_t)env * p.W + rhead), tsv);
      if (hrow) {
        ost(hrow + p.F, port0);
        ost(gs.hist_ts + ((size_t)env * p.hrows + hcnt), tsv);
      }
    }
    if (hrow) {  // hist_mark
      klast = kmark;
      hcnt += 1;
      if (ls == 0) {
        ost(ghend + ((size_t)klast * p.N + env), (int32_t)hcnt);
        ost(ghlen + ((size_t)klast * p.N + env), (int32_t)rlen);
      }
    }
  };
  // the finish role's state write-back (the n-step ring's in the epilogue)
  bool fstored = false;
  const auto f_store = [&]() {
    if (ls == 0) {
      if (WIN) {
        p.rhead[env] = rhead;
        p.rlen[env] = rlen;
      }
      p.ep[(size_t)env * 2] = ep_ret;
      p.ep[(size_t)env * 2 + 1] = ep_len;
      if (D == 1) {
        p.sA[env] = g.shA;
        p.sB[env] = g.shB;
      }
    }
    if (D != 1 && s.valid[0]) {
      p.sA[(size_t)env * A + s.asset[0]] = g.shA;
      p.sB[(size_t)env * A + s.asset[0]] = g.shB;
    }
  };
  drain_vmem();
  __builtin_amdgcn_s_setprio(kPrioF);
  MGN_ST(unsigned long long T0 = 0, T1 = 0, T2 = 0, acc0 = 0, acc1 = 0, Tf1 = 0, Tf2 = 0, facc[3] = {0, 0, 0};)
  for (int j = 0;; ++j) {
    const int cur = j & 1, prv = cur ^ 1;
    MGN_T(T0);
    MGN_ST(Tf1 = Tf2 = 0;)
    int rst_out = 0;
    bool tail_rst = false;  // TAIL: the launch's last step ended its episode
    // the step L ran in iteration j-1, unless F voided it at iteration j-1
    const int flags = j > 0 ? sh.rFlags[prv][el] : 0;
    // the step's records are read with its flags, ahead of the tests on them
    // (one LDS round trip on this role's chain instead of three; iteration 0
    // reads records no role wrote, and uses none)
    const int rsv = j > 0 ? sh.reset[prv][el] : 0;
    const int krec = sh.rK[prv][el];
    double Lrec[M], Prec[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      Lrec[m] = sh.rL[prv][lx + m];
      Prec[m] = sh.price[prv][lx + m];
    }
    const double cashrec = sh.rCash[prv][el], prevrec = sh.rPrevEq[prv][el];
    // (a compiler-only memory barrier: the reads stay ahead of the tests --
    // the compiler would sink them into the branch -- and nothing waits here)
    asm volatile("" ::: "memory");
    if (!kAblF && live && (flags & TR_STEP) && !rsv) {
      const int k = krec;
      // NRUN: the sums re-formed from the ring every n pops (term kk on lane
      // kk mod S; the entries before this step's), then the step's first pop
      // less its new entry's term and that entry's weight and the oldest
      // entry, formed ahead of the reward chain (nrun_pre)
      NstPre npre{};
      double nst_w = 0., nst_r0 = 0., nst_w2 = 0., nst_rt0 = 0.;
      if constexpr (NRUN) {
        const int n = p.nstep;
        const double* ring = s_nst + (size_t)el * NPADS * nst_pad(n, S);
        if (nsl >= n) {
          nrun_zero(nrs);
          for (int kk = ls; kk < nlen; kk += S) {
            int idx = nhead + kk;
            idx -= (idx >= n) ? n : 0;
            if (SBR && p.shaper == MGN_SHAPER_SORTINO_B)
              nrun_add_sb(nrs, ring[idx], ring[nst_pad(n, S) + idx], s_disc[kk], s_disc2[kk]);
            else
              nrun_add(nrs, ring[idx], s_disc[kk]);
          }
          nrun_allsum<S>(nrs);
          nsl = 0;
        }
        nst_w = s_disc[nlen];
        nst_r0 = ring[nhead];
        if (SBR && p.shaper == MGN_SHAPER_SORTINO_B) {
          nst_w2 = s_disc2[nlen];
          nst_rt0 = ring[nst_pad(n, S) + nhead];
        }
        npre = nrun_pre(p.shaper, nrs, nlen + 1, g.shA, g.shB);
      }
      Lane<M> f = s;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        f.L[m] = Lrec[m];
        f.P[m] = Prec[m];
      }
      const double cashv = cashrec;
      const double prevEq = prevrec;
      // post-tick sums, equity, done (rec_done, the one definition), reward
      // (Env.h:211-223)
      Sums q;
      double curEq;
      const bool done = rec_done<M, S, ONE>(f.L, f.P, cashv, sh.rMl[prv][el], sh.rSh[prv][el], sh.rB[prv][el],
                                            (flags & TR_ANYMC) != 0, p, q, curEq);
      if (j == 1) MGN_IT(55, 2 * TRIO_W);
      const double ratio = curEq / prevEq;
      const double clampv = (in_kind == IN_SINGLE) ? 0.01 : 0.3;
      const double reward = log_ratio((ratio < clampv) ? clampv : ratio);
      if (j == 1) MGN_IT(56, 2 * TRIO_W);
      // ledgerNormedFull, agent reward, PPC, shaper (as k_step_duo's finish)
      double ar[M], portA[M];
      // lobs (one-step launches): State is stored by the ledger role; the
      // portfolio fractions only where the PPC cosine needs them (the divisions
      // kept in their branch: the compiler would run them beside it)
      const bool need_pa = !lobs || p.shaper == MGN_SHAPER_PPC;
      double port0 = 0.;
      if (need_pa) {
        double x = cashv - q.b;
        asm volatile("" : "+v"(x));
        port0 = x / curEq;
      }
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const double Lc = f.L[m], P = f.P[m];
        ar[m] = 0.;
        if (f.valid[m] && need_ar) {
          const int x = lx + m;
          double v = (((Lc * P) - sh.rPv[prv][x]) - (sh.rTu[prv][x] * sh.rTp[prv][x] + sh.rTc[prv][x])) / prevEq;
          v += 1;
          v = (v < .35) ? .35 : v;
          ar[m] = log_ratio(v);
        }
        portA[m] = 0.;
        if (need_pa) {
          double x = Lc * P;
          asm volatile("" : "+v"(x));
          portA[m] = x / curEq;
        }
      }
      double cos_term = 0.;
      if (p.shaper == MGN_SHAPER_PPC) {
        double pp[M], pq[M];
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const double qv = f.valid[m] ? s_tgt[1 + f.asset[m]] : 0.;
          const double pv = f.valid[m] ? portA[m] : 0.;
          pp[m] = pv * pv;
          pq[m] = pv * qv;
        }
        const double np_ = sqrt(port0 * port0 + canon<M, S, ONE>(pp));
        const double dot = port0 * s_tgt[0] + canon<M, S, ONE>(pq);
        cos_term = p.cos_temp * (dot / (np_ * g.cos_qn));
      }
      double shaped_s = 0., rin_s = 0., shaped_v = 0.;
      int pops = 1;
      MGN_ST(Tf1 = __builtin_amdgcn_s_memtime();)
      if (NST) {
        // NStepBuffer.add + pop_nstep_sarsd (nstep_buffer.py:315-356, driven as
        // replay_buffer.py:68-80) for the env's scalar column: append, pop once
        // when full, every entry on done; the row of step k (n entries, zero
        // after the pops) is stored here
        rin_s = (p.reward_mode == MGN_REWARD_AGENT_SUM) ? canon<M, S, ONE>(ar) : reward;
        const int n = p.nstep;
        double* ring = s_nst + (size_t)el * NPADS * nst_pad(n, S);  // ring, then the pop's summands
        double* scr = ring + nst_pad(n, S);
        const double v = (p.shaper == MGN_SHAPER_PPC) ? rin_s + cos_term : rin_s;
        const int L1 = nlen + 1;
        pops = done ? L1 : (L1 >= n ? 1 : 0);
        MGN_G double* row = (om & O_SHP) ? ov.shaped + kidx(k, sN, (size_t)env) * (size_t)n : nullptr;
        // append v; then the pops (one when the buffer is full, every entry
        // on done), each by all the env's lanes: summand kk on lane kk mod S
        // (nstep_column's operands) into LDS, slots [len, R S) +0.0 (the
        // ordered sum is unchanged: acc starts at +0.0 and is never -0.0),
        // then every lane sums them in kk order (S per chunk, the next
        // chunk's reads issued before this chunk's adds); the shaper state
        // steps between pops as nstep_column's does
        int tail = nhead + nlen;
        tail -= (tail >= n) ? n : 0;
        int len = L1, head = nhead;
        if constexpr (NRUN) {
          // the running-sum pop (nrun_pre / nrun_fin): every lane of the env
          // keeps the sums, appends the entry and pops -- the same values on
          // every lane, the first stores
          // (sortino_shaperB: the entry's root, kept beside the ring)
          const bool SB = SBR && p.shaper == MGN_SHAPER_SORTINO_B;
          double* rts = ring + nst_pad(n, S);
          const double vrt = (SB && v < 0.) ? root_e(-v, p.sexp) : 0.;
          ring[tail] = v;  // (every lane writes it: each lane's own reads below see it)
          if (SB) {
            rts[tail] = vrt;
            nrun_add_sb(nrs, v, vrt, nst_w, nst_w2);
          } else {
            nrun_add(nrs, v, nst_w);
          }
          // sortino_shaperB with an entry below -1 in the buffer (the
          // per-term clip can bind): the exact pop, naive_n's order
          // (sortinoB_term over the entries in order -- naive_n's sum; one entry:
          // naive1's, the same operations with gamma^0 = 1 -- inline: a call
          // would spill the caller's registers)
          const auto sb_exact = [&]() {
            double acc = 0.0;
            for (int kk = 0, idx = head; kk < len; ++kk, idx = (idx + 1 == n) ? 0 : idx + 1)
              acc += sortinoB_term(ring[idx], s_disc[kk], p.sexp);
            return clip1(acc);
          };
          // one pop: the shaper state steps (update_parameters, exact), the
          // oldest entry leaves the sums
          const auto pop_done = [&](int pj, double res, double r0, double rt0) {
            if (p.shaper == MGN_SHAPER_DSR || p.shaper == MGN_SHAPER_DDR) {
              g.shA += p.eta * (r0 - g.shA);
              if (p.shaper == MGN_SHAPER_DSR) {
                g.shB += p.eta * (r0 * r0 - g.shB);
              } else {
                double m = r0 < 0. ? r0 : 0.;
                if (r0 != r0) m = r0;
                g.shB += p.eta * (m * m - g.shB);
              }
            }
            if (row && ls == 0) ost(row + pj, res);
            head = (head + 1 == n) ? 0 : head + 1;
            len -= 1;
            if (len == 0) {  // a flushed buffer: the sums are exactly zero again
              nrun_zero(nrs);
              nsl = 0;
            } else {
              if (SB) nrun_slide_sb(nrs, r0, rt0, p.nst_rg, p.nst_rg2);
              else nrun_slide(nrs, r0, p.nst_rg);
              nsl += (r0 - r0 == 0.) ? 1 : n;  // a non-finite entry left: re-form at the next step
            }
          };
          // (the first pop taken out of the loop measured 2.73-2.79 against
          // 2.60 us/step, profiles/r06h_ab.txt)
          for (int pj = 0; pj < pops; ++pj) {
            double res;
            if (SB && nrs.prr > 0.) res = sb_exact();
            else if (pj == 0) res = SB ? nrun_fin_sb(npre, v, vrt, nst_w, nst_w2) : nrun_fin(p.shaper, npre, v, nst_w);
            else res = nrun_pop(p.shaper, nrs, len, g.shA, g.shB);  // a done flush's further pops
            if (pj == 0) pop_done(0, res, nlen == 0 ? v : nst_r0, nlen == 0 ? vrt : nst_rt0);
            else pop_done(pj, res, ring[head], rts[head]);
          }
        } else {
        if (ls == 0) ring[tail] = v;
        for (int pj = 0; pj < pops; ++pj) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          if (p.shaper == MGN_SHAPER_SHARPE || p.shaper == MGN_SHAPER_SORTINO_A ||
              (p.shaper == MGN_SHAPER_SORTINO_B && len == 1)) {
            // the naive shapers (sharpe_shaper, sortino_shaperA / B,
            // nstep_buffer.py:207-312) over the ring by the env's first lane,
            // nstep_column's evaluation: the single-entry heuristic or the
            // discounted sums in entry order (sortino_shaperB's one sum, over
            // more than one entry, takes the summand path below)
            if (ls == 0) {
              const double res = (len == 1) ? naive1(p.shaper, ring[head], p.sexp)
                                            : naive_n(p.shaper, ring, n, 1, 0, head, len, s_disc, p.sexp);
              if (row) ost(row + pj, res);
            }
            head = (head + 1 == n) ? 0 : head + 1;
            len -= 1;
            continue;
          }
          const PopPre c = pop_pre(p.shaper, g.shA, g.shB);
          double acc = 0.0;
          nst_summands(ring, scr, head, len, g.shA, g.shB, c);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          // the ordered sum only feeds the popped value the env's first lane
          // stores: only that lane reads the summands back
          if (ls == 0) acc = nst_sum(scr, len);
          double res = acc;
          if (p.shaper == MGN_SHAPER_SORTINO_B) res = clip1(acc);  // (naive_n, len > 1)
          if (p.shaper == MGN_SHAPER_DSR || p.shaper == MGN_SHAPER_DDR) {
            res = clip1(acc / len);
            const double r0 = ring[head];
            g.shA += p.eta * (r0 - g.shA);
            if (p.shaper == MGN_SHAPER_DSR) {
              g.shB += p.eta * (r0 * r0 - g.shB);
            } else {
              double m = r0 < 0. ? r0 : 0.;
              if (r0 != r0) m = r0;
              g.shB += p.eta * (m * m - g.shB);
            }
          }
          if (row && ls == 0) ost(row + pj, res);
          head = (head + 1 == n) ? 0 : head + 1;
          len -= 1;
        }
        }
        if (!kAblNstRow && row)
          for (int jj = pops + ls; jj < n; jj += S) ost(row + jj, 0.);
        nhead += pops;
        while (nhead >= n) nhead -= n;
        nlen = L1 - pops;
      } else if (D == 1) {
        rin_s = (p.reward_mode == MGN_REWARD_AGENT_SUM) ? canon<M, S, ONE>(ar) : reward;
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
        shaped_v = f.valid[0] ? shape(p.shaper, ar[0], g.shA, g.shB, p.eta, cos_term, p.sexp) : 0.;  // M = 1
      }
      if (j == 1) MGN_IT(57, 2 * TRIO_W);
      MGN_ST(Tf2 = __builtin_amdgcn_s_memtime();)
      // outputs of step k (the speculative runs never reach F)
#pragma unroll
      for (int m = 0; m < M; ++m) {
        if (kAblNoStoreAsset) break;
        if (f.valid[m]) {
          const size_t i = kidx(k, sNA, bA) + m;
          if (!RP && !lobs && (om & O_OPR)) ost(ov.obs_price + (kidx(k, sNF, bP) + m), f.P[m]);
          if (!lobs && (om & O_OPT)) ost(ov.obs_port + (kidx(k, sNA1, bO) + 1 + f.asset[m]), portA[m]);
          if (D != 1) {
            if (om & O_AREW) ost(ov.agent_reward + i, ar[m]);
            if (om & O_SHP) ost(ov.shaped + i, shaped_v);
          }
        }
      }
      if (!kAblNoStoreAsset && RP && live && (om & O_OPR))
        put_price(ov.obs_price + kidx(k, sNF, (size_t)env * p.F), f.P, false, prv);
      if (!kAblNoStoreEnv && ls == 0) {
        const size_t ie = kidx(k, sN, (size_t)env);
        if (!lobs && (om & O_OPT)) ost(ov.obs_port + kidx(k, sNA1, bO), port0);
        if (om & O_DONE) ost(ov.done + ie, (uint8_t)(done ? 1 : 0));
        if (om & O_MC) {
          // TR_MCALL: orders ran (in_kind != NONE); the check on the sums after them
          const Sums qa{sh.rLpA[prv][el], q.ml, q.sh, q.b};
          const bool mcall = (flags & TR_MCALL) && margin_call(qa, cashv, p.mainM);
          ost(ov.margin_call + ie, (uint8_t)(mcall ? 1 : 0));
        }
        if (om & O_DEND) ost(ov.data_end + ie, (uint8_t)(RP ? sh.dend[prv][el] : 0u));
        if (om & O_REW) ost(ov.reward + ie, reward);
        if (om & O_NSH) ost(ov.n_shaped + ie, (uint8_t)pops);
        if (om & O_TS) ost(ov.timestamp + ie, (uint64_t)sh.ts[prv][el]);
        if (D == 1) {
          if (om & O_AREW) ost(ov.agent_reward + ie, rin_s);
          if (!NST && (om & O_SHP)) ost(ov.shaped + ie, shaped_s);
        }
      }
      if (WIN) {
        push_row(f.P, portA, port0, (uint64_t)sh.ts[prv][el], k, prv);
        if (done && p.auto_reset) {  // a reset empties the window before its refill ticks
          rlen = 0;
          rhead = p.W - 1;
        }
      }
      // episode statistics
      ep_ret += reward;
      ep_len += 1;
      if (done) {
        if (ls == 0) {
          MGN_G double* st = gs.epstats + (size_t)env * 4;
          st[0] = ep_ret;
          st[1] = ep_len;
          st[2] = curEq;
          n_done = n_done + 1;
          st[3] = n_done;
        }
        ep_ret = 0;
        ep_len = 0;
        if (p.auto_reset) {
          rst_out = 1;
          tail_rst = TAIL && K == 1;
        }
      }
    }
    if (WIN && live && (flags & TR_REFILL)) {
      // a refill tick's row: the fresh Broker's portfolio on the tick's prices
      // (the sums ring_push / k_step_duo's refill record evaluate)
      double Pf[M], Lf[M], tlp[M], pa[M];
#pragma unroll
      for (int m = 0; m < M; ++m) {
        Pf[m] = sh.price[prv][lx + m];
        Lf[m] = sh.rL[prv][lx + m];
        tlp[m] = Lf[m] * Pf[m];
      }
      const double cashf = sh.rCash[prv][el], bf = sh.rB[prv][el];
      const double eq = (cashf + canon<M, S, ONE>(tlp)) - bf;
#pragma unroll
      for (int m = 0; m < M; ++m) pa[m] = (Lf[m] * Pf[m]) / eq;
      push_row(Pf, pa, (cashf - bf) / eq, (uint64_t)sh.ts[prv][el], klast, prv);
    }
    if constexpr (TAIL_EXACT) {
      // one-step launches: the last iteration -- the state write-back issued
      // before its barrier (it no longer changes)
      if (K == 1 && j == 1 && live) {
        f_store();
        fstored = true;
      }
    }
    if (ls == 0) sh.reset[cur][el] = rst_out;
    // the reset tick runs next iteration -- a tail reset's in this one, by the
    // idle generator role (adopted after the loop)
    if (rst_out && !tail_rst) sh.more[j % 3] = 1;
    if (j == 1) MGN_IT(50, 2 * TRIO_W);
    MGN_T(T1);
    __syncthreads();
    MGN_T(T2);
    MGN_ST(acc0 += T1 - T0; acc1 += T2 - T1;
           if (Tf2) {  // the iterations that evaluated a step: before / in / after the reward's shaping
             facc[0] += Tf1 - T0;
             facc[1] += Tf2 - Tf1;
             facc[2] += T1 - Tf2;
           })
    if (trio_exit(j, K, sh.more[j % 3])) break;
  }
  MGN_ST(if (l == 0) {
    atomicAdd(&g_duo_stamps[16], acc0);
    atomicAdd(&g_duo_stamps[17], acc1);
    atomicAdd(&g_duo_stamps[9], facc[0]);
    atomicAdd(&g_duo_stamps[11], facc[1]);
    atomicAdd(&g_duo_stamps[12], facc[2]);
  })
  if constexpr (kAblEpi) return;
  if (!live) return;
  if constexpr (NST != 0) {
    const double* ring = s_nst + (size_t)el * NPADS * nst_pad(p.nstep, S);
    for (int i = ls; i < p.nstep; i += S) p.nring[(size_t)env * p.nstep + i] = ring[i];
    if (ls == 0) {
      p.nlen[env] = nlen;
      p.nhead[env] = nhead;
    }
  }
  if (!fstored) f_store();
  MGN_IT_DRAIN();
  MGN_IT(46, 2 * TRIO_W);
}

}  // namespace mgn
