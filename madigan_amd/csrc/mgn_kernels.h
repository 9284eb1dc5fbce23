// mgn_kernels.h -- HIP kernels of the batched market-simulation step (gfx950).
//
// Thread mapping: an environment is owned by a segment of S adjacent lanes of
// one wavefront; each lane holds M consecutive assets (S*M = APAD, the next
// power of two >= n_assets) in registers.  State is struct-of-arrays, env-major
// (N,A) row-major in HBM, so a wave-wide load of one field is one contiguous
// burst.  Portfolio-wide quantities (asset value, pnl, balance, borrowed
// margin) are reduced with the canonical pairwise tree: a register tree over
// the lane's M slots, then an xor butterfly across the S lanes -- the same tree
// the oracle evaluates, so ledger state is bit-identical.
//
// The Broker's per-asset loop is a true serial dependency (each order's risk
// check sees the cash/ledger left by the previous one, Broker.cpp:149-155):
// round i is executed by the lane owning asset i after a segment reduction,
// and the new cash is broadcast back to the segment.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/madigan_amd.h"
#include "mgn_diag.h"
#include "mgn_math.h"

namespace mgn {

constexpr int BLOCK = 256;

// wait for every outstanding vector-memory load / store of this wave, as a
// real S_WAITCNT (gfx9 simm16: vmcnt 0, expcnt 7, lgkmcnt 15) that the
// wait-count insertion pass sees: loads issued before it are complete after it
__device__ __forceinline__ void drain_vmem() { __builtin_amdgcn_s_waitcnt(0x0F70); }

struct KParams {
  int N, A, W, D;
  int F;       // State.price width (features): A for the generators
  int ring_log;  // window norm "log": the ring stores log(max(x, 1e-5)) (applied once at push)
  int replay;  // every asset from the replay tape (MGN_SRC_REPLAY)
  int64_t env_offset;
  uint64_t seed;
  double init_cash, reqM, mainM, slip_rel, slip_abs, tc_rel, tc_abs;
  int shaper, reward_mode, auto_reset, atoms;
  int reqm_one;  // required_margin == 1.0
  int ablate;  // diagnostic timing builds only (mgn_set_ablation); 0 in every real run
  double eta, cos_temp, unit_size;
  double sexp;  // sortino_shaperA/B exponent
  // state
  double *L, *mep, *Bm, *P, *sx, *oum, *dy;
  int32_t *tlen;
  uint8_t *tfl;
  double *cash;
  uint64_t *ts;
  uint64_t *dskip;  // (N) resets so far: the variates' draw index is ts + dskip
  double *sA, *sB;
  double *ep;       // (N,2)
  double *epstats;  // (N,4)
  const double *ext;
  double *ring;
  uint64_t *ring_ts;
  int32_t *rhead, *rlen;
  const mgn_asset_source *src;  // (A); the step kernels point it at an LDS copy
  const mgn_asset_source *src_g;  // (A) in global memory (the noinline multi-component paths)
  const double *target;         // (A+1)
  // NStepBuffer (n > 1): ring (N,n,D), fill count / oldest index (N), gamma^i (n)
  int nstep;
  int nst_run;    // MGN_NSTEP_POP_RUNNING granted (mgn_api.hip kparams): the three-role running-sum pop
  double nst_rg;  // 1 / gamma (nst_run)
  double nst_rg2;        // sortino_shaperB: 1 / gamma^(1/exp)
  const double *disc2;   // sortino_shaperB: (gamma^k)^(1/exp) (n), after disc in the arena
  double *nring;
  int32_t *nlen, *nhead;
  const double *disc;
  // replay tape (mgn_attach_replay): (rows, A) prices, (rows, F) features,
  // timestamps, dataEnd flags; per-env cursor = next tape row
  const double *rp_price;
  const double *rp_feat;
  const uint64_t *rp_ts;
  const uint8_t *rp_end;
  int64_t rp_rows, rp_stride;
  int64_t *rcur;
  double *aux;  // (N, A, MGN_AUX_WIDTH) multi-component source state
  // per-launch window history (mgn_rollout_hist; null otherwise): every ring
  // push of the launch is also appended to hist (N, hrows, F+A+1) / hist_ts
  // (N, hrows) from row W on (rows [W-len0, W) hold the window before the
  // launch); after step k (and its reset refill) hend[k*N+env] = rows so far,
  // hlen[k*N+env] = the window's fill
  double *hist;
  uint64_t *hist_ts;
  int32_t *hend, *hlen;
  int hrows;
};

// ---------------------------------------------------------------------------
// reductions
template <int M>
__device__ __forceinline__ double tree(const double (&v)[M]) {
  if constexpr (M == 1) {
    return v[0];
  } else {
    double t[M / 2];
#pragma unroll
    for (int i = 0; i < M / 2; ++i) t[i] = v[2 * i] + v[2 * i + 1];
    return tree<M / 2>(t);
  }
}

// DPP lane moves (VALU latency, no LDS crossbar).  Controls (gfx9 / gfx950):
// quad_perm = p0 | p1<<2 | p2<<4 | p3<<6, row_mirror 0x140, row_half_mirror
// 0x141, row_newbcast:n 0x150+n (broadcast lane n of each 16-lane row).
// Every control used here reads an in-range lane, so bound_ctrl is set and no
// "old" value has to be materialized; row_newbcast moves 64 bits in one
// v_mov_b64_dpp.
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
  return __builtin_amdgcn_update_dpp(v, v, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  return __builtin_amdgcn_update_dpp(v, v, CTRL, 0xF, 0xF, true);
}

// Segment all-reduce over S aligned lanes.  Every stage pairs each lane with a
// lane of the sibling block, so every lane ends with the pairwise tree
// ((v0+v1)+(v2+v3))+((v4+v5)+(v6+v7))... -- the canonical order.
template <int S>
__device__ __forceinline__ double seg_sum(double v) {
  if constexpr (S >= 2) v = v + dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  if constexpr (S >= 4) v = v + dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  if constexpr (S >= 8) v = v + dpp_f64<0x141>(v);  // row_half_mirror
  if constexpr (S >= 16) v = v + dpp_f64<0x140>(v); // row_mirror
  if constexpr (S >= 32) v = v + __shfl_xor(v, 16, 64);
  if constexpr (S >= 64) v = v + __shfl_xor(v, 32, 64);
  return v;
}

template <int S>
__device__ __forceinline__ int seg_or(int v) {
  if constexpr (S >= 2) v = v | dpp_i32<0xB1>(v);
  if constexpr (S >= 4) v = v | dpp_i32<0x4E>(v);
  if constexpr (S >= 8) v = v | dpp_i32<0x141>(v);
  if constexpr (S >= 16) v = v | dpp_i32<0x140>(v);
  if constexpr (S >= 32) v = v | __shfl_xor(v, 16, 64);
  if constexpr (S >= 64) v = v | __shfl_xor(v, 32, 64);
  return v;
}

// Broadcast lane J of every S-lane segment to the segment (J compile-time).
template <int S, int J>
__device__ __forceinline__ double seg_bcast(double v) {
  if constexpr (S == 1) {
    return v;
  } else if constexpr (S == 2) {
    return dpp_f64<J | (J << 2) | ((2 + J) << 4) | ((2 + J) << 6)>(v);
  } else if constexpr (S == 4) {
    return dpp_f64<J * 0x55>(v);
  } else if constexpr (S == 8) {
    const double a = dpp_f64<0x150 + J>(v);
    const double b = dpp_f64<0x150 + 8 + J>(v);
    return (__lane_id() & 8) ? b : a;
  } else if constexpr (S == 16) {
    return dpp_f64<0x150 + J>(v);
  } else {
    return __shfl(v, (int)(__lane_id() & ~(S - 1)) + J, 64);
  }
}

// ONE: a one-asset env on an S = 2 lane segment (the pipelined kernels'
// narrowest layout): its canonical sum is the one leaf itself -- lane 0's --
// not leaf + (+0.0), which differs from it in the sign of a -0.0 leaf
template <int M, int S, bool ONE = false>
__device__ __forceinline__ double canon(const double (&v)[M]) {
  if constexpr (ONE) return seg_bcast<S, 0>(tree<M>(v));
  return seg_sum<S>(tree<M>(v));
}

struct Sums {
  double lp, ml, sh, b;
};

// Portfolio.cpp:180-209 -- the four sums every valuation is built from
template <int M, int S, bool ONE = false>
__device__ __forceinline__ Sums port_sums(const double (&L)[M], const double (&mep)[M],
                                          const double (&Bm)[M], const double (&P)[M]) {
  double tlp[M], tml[M], tsh[M], tb[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    tlp[m] = L[m] * P[m];
    tml[m] = mep[m] * L[m];
    const double mask = (L[m] < 0.) ? 1.0 : 0.0;
    tsh[m] = L[m] * (mep[m] * mask);
    tb[m] = Bm[m];
  }
  Sums s;
  s.lp = canon<M, S, ONE>(tlp);
  s.ml = canon<M, S, ONE>(tml);
  s.sh = canon<M, S, ONE>(tsh);
  s.b = canon<M, S, ONE>(tb);
  return s;
}

// Portfolio::checkRisk() == margin_call, Portfolio.cpp:243-252
__device__ __forceinline__ bool margin_call(const Sums& s, double cash, double mainM) {
  const double pnl = s.lp - s.ml;
  const double equity = (cash + s.lp) - s.b;
  const double balance = cash + s.sh;
  const double mr = mainM * pnl;
  return (equity <= -mr) || ((balance + pnl) <= -mr);
}

// ---------------------------------------------------------------------------
// per-lane register state
template <int M>
struct Lane {
  double L[M], mep[M], Bm[M], P[M], sx[M], oum[M], dy[M];
  int32_t tlen[M];
  uint8_t tfl[M];  // bit0 trending, bit1 dir<0
  int kind[M];
  int asset[M];
  bool valid[M];
  int64_t rcur;  // replay: next tape row (same in every lane of the segment)
  int64_t row;   // replay: tape row of the current State
  // replay prefetch: row rcur's prices (and this lane's feature column fcol,
  // when every feature has a lane) are loaded one tick ahead, so a tick's
  // tape reads leave the step's dependency chain
  double pfP[M], pfF, curF;
  int fcol = -1;       // feature column of this lane (-1: features read per row)
  bool pf_ok = false;  // pfP / pfF hold row rcur
  // variates (mgn_math.h, v3): the env's resets so far (draw index d =
  // timestamp + dskip), and per slot the cached odd half of the last pair
  uint64_t dskip = 0;
  double zc[M] = {};
  uint64_t ztag[M] = {};
};

// ---------------------------------------------------------------------------
// multi-component sources (views.aux; restated identically by the oracle)

// WaveTableOsc<double> as setSineOsc fills it (WaveTableOsc.h:104-174): every
// table holds len samples sin(i*2*pi/len) with sample len = sample 0; the
// interpolated read (getOutput :84-95) after updatePhase (:31).  Samples are
// evaluated where read, with the statement the table was built from.
__device__ __forceinline__ double wt_sample(int i, int len) {
  if (i == len) i = 0;
  return 1.0 * det_sin((double)i * 2. * 3.14159265358979323846 / len);
}
__device__ __forceinline__ double wt_process(double& phasor, double incr, int len) {
  phasor += incr;
  if (phasor >= 1.) phasor -= 1.;
  const double temp = phasor * len;
  const int ip = (int)temp;
  const double frac = temp - ip;
  const double s0 = wt_sample(ip, len), s1 = wt_sample(ip + 1, len);
  return s0 + (s1 - s0) * frac;
}
// std::max(lo, std::min(hi, v))
__device__ __forceinline__ double clamp_range(double lo, double hi, double v) {
  const double m = (v < hi) ? v : hi;
  return (lo < m) ? m : lo;
}
// SineDynamic(Trend)::updateParams (DataSource.cpp:802-813, :1002-1015)
__device__ __noinline__ void sd_update(const double* q, double* ax, uint32_t bits) {
  const int C = (int)q[0];
  for (int c = 0; c < C; ++c) {
    const double* r = q + 3 + C + 9 * c;
    double* a = ax + 4 * c;
    a[2] = clamp_range(r[3], r[4], a[2] + (((bits >> (3 * c)) & 1) ? r[5] : -r[5]));
    a[3] = clamp_range(r[6], r[7], a[3] + (((bits >> (3 * c + 1)) & 1) ? r[8] : -r[8]));
    a[1] = clamp_range(r[0], r[1], a[1] + (((bits >> (3 * c + 2)) & 1) ? r[2] : -r[2]));
  }
}
// freq, mu, amp ~ U[lo, hi] per component (initParams :777-782, reset :794-800)
__device__ __noinline__ void sd_sample(const double* q, double* ax, uint64_t seed, uint64_t genv,
                                       uint32_t asset, uint64_t tick) {
  const int C = (int)q[0];
  for (int c = 0; c < C; ++c) {
    const double* r = q + 3 + C + 9 * c;
    const u4 x = block(seed, genv, asset, 16u + (uint32_t)c, tick);
    ax[4 * c + 1] = (r[1] - r[0]) * ((double)x.x * TWO_M32) + r[0];
    ax[4 * c + 2] = (r[4] - r[3]) * ((double)x.y * TWO_M32) + r[3];
    ax[4 * c + 3] = (r[7] - r[6]) * ((double)x.z * TWO_M32) + r[6];
  }
}
// SineAdder::getData (DataSource.cpp:663-673)
__device__ __noinline__ double sineadder_tick(const double* q, double* ax, uint64_t seed,
                                              uint64_t genv, uint32_t asset, uint64_t tick) {
  const int C = (int)q[0];
  const double PI2 = 3.141592653589793238463 * 2;
  double sum = 0.;
  for (int c = 0; c < C; ++c) {
    double nz = 0.0;  // component c's noise: the block of counter slot c
    if (q[2] != 0.0) nz = normal_of(block(seed, genv, asset, (uint32_t)c, tick)) * q[2] + 0.0;
    sum += (nz + q[3 + C + c]) + q[3 + 2 * C + c] * det_sin(PI2 * ax[c] * q[3 + c]);
    ax[c] += q[1];
  }
  return sum;
}
// SineDynamic::getData (DataSource.cpp:829-841) / SineDynamicTrend::getData (:1017-1047)
__device__ __noinline__ double sinedyn_tick(const double* q, double* ax, bool trend, uint64_t seed,
                                            uint64_t genv, uint32_t asset, uint64_t tick) {
  const int C = (int)q[0];
  const u4 x0 = block(seed, genv, asset, 0, tick);
  sd_update(q, ax, x0.w);
  double tc = ax[16];
  double sum = 0.;
  for (int c = 0; c < C; ++c) {
    double* a = ax + 4 * c;
    const double out = wt_process(a[0], a[1] / q[1], (int)q[3 + c]);  // setFreq(freq / sampleRate)
    if (trend) sum += tc * (a[2] + a[3] * out);
    else sum += a[2] + a[3] * out;
  }
  double nz = 0.0;
  if (q[2] != 0.0) nz = normal_of(x0) * q[2] + 0.0;
  if (!trend) return sum + nz;
  const double* tq = q + 3 + 10 * C;  // T, then per trend {minLen, maxLen, incr, prob}
  const int T = (int)tq[0];
  u4 x1 = {0u, 0u, 0u, 0u};
  bool have1 = false;
  for (int t = 0; t < T; ++t) {
    const double* r = tq + 1 + 4 * t;
    double* st = ax + 17 + 3 * t;  // trending, direction, length
    if (st[0] != 0.) {
      tc += (tc * r[2]) * st[1];
      st[2] -= 1.;
      if (st[2] == 0.) st[0] = 0.;
    } else {
      if (!have1) {
        x1 = block(seed, genv, asset, 1, tick);
        have1 = true;
      }
      const double u = (double)(t == 0 ? x1.x : x1.y) * TWO_M32;
      if (u < r[3]) {
        st[0] = 1.;
        st[1] = ((x0.w >> (12 + t)) & 1) ? -1. : 1.;
        const int lo = (int)r[0], hi = (int)r[1];
        const int len = lo + (int)(((double)(t == 0 ? x1.z : x1.w) * TWO_M32) * (double)(hi - lo + 1));
        st[2] = (double)(len > hi ? hi : len);
      }
    }
    if (tc <= .1) st[1] = 1.;
    tc = (0.01 < tc) ? tc : 0.01;
  }
  ax[16] = tc;
  return (sum + tc) + tc * nz;
}

// DataSource::getData for the lane's slots (DataSource.cpp:535-543, 1173-1180,
// 1457-1493; Composite concatenation :439-451) ; tick = timestamp before ++.
// RP: the kernel may serve a replay tape (k_step); AUX: multi-component kinds
// (views.aux).  The two-role kernel compiles neither (their calls would cost
// the hot generator registers) and is not selected for such handles.  GK >= 0:
// every asset of the handle is of kind GK (the launcher checks), so the
// per-lane kind dispatch folds away at compile time.
// qreg: the lane's parameters in registers (the three-role kernel with a
// compile-time kind, M = 1), else read from p.src
// INL: the Sine kinds' sin inlined (the pipelined kernels), else called
// SEQ: the slots ticked one after another (a scheduling fence between them:
// the three-role kernel's 168-register budget at two slots per lane)
template <int M, bool RP = true, bool AUX = true, int GK = -1, bool INL = false, bool SEQ = false>
__device__ __forceinline__ void gen_tick(Lane<M>& s, const KParams& p, int env, uint64_t tick,
                                         const double* qreg = nullptr) {
  if (RP && p.replay) {
    // HDFSourceSingle::getData (DataSource.cpp:391-398) on the tape: the
    // row iterCache / loadData would serve, then advance (wrap = the
    // reference's rewind to boundsIdx_.first, :368-371, :397-399)
    const int64_t row = s.rcur;
    const bool fown = s.fcol >= 0 && s.fcol < p.F;
#pragma unroll
    for (int m = 0; m < M; ++m)
      if (s.valid[m]) s.P[m] = s.pf_ok ? s.pfP[m] : p.rp_price[(size_t)row * p.A + s.asset[m]];
    if (fown) s.curF = s.pf_ok ? s.pfF : p.rp_feat[(size_t)row * p.F + s.fcol];
    s.row = row;
    s.rcur = (row + 1 == p.rp_rows) ? 0 : row + 1;
    // the next tick reads row rcur (a source reset keeps the cursor)
#pragma unroll
    for (int m = 0; m < M; ++m)
      if (s.valid[m]) s.pfP[m] = p.rp_price[(size_t)s.rcur * p.A + s.asset[m]];
    if (fown) s.pfF = p.rp_feat[(size_t)s.rcur * p.F + s.fcol];
    s.pf_ok = true;
    return;
  }
  const uint64_t genv = (uint64_t)(p.env_offset + env);
  tick += s.dskip;  // the draw index (mgn_math.h, v3)
#pragma unroll
  for (int m = 0; m < M; ++m) {
    if constexpr (SEQ) {
      if (m > 0) __builtin_amdgcn_sched_barrier(0);
    }
    if (!s.valid[m]) continue;
    const int a = s.asset[m];
    const double* q = qreg ? qreg : p.src[a].p;
    const int kind = GK >= 0 ? GK : s.kind[m];
    // the slot-0 variates, drawn once for every kind that reads them: a
    // Composite source's lanes (Synth / OU / TrendOU in one wave) then run one
    // Philox + Box-Muller instead of one per kind branch (same bits: the draw
    // is a pure function of its counter)
    const bool sine_fam = kind == MGN_SRC_SINE || kind == MGN_SRC_SAWTOOTH || kind == MGN_SRC_TRIANGLE;
    const bool need0 = kind == MGN_SRC_TRENDOU || kind == MGN_SRC_OU || kind == MGN_SRC_SIMPLETREND ||
                       kind == MGN_SRC_TRENDYOU || kind == MGN_SRC_GAUSSIAN || kind == MGN_SRC_OUPAIR ||
                       (sine_fam && q[5] != 0.0);
    Draw d = {0.0, 0.0, 0u};
    if (need0) d = draw_d(p.seed, genv, (uint32_t)a, tick, s.zc[m], s.ztag[m]);
    if (kind == MGN_SRC_TRENDOU) {
      double y = s.P[m];
      if (s.tfl[m] & 1) {
        const double n = d.z * q[8] + 0.0;
        const double dir = (s.tfl[m] & 2) ? -1.0 : 1.0;
        y += y * (s.dy[m] * dir + n);
        s.tlen[m] -= 1;
        if (s.tlen[m] == 0) {
          s.tfl[m] &= ~1;
          s.oum[m] = y;
        }
        y = (0.01 < y) ? y : 0.01;
        if (y <= .1) s.tfl[m] &= ~2;
      } else {
        const double n = d.z * q[7] + 0.0;
        const double ou_noise = y * n;
        const double ou_rev = q[6] * (s.oum[m] - y);
        y += ou_rev + ou_noise;
        if (d.ut < q[0]) {  // regime switch (DataSource.cpp:1484-1489)
          double u_len, u_dy;
          uniform2(p.seed, genv, (uint32_t)a, 1, tick, u_len, u_dy);
          const int32_t lo = (int32_t)q[1], hi = (int32_t)q[2];
          int32_t len = lo + (int32_t)(u_len * (double)(hi - lo + 1));
          if (len > hi) len = hi;
          s.tlen[m] = len;
          s.dy[m] = (q[4] - q[3]) * u_dy + q[3];
          s.tfl[m] = (uint8_t)(1 | (d.dbit ? 2 : 0));
        }
      }
      s.P[m] = y;
    } else if (kind == MGN_SRC_OU) {
      const double z = d.z * 1.0 + 0.0;
      double x = s.P[m];
      x += (q[1] * (q[0] - x)) + q[0] * q[2] * z;
      s.P[m] = x;
    } else if (sine_fam) {
      // Synth / SawTooth / Triangle::getData (DataSource.cpp:535-543, 557-577)
      double noise = 0.0;
      if (q[5] != 0.0) noise = d.z * q[5] + 0.0;
      const double PI2 = 3.141592653589793238463 * 2;
      double wave;
      if (kind == MGN_SRC_SINE) wave = q[2] * (INL ? det_sin_inl(PI2 * s.sx[m] * q[0]) : det_sin(PI2 * s.sx[m] * q[0]));
      else if (kind == MGN_SRC_SAWTOOTH) wave = q[2] * frac_part(s.sx[m] * q[0]);
      else wave = 4 * q[2] / PI2 * det_asin(det_sin(PI2 * s.sx[m] / q[0]));
      s.P[m] = noise + q[1] + wave;
      s.sx[m] += q[4];
    } else if (kind == MGN_SRC_SIMPLETREND) {
      // SimpleTrend::getData (DataSource.cpp:1322-1347)
      double y = s.P[m];
      if (s.tfl[m] & 1) {
        const double dir = (s.tfl[m] & 2) ? -1.0 : 1.0;
        y += y * s.dy[m] * dir;
        s.tlen[m] -= 1;
        if (s.tlen[m] == 0) s.tfl[m] &= ~1;
      } else if (d.ut < q[0]) {
        double u_len, u_dy;
        uniform2(p.seed, genv, (uint32_t)a, 1, tick, u_len, u_dy);
        const int32_t lo = (int32_t)q[1], hi = (int32_t)q[2];
        int32_t len = lo + (int32_t)(u_len * (double)(hi - lo + 1));
        s.tlen[m] = len > hi ? hi : len;
        s.dy[m] = (q[6] - q[5]) * u_dy + q[5];
        s.tfl[m] = (uint8_t)(1 | (d.dbit ? 2 : 0));
      }
      if (y <= .1) s.tfl[m] &= ~2;
      y += y * (d.z * q[3] + 0.0);
      s.P[m] = (0.01 < y) ? y : 0.01;
    } else if (kind == MGN_SRC_TRENDYOU) {
      // TrendyOU::getData (DataSource.cpp:1608-1640): sx = ouComponent, oum = trendComponent
      const double ou_noise = s.oum[m] * (d.z * q[7] + 0.0);
      const double ou_rev = q[6] * (-s.sx[m]);
      s.sx[m] += ou_rev + ou_noise;
      const int32_t lo = (int32_t)q[1], hi = (int32_t)q[2];
      if (s.tfl[m] & 1) {
        double tc = s.oum[m];
        const double dir = (s.tfl[m] & 2) ? -1.0 : 1.0;
        tc += tc * (s.dy[m] * dir);
        tc = (0.1 < tc) ? tc : 0.1;
        if (tc <= .1) {  // floored: restart an up-trend of a fresh length
          double u_len, u_dy;
          uniform2(p.seed, genv, (uint32_t)a, 1, tick, u_len, u_dy);
          const int32_t len = lo + (int32_t)(u_len * (double)(hi - lo + 1));
          s.tlen[m] = len > hi ? hi : len;
          s.tfl[m] = 1;
        }
        s.oum[m] = tc;
        s.tlen[m] -= 1;
        if (s.tlen[m] == 0) s.tfl[m] &= ~1;
      } else if (d.ut < q[0]) {
        double u_len, u_dy;
        uniform2(p.seed, genv, (uint32_t)a, 1, tick, u_len, u_dy);
        const int32_t len = lo + (int32_t)(u_len * (double)(hi - lo + 1));
        s.tlen[m] = len > hi ? hi : len;
        s.dy[m] = (q[4] - q[3]) * u_dy + q[3];
        s.tfl[m] = (uint8_t)(1 | (d.dbit ? 2 : 0));
      }
      s.P[m] = s.sx[m] + s.oum[m];
    } else if (kind == MGN_SRC_GAUSSIAN) {
      // Gaussian::getData (DataSource.cpp:1108-1114): normal(mean, var)
      s.P[m] = d.z * q[1] + q[0];
    } else if (kind == MGN_SRC_OUPAIR) {
      // OUPair::getData (DataSource.cpp:1236-1244): the pair's shared mean random
      // walk is recomputed identically by the lanes of both assets (its variate
      // is keyed by the pair's first asset, counter slot 2)
      const uint32_t a0 = (uint32_t)(a - (q[3] != 0.0 ? 1 : 0));
      double mean = s.oum[m];
      mean += mean * (normal_of(block(p.seed, genv, a0, 2, tick)) * q[2] + 0.0);
      const double z = d.z * q[1] + 0.0;
      double x = s.P[m];
      x += (q[0] * (mean - x)) + mean * z;
      s.P[m] = x;
      s.oum[m] = mean;
    } else if (AUX && kind == MGN_SRC_SINEADDER) {
      s.P[m] = sineadder_tick(p.src_g[a].p, p.aux + ((size_t)env * p.A + a) * MGN_AUX_WIDTH, p.seed, genv,
                              (uint32_t)a, tick);
    } else if (AUX && (kind == MGN_SRC_SINEDYNAMIC || kind == MGN_SRC_SINEDYNTREND)) {
      s.P[m] = sinedyn_tick(p.src_g[a].p, p.aux + ((size_t)env * p.A + a) * MGN_AUX_WIDTH,
                            kind == MGN_SRC_SINEDYNTREND, p.seed, genv, (uint32_t)a, tick);
    } else {
      s.P[m] = p.ext[(size_t)env * p.A + a];
      drain_vmem();  // in this branch: the kinds' merge point then needs no wait
    }
  }
}

// timestamp_ after a getData: the tape's timestamp for replay (HDFSourceSingle
// :396), else timestamp_ += 1
template <int M>
__device__ __forceinline__ uint64_t next_ts(const Lane<M>& s, const KParams& p, uint64_t ts) {
  return p.replay ? p.rp_ts[s.row] : ts + 1;
}

// State.price of the current tick for the lane's columns (features): the
// replay tape's feature row, else the generator prices (F = A)
__device__ __forceinline__ double log_norm(double x) { return log((x < 1e-5) ? 1e-5 : x); }

// lg: apply StackerDiscrete's log normaliser (preprocessor.py:79-81)
template <int M, int S>
__device__ __forceinline__ void put_feats(const Lane<M>& s, const KParams& p, int ls,
                                          double* __restrict__ dst, bool lg = false) {
  if (p.replay && s.fcol >= 0) {
    if (s.fcol < p.F) dst[s.fcol] = lg ? log_norm(s.curF) : s.curF;
  } else if (p.replay) {
    for (int f = ls; f < p.F; f += S) {
      const double v = p.rp_feat[(size_t)s.row * p.F + f];
      dst[f] = lg ? log_norm(v) : v;
    }
  } else {
#pragma unroll
    for (int m = 0; m < M; ++m)
      if (s.valid[m]) dst[s.asset[m]] = lg ? log_norm(s.P[m]) : s.P[m];
  }
}

// source reset (DataSource.h:466, :232; DataSource.cpp:1495-1502; the replay
// source carries on, DataSource.cpp:200-206)
template <int M, bool AUX = true, int GK = -1>
__device__ __forceinline__ void src_reset(Lane<M>& s, const KParams& p, int env, uint64_t tick,
                                          const double* qreg = nullptr) {
  // every Env::reset skips one draw index (mgn_math.h, v3): the reset's
  // getData draws at timestamp + resets
  s.dskip += 1;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    if (!s.valid[m]) continue;
    const double* q = qreg ? qreg : p.src[s.asset[m]].p;
    const int kind = GK >= 0 ? GK : s.kind[m];
    if (kind == MGN_SRC_TRENDOU) {
      s.tfl[m] &= ~1;
      s.P[m] = q[5];
      s.tlen[m] = 0;
      s.oum[m] = q[5];
    } else if (kind == MGN_SRC_SIMPLETREND) {  // DataSource.cpp:1349-1356
      s.P[m] = q[4];
      s.tfl[m] = 0;  // not trending, direction +1
      s.tlen[m] = 0;
    } else if (kind == MGN_SRC_TRENDYOU) {     // DataSource.cpp:1642-1653
      s.sx[m] = 0.;
      s.oum[m] = q[5];
      s.tfl[m] &= ~1;
      s.P[m] = q[5];
      s.tlen[m] = 0;
    } else if (kind == MGN_SRC_OUPAIR) {       // DataSource.cpp:1246-1250
      s.P[m] = 10.;
      s.oum[m] = 10.;
    } else if (AUX && (kind == MGN_SRC_SINEDYNAMIC || kind == MGN_SRC_SINEDYNTREND)) {  // :794-800, :994-1000
      sd_sample(p.src_g[s.asset[m]].p, p.aux + ((size_t)env * p.A + s.asset[m]) * MGN_AUX_WIDTH, p.seed,
                (uint64_t)(p.env_offset + env), (uint32_t)s.asset[m], tick + s.dskip);
    }
  }
}

// StackerDiscrete.stream_state of the current State (preprocessor.py:172-175)
// (with a launch history, the same row is appended at history row hcnt)
template <int M, int S>
__device__ __forceinline__ void ring_push(const Lane<M>& s, const KParams& p, int env, int ls,
                                          double cash, uint64_t ts, int32_t& head, int32_t& len,
                                          int hcnt = -1) {
  const Sums q = port_sums<M, S>(s.L, s.mep, s.Bm, s.P);
  const double eq = (cash + q.lp) - q.b;
  head = (head + 1 == p.W) ? 0 : head + 1;
  if (len < p.W) len += 1;
  const int R = p.F + p.A + 1;
  double* row = p.ring + ((size_t)env * p.W + head) * R;
  double* hrow = (hcnt >= 0) ? p.hist + ((size_t)env * p.hrows + hcnt) * R : nullptr;
  put_feats<M, S>(s, p, ls, row, p.ring_log != 0);
  if (hrow) put_feats<M, S>(s, p, ls, hrow, p.ring_log != 0);
#pragma unroll
  for (int m = 0; m < M; ++m) {
    if (!s.valid[m]) continue;
    const double v = (s.L[m] * s.P[m]) / eq;
    row[p.F + 1 + s.asset[m]] = v;
    if (hrow) hrow[p.F + 1 + s.asset[m]] = v;
  }
  if (ls == 0) {
    const double c = (cash - q.b) / eq;
    row[p.F] = c;
    p.ring_ts[(size_t)env * p.W + head] = ts;
    if (hrow) {
      hrow[p.F] = c;
      p.hist_ts[(size_t)env * p.hrows + hcnt] = ts;
    }
  }
}

// after a history row: count it and mark step k's window end and fill
__device__ __forceinline__ void hist_mark(const KParams& p, int env, int ls, int& hcnt, int len,
                                          int k) {
  hcnt += 1;
  if (ls == 0) {
    p.hend[(size_t)k * p.N + env] = hcnt;
    p.hlen[(size_t)k * p.N + env] = len;
  }
}

// Env::reset (+ agent preprocessor reset) for one env, in registers.
template <int M, int S>
__device__ __forceinline__ void env_reset(Lane<M>& s, const KParams& p, int env, int ls,
                                          double& cash, uint64_t& ts, int32_t& head, int32_t& len) {
  src_reset<M>(s, p, env, ts);
#pragma unroll
  for (int m = 0; m < M; ++m) {
    s.L[m] = 0.;
    s.mep[m] = 0.;
    s.Bm[m] = 0.;
  }
  cash = p.init_cash;
  gen_tick<M>(s, p, env, ts);
  ts = next_ts<M>(s, p, ts);
  if (p.W > 0) {
    len = 0;
    head = p.W - 1;
    ring_push<M, S>(s, p, env, ls, cash, ts, head, len);
    while (len < p.W) {
      gen_tick<M>(s, p, env, ts);
      ts = next_ts<M>(s, p, ts);
      ring_push<M, S>(s, p, env, ls, cash, ts, head, len);
    }
  }
}

template <int M>
__device__ __forceinline__ void load_lane(Lane<M>& s, const KParams& p, int env, int ls) {
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int a = ls * M + m;
    s.asset[m] = a;
    s.valid[m] = a < p.A;
    if (s.valid[m]) {
      const size_t i = (size_t)env * p.A + a;
      s.L[m] = p.L[i];
      s.mep[m] = p.mep[i];
      s.Bm[m] = p.Bm[i];
      s.P[m] = p.P[i];
      s.sx[m] = p.sx[i];
      s.oum[m] = p.oum[i];
      s.dy[m] = p.dy[i];
      s.tlen[m] = p.tlen[i];
      s.tfl[m] = p.tfl[i];
      s.kind[m] = p.src[a].kind;
    } else {
      s.L[m] = s.mep[m] = s.Bm[m] = s.P[m] = s.sx[m] = s.oum[m] = s.dy[m] = 0.;
      s.tlen[m] = 0;
      s.tfl[m] = 0;
      s.kind[m] = -1;
    }
  }
  s.rcur = p.replay ? p.rcur[env] : 0;
  s.row = 0;
  s.pf_ok = false;
  s.fcol = -1;
}

template <int M>
__device__ __forceinline__ void store_lane(const Lane<M>& s, const KParams& p, int env) {
#pragma unroll
  for (int m = 0; m < M; ++m) {
    if (!s.valid[m]) continue;
    const size_t i = (size_t)env * p.A + s.asset[m];
    p.L[i] = s.L[m];
    p.mep[i] = s.mep[m];
    p.Bm[i] = s.Bm[m];
    p.P[i] = s.P[m];
    p.sx[i] = s.sx[m];
    p.oum[i] = s.oum[m];
    p.dy[i] = s.dy[m];
    p.tlen[i] = s.tlen[m];
    p.tfl[i] = s.tfl[m];
  }
}


template <typename T>
__device__ __forceinline__ T in_vgpr(T x) {
  asm volatile("" : "+v"(x));
  return x;
}


// x / required_margin; x / 1.0 == x exactly in IEEE, so the common
// required_margin == 1 case skips the division with identical bits.
__device__ __forceinline__ double div_reqm(double x, const KParams& p) {
  double r;
  if (p.reqm_one) r = x;
  else r = x / p.reqM;
  return r;
}

// One Broker round (Broker.cpp:124-142): asset i = J*M + MM, decided by the
// owning lane J of every segment after a segment reduction of the portfolio
// sums; the owner's new cash is then broadcast to its segment.  Written as
// straight-line predicated code (every branch of Portfolio::checkRisk and
// Portfolio::handleTransaction is evaluated and the taken one selected), so the
// round has no divergent control flow; the selected values are exactly the
// ones the reference's branches produce.
template <int M, int S, int J, int MM>
__device__ __forceinline__ void broker_round(Lane<M>& s, const KParams& p, double& cash,
                                             const double (&uc)[M], double (&tp)[M],
                                             double (&tu)[M], double (&tc)[M], int (&rk)[M],
                                             int ls) {
  const bool act = (ls == J) && (uc[MM] != 0.);
  const Sums q = port_sums<M, S>(s.L, s.mep, s.Bm, s.P);
  const double pnl = q.lp - q.ml;
  const double balance = cash + q.sh;
  const double availM = div_reqm(balance + pnl, p);
  const double u = uc[MM];
  const double cur = s.L[MM];
  const double price = s.P[MM];
  // Portfolio::checkRisk(i, u), Portfolio.cpp:254-279
  const bool opp = signbit(u) != signbit(cur);
  const bool rev = u > -1 * cur;
  const double excess = u + cur;
  const bool insuff_opp = rev && ((availM <= fabs(price * excess)) || (balance <= 0.));
  const double equity = (cash + q.lp) - q.b;
  const double mr = p.mainM * pnl;
  const bool mc = (equity <= -mr) || ((balance + pnl) <= -mr);
  const bool insuff_same = (availM <= fabs(price * u)) || (balance <= 0.);
  const int risk = opp ? (insuff_opp ? MGN_INSUFF_MARGIN : MGN_GREEN)
                       : (mc ? MGN_MARGIN_CALL : (insuff_same ? MGN_INSUFF_MARGIN : MGN_GREEN));
  // Broker.cpp:128-135 and Portfolio::handleTransaction, Portfolio.cpp:284-323
  const double slippage = (price * p.slip_rel) + p.slip_abs;
  const double tprice = u < 0 ? (price - slippage) : (price + slippage);
  const double tcost = fabs(u * price) * p.tc_rel + p.tc_abs;
  const bool close = opp && (fabs(u) > fabs(cur));
  const double units = close ? u + cur : u;
  const double c1 = close ? cash + cur * tprice : cash;
  const double cu1 = close ? 0. : cur;
  const double me0 = s.mep[MM];
  const double me_avg = me0 + (tprice - me0) * (u / (u + cur));
  const double me1 = close ? tprice : (opp ? me0 : me_avg);
  const double amt = tprice * units;
  const double use = amt * p.reqM;
  const double brw = amt - use;
  const double bm0 = s.Bm[MM];
  const double bm1 = bm0 + brw;
  const double c2 = c1 - (use + tcost);
  const double cu2 = cu1 + units;
  const bool closed = fabs(cu2) < 0.000001;
  const double me2 = closed ? 0. : me1;
  const bool repay = closed && (bm1 > 0.);
  const double c3 = repay ? c2 - bm1 : c2;
  const double bm2 = repay ? 0. : bm1;
  const bool neg = bm2 < 0.;
  const double c4 = neg ? c3 - bm2 : c3;
  const double bm3 = neg ? 0. : bm2;
  const bool go = act && (risk == MGN_GREEN);
  rk[MM] = act ? risk : rk[MM];
  s.L[MM] = go ? cu2 : cur;
  s.mep[MM] = go ? me2 : me0;
  s.Bm[MM] = go ? bm3 : bm0;
  tp[MM] = go ? tprice : tp[MM];
  tu[MM] = go ? u : tu[MM];
  tc[MM] = go ? tcost : tc[MM];
  cash = seg_bcast<S, J>(go ? c4 : cash);
}

// Rounds in asset order i = 0..APAD-1 (Broker.cpp:149-155); padding slots
// i >= A carry units 0 and change nothing.
template <int M, int S, int I>
struct Rounds {
  static __device__ __forceinline__ void run(Lane<M>& s, const KParams& p, double& cash,
                                             const double (&uc)[M], double (&tp)[M],
                                             double (&tu)[M], double (&tc)[M], int (&rk)[M],
                                             int ls) {
    if constexpr (I < M * S) {
      broker_round<M, S, I / M, I % M>(s, p, cash, uc, tp, tu, tc, rk, ls);
      Rounds<M, S, I + 1>::run(s, p, cash, uc, tp, tu, tc, rk, ls);
    }
  }
};

// ---------------------------------------------------------------------------
// Broker rounds, exchange form (APAD <= 16).
//
// Everything in one round except the risk check and the cash update depends
// only on that round's own asset (its units, ledger, price): the transaction
// price, cost, new ledger / mean entry / borrowed, the cash increments and the
// four portfolio-sum leaves before and after the order.  Each lane computes
// those for its own slots in parallel and publishes them to LDS (OrderRec).
// The serial chain then runs redundantly in every lane of the segment, in
// registers: risk check against the current sums, select the leaf, and update
// the canonical pairwise tree along one leaf-to-root path (nodes whose leaves
// are all decided are final; nodes with none decided keep their pre-order
// value).  Every node is the same sum of the same two children as in the full
// tree, so the sums are bit-identical to recomputing the canonical tree after
// each order (and to the oracle).
struct alignas(16) OrderRec {
  double pre[4];   // leaves {L*P, mep*L, L*(mep*[L<0]), Bm} before the order
  double post[4];  // the same leaves if the order executes
  double aPX;      // |price*excess| (reversal) or |price*units| (same side)
  double X1;       // close ? L*tprice : -0.0   (cash += X1 is exact when not closing)
  double y;        // usedMargin + cost
  double Z;        // borrowed repaid / negative-borrow cleared, else +0.0
  uint32_t act, need_mc, need_insuff, pad;
};
// (XRounds' records; the speculative broker keeps its orders in registers.)
// The stride of an env's records is 4 (mod 8) dwords, so the segments of a
// wave start in distinct groups of four LDS banks
template <int APAD>
struct alignas(16) EnvRecs {
  static constexpr int kBaseDw = APAD * 28;
  static constexpr int kPadD = (((4 - kBaseDw) % 8 + 8) % 8) / 2;
  OrderRec r[APAD];
  double pad[kPadD > 0 ? kPadD : 4];
};

// heap-indexed canonical tree over APAD leaves: node K (1-based) spans
// leaves [lo(K), hi(K)); leaves are nodes APAD..2APAD-1
constexpr int ilog2(int x) { return x <= 1 ? 0 : 1 + ilog2(x / 2); }
template <int APAD, int K>
struct Node {
  static constexpr int depth = ilog2(K);
  static constexpr int span = APAD >> depth;
  static constexpr int lo = (K - (1 << depth)) * span;
  static constexpr int hi = lo + span;
};

// leaf L of the heap tree changed: recompute its ancestors bottom-up (each node
// the sum of its two children, the canonical order)
template <int APAD, int K>
__device__ __forceinline__ void update_up(double (&t)[2 * APAD]) {
  if constexpr (K >= 1) {
    t[K] = t[2 * K] + t[2 * K + 1];
    update_up<APAD, K / 2>(t);
  }
}

template <int APAD, int K>
__device__ __forceinline__ void build_pre(double (&pre)[2 * APAD]) {
  if constexpr (K >= 2) {
    pre[K] = pre[2 * K] + pre[2 * K + 1];
    build_pre<APAD, K - 1>(pre);
  }
}

using d2 = double __attribute__((ext_vector_type(2)));
using v4u = uint32_t __attribute__((ext_vector_type(4)));

// the per-round part of one OrderRec, as vector loads
struct RoundIn {
  d2 post01, post23, ax1, yz;
  v4u fl;
};
template <int APAD>
__device__ __forceinline__ RoundIn load_round(const EnvRecs<APAD>& er, int i) {
  const d2* rv = reinterpret_cast<const d2*>(&er.r[i]);
  RoundIn r;
  r.post01 = rv[2];
  r.post23 = rv[3];
  r.ax1 = rv[4];
  r.yz = rv[5];
  r.fl = *reinterpret_cast<const v4u*>(&er.r[i].act);
  return r;
}

// Portfolio::checkRisk(i, u) (Portfolio.cpp:254-279) + Broker cash update
// (Broker.cpp:128-135, Portfolio.cpp:284-323) for round I; RQ1: required
// margin == 1 (x / 1.0 == x, division skipped with identical bits).  The next
// round's record is loaded before this round computes (LDS latency hidden),
// and the logic is straight-line (no short-circuit branches).  t[q] is the
// canonical tree of sum q over the current leaves: leaves < I hold their
// decided values, leaves >= I their pre-order values, so t[q][1] is the sum
// the reference's accessor recomputes before order I.
template <int M, int S, bool RQ1, int I>
struct XRounds {
  static constexpr int APAD = M * S;
  static __device__ __forceinline__ void run(const EnvRecs<APAD>& er, const RoundIn& r,
                                             const KParams& p, double& cash,
                                             double (&t)[4][2 * APAD], bool (&go_own)[M],
                                             int (&rk)[M], int& any_mc, int ls) {
    if constexpr (I < APAD) {
      RoundIn nxt;
      if constexpr (I + 1 < APAD) nxt = load_round<APAD>(er, I + 1);
      const double post[4] = {r.post01.x, r.post01.y, r.post23.x, r.post23.y};
      const double pnl = t[0][1] - t[1][1];
      const double balance = cash + t[2][1];
      const double bp = balance + pnl;
      const double availM = RQ1 ? bp : bp / p.reqM;
      const double equity = (cash + t[0][1]) - t[3][1];
      const double mr = p.mainM * pnl;
      const int mc = (r.fl.y != 0) & ((equity <= -mr) | (bp <= -mr));
      const int insuff = (r.fl.z != 0) & ((availM <= r.ax1.x) | (balance <= 0.));
      const int go = (r.fl.x != 0) & !mc & !insuff;
      any_mc |= (r.fl.x != 0) & mc;
      const double c4 = ((cash + r.ax1.y) - r.yz.x) - r.yz.y;
      cash = go ? c4 : cash;
      if constexpr (I + 1 < APAD) {  // the last round's sums are recomputed by the caller
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          t[q][APAD + I] = go ? post[q] : t[q][APAD + I];
          update_up<APAD, (APAD + I) / 2>(t[q]);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) t[q][APAD + I] = go ? post[q] : t[q][APAD + I];
      }
      const int risk = mc ? MGN_MARGIN_CALL : (insuff ? MGN_INSUFF_MARGIN : MGN_GREEN);
      const bool own = ls == I / M;
      go_own[I % M] = own ? (go != 0) : go_own[I % M];
      rk[I % M] = (own & (r.fl.x != 0)) ? risk : rk[I % M];
      if constexpr (I + 1 < APAD)
        XRounds<M, S, RQ1, I + 1>::run(er, nxt, p, cash, t, go_own, rk, any_mc, ls);
    }
  }
};

// Per-order records of the lane's slots (the order-local half of
// Broker::handleTransaction, Broker.cpp:128-135, and Portfolio::
// handleTransaction, Portfolio.cpp:284-323): transaction price and cost, the
// ledger / mean entry / borrowed the order would leave, the four sum leaves
// before and after it, and the cash increments; published to the segment's
// LDS records.  The risk checks and cash updates that chain the orders are
// resolved afterwards (XRounds, or the speculative form in mgn_duo.h).
// WPP: publish the sum leaves (pre / post) and the check operands to LDS
// (the in-register DPP tree of broker_spec keeps them in lf_pre / lf_post /
// own instead; every order's cash terms X1, y, Z are published either way)
struct OwnChk {
  double aPX;
  double X1, y, Z;  // the order's cash terms (the chain's, broker_spec's dpp_chain)
  bool need_mc, need_insuff;
};
template <int M, int S, bool WPP = true>
__device__ __forceinline__ void order_prep(const Lane<M>& s, const KParams& p, EnvRecs<M * S>& er,
                                           const double (&uc)[M], int ls, double (&cu2)[M],
                                           double (&me2)[M], double (&bm3)[M], double (&tpr)[M],
                                           double (&tco)[M], double* lf_pre = nullptr,
                                           double* lf_post = nullptr, OwnChk* own = nullptr) {
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const double u = uc[m];
    const double cur = s.L[m];
    const double price = s.P[m];
    const double me0 = s.mep[m];
    const double bm0 = s.Bm[m];
    const bool opp = signbit(u) != signbit(cur);
    const bool rev = u > -1 * cur;
    const double excess = u + cur;
    const double slippage = (price * p.slip_rel) + p.slip_abs;
    const double tprice = u < 0 ? (price - slippage) : (price + slippage);
    const double tcost = fabs(u * price) * p.tc_rel + p.tc_abs;
    const bool close = opp && (fabs(u) > fabs(cur));
    const double units = close ? u + cur : u;
    const double cu1 = close ? 0. : cur;
    double me1;
    if (close) me1 = tprice;
    else if (opp) me1 = me0;
    else me1 = me0 + (tprice - me0) * (u / (u + cur));
    const double amt = tprice * units;
    const double use = amt * p.reqM;
    const double brw = amt - use;
    const double bm1 = bm0 + brw;
    const double c2l = cu1 + units;
    const bool closed = fabs(c2l) < 0.000001;
    const bool repay = closed && (bm1 > 0.);
    const bool neg = !repay && (bm1 < 0.);
    cu2[m] = c2l;
    me2[m] = closed ? 0. : me1;
    bm3[m] = (repay || neg) ? 0. : bm1;
    tpr[m] = tprice;
    tco[m] = tcost;
    OrderRec& r = er.r[ls * M + m];
    const double mk0 = (cur < 0.) ? 1.0 : 0.0;
    const double mk1 = (cu2[m] < 0.) ? 1.0 : 0.0;
    const double pr[4] = {cur * price, me0 * cur, cur * (me0 * mk0), bm0};
    const double po[4] = {cu2[m] * price, me2[m] * cu2[m], cu2[m] * (me2[m] * mk1), bm3[m]};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if constexpr (WPP) {
        r.pre[q] = pr[q];
        r.post[q] = po[q];
      } else {
        lf_pre[4 * m + q] = pr[q];
        lf_post[4 * m + q] = po[q];
      }
    }
    const double aPX = opp ? fabs(price * excess) : fabs(price * u);
    const double X1v = close ? cur * tprice : -0.0, Zv = (repay || neg) ? bm1 : 0.0;
    const bool act = u != 0.;
    if constexpr (WPP) {  // XRounds reads every order's check operands and cash terms from LDS
      r.X1 = X1v;
      r.y = use + tcost;
      r.Z = Zv;
      r.aPX = aPX;
      r.act = act;
      r.need_mc = !opp;
      r.need_insuff = !opp || rev;
      r.pad = 0;
    } else {  // broker_spec: the lane checks its own order and holds its cash terms
      own[m].aPX = aPX;
      own[m].X1 = X1v;
      own[m].y = use + tcost;
      own[m].Z = Zv;
      own[m].need_mc = !opp;
      own[m].need_insuff = !opp || rev;
    }
  }
  if constexpr (WPP) {
    // the segment's records are written by its own lanes: wave-scope ordering
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }

}

// the orders' effect on the lane's slots once their fate is known
template <int M>
__device__ __forceinline__ void apply_orders(Lane<M>& s, const bool (&go_own)[M],
                                             const double (&cu2)[M], const double (&me2)[M],
                                             const double (&bm3)[M], const double (&tpr)[M],
                                             const double (&tco)[M], const double (&uc)[M],
                                             double (&tp)[M], double (&tu)[M], double (&tc)[M]) {
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const bool go = go_own[m];
    s.L[m] = go ? cu2[m] : s.L[m];
    s.mep[m] = go ? me2[m] : s.mep[m];
    s.Bm[m] = go ? bm3[m] : s.Bm[m];
    tp[m] = go ? tpr[m] : tp[m];
    tu[m] = go ? uc[m] : tu[m];
    tc[m] = go ? tco[m] : tc[m];
  }
}

// The whole Broker::handleTransaction(units) (Broker.cpp:144-158) for the
// lane's segment, exchange form.  On return the lane's slots hold the new
// ledger, tp/tu/tc/rk the responses, `after` the canonical sums of the
// post-transaction portfolio, and any_mc whether any order of the segment
// was refused with MARGIN_CALL (the env's done condition, Env.h:216-218).
template <int M, int S, bool RQ1>
__device__ __forceinline__ void broker_x(Lane<M>& s, const KParams& p, EnvRecs<M * S>& er,
                                         double& cash, const Sums& s0, const double (&uc)[M],
                                         double (&tp)[M], double (&tu)[M], double (&tc)[M],
                                         int (&rk)[M], int ls, Sums& after, int& any_mc) {
  constexpr int APAD = M * S;
  double cu2[M], me2[M], bm3[M], tpr[M], tco[M];
  order_prep<M, S>(s, p, er, uc, ls, cu2, me2, bm3, tpr, tco);
  double t[4][2 * APAD];
#pragma unroll
  for (int a = 0; a < APAD; ++a) {
    const d2* rv = reinterpret_cast<const d2*>(&er.r[a]);
    const d2 p01 = rv[0], p23 = rv[1];
    t[0][APAD + a] = p01.x;
    t[1][APAD + a] = p01.y;
    t[2][APAD + a] = p23.x;
    t[3][APAD + a] = p23.y;
  }
  // internal nodes over the pre-order leaves; the root equals the carried s0
#pragma unroll
  for (int q = 0; q < 4; ++q) build_pre<APAD, APAD - 1>(t[q]);
  t[0][1] = s0.lp;
  t[1][1] = s0.ml;
  t[2][1] = s0.sh;
  t[3][1] = s0.b;
  bool go_own[M];
#pragma unroll
  for (int m = 0; m < M; ++m) go_own[m] = false;
  XRounds<M, S, RQ1, 0>::run(er, load_round<APAD>(er, 0), p, cash, t, go_own, rk, any_mc, ls);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();

  apply_orders<M>(s, go_own, cu2, me2, bm3, tpr, tco, uc, tp, tu, tc);
#pragma unroll
  for (int q = 0; q < 4; ++q) update_up<APAD, (2 * APAD - 1) / 2>(t[q]);
  after.lp = t[0][1];
  after.ml = t[1][1];
  after.sh = t[2][1];
  after.b = t[3][1];
}

// input selector
enum { IN_NONE = 0, IN_UNITS = 1, IN_SINGLE = 2, IN_DISCRETE = 3 };

__device__ __forceinline__ double dsr_one(double r, double A, double B) {
  const double dA = r - A;
  const double dB = r * r - B;
  const double t = B - A * A;
  // ((B - A^2)^2)^(3/4) = |B - A^2|^(3/2), evaluated as a*sqrt(a): within 2 ulp of
  // libm pow (outputs are compared at rtol 1e-12; they never feed back into state)
  const double a = fabs(t);
  return rt_div(B * dA - (A * dB) / 2, a * rt_sqrt(a) + 1.1920928955078125e-07);
}
__device__ __forceinline__ double ddr_one(double r, double A, double B) {
  // r > 0: (r - A/2) / (sqrt(B) + eps); else (B(r - A/2) - A r^2/2) / (B^(3/2) + eps),
  // B^(3/2) as B*sqrt(B); one division with the branch's operands selected
  const double sB = rt_sqrt(B);
  const double h = r - A / 2;
  const bool pos = r > 0.;
  const double num = pos ? h : (B * h - (A * (r * r)) / 2);
  const double den = (pos ? sB : B * sB) + 1.1920928955078125e-07;
  return rt_div(num, den);
}
// ddr_one with its reward-independent operands (A/2 and the two
// denominators) evaluated ahead of the reward: the same operations on the
// same operands, so the same result
struct DdrPre {
  double hA, dpos, dneg;
};
__device__ __forceinline__ DdrPre ddr_pre(double A, double B) {
  const double sB = rt_sqrt(B);
  return DdrPre{A / 2, sB + 1.1920928955078125e-07, B * sB + 1.1920928955078125e-07};
}
__device__ __forceinline__ double ddr_one_pre(double r, double A, double B, const DdrPre& q) {
  const double h = r - q.hA;
  const bool pos = r > 0.;
  const double num = pos ? h : (B * h - (A * (r * r)) / 2);
  return rt_div(num, pos ? q.dpos : q.dneg);
}
// ddr_one_pre / dsr_one_den with the reciprocals of their denominators formed
// once per pop rather than per summand, as rt_div forms them (the IEEE
// division where a denominator is not a normal number): the same operations
// on the same operands
__device__ __forceinline__ double rt_rcp(double b) {
  double r = __builtin_amdgcn_rcp(b);
  r = __builtin_fma(r, __builtin_fma(-b, r, 1.0), r);
  return __builtin_fma(r, __builtin_fma(-b, r, 1.0), r);
}
__device__ __forceinline__ double div_pre(double a, double b, double rb) {
  double q = a * rb;
  if (!__builtin_amdgcn_class(b, kNormalClass)) {  // (rt_div's IEEE case, kept in its branch)
    double x = a;
    asm volatile("" : "+v"(x));
    q = x / b;
  }
  return q;
}
struct DdrPreR {
  DdrPre q;
  double rpos, rneg;
};
__device__ __forceinline__ DdrPreR ddr_pre_r(double A, double B) {
  const DdrPre q = ddr_pre(A, B);
  return DdrPreR{q, rt_rcp(q.dpos), rt_rcp(q.dneg)};
}
__device__ __forceinline__ double ddr_one_r(double r, double A, double B, const DdrPreR& c) {
  const double h = r - c.q.hA;
  const bool pos = r > 0.;
  const double num = pos ? h : (B * h - (A * (r * r)) / 2);
  return div_pre(num, pos ? c.q.dpos : c.q.dneg, pos ? c.rpos : c.rneg);
}
__device__ __forceinline__ double dsr_one_r(double r, double A, double B, double den, double rden) {
  const double dA = r - A;
  const double dB = r * r - B;
  return div_pre(B * dA - (A * dB) / 2, den, rden);
}
__device__ __forceinline__ double clip1(double v) { return v < -1. ? -1. : (v > 1. ? 1. : v); }
// dsr_one with its reward-independent denominator evaluated once per pop (the
// same operations on the same operands)
__device__ __forceinline__ double dsr_den(double A, double B) {
  const double a = fabs(B - A * A);
  return a * rt_sqrt(a) + 1.1920928955078125e-07;
}
__device__ __forceinline__ double dsr_one_den(double r, double A, double B, double den) {
  const double dA = r - A;
  const double dB = r * r - B;
  return rt_div(B * dA - (A * dB) / 2, den);
}
// the summand of one NStepBuffer entry at discount slot k (nstep_buffer.py:62-91,
// :128-162; PPC / none: the stored value)
struct PopPre {
  DdrPre q;
  double dden;
};
__device__ __forceinline__ PopPre pop_pre(int shaper, double A, double B) {
  PopPre c;
  c.q = DdrPre{0., 0., 0.};
  c.dden = 0.;
  if (shaper == MGN_SHAPER_DDR) c.q = ddr_pre(A, B);
  else if (shaper == MGN_SHAPER_DSR) c.dden = dsr_den(A, B);
  return c;
}
__device__ __forceinline__ double pop_term(int shaper, double r, double A, double B, const PopPre& c,
                                           double disc_k) {
  double f = r;
  if (shaper == MGN_SHAPER_DSR) f = dsr_one_den(r, A, B, c.dden);
  else if (shaper == MGN_SHAPER_DDR) f = ddr_one_pre(r, A, B, c.q);
  return disc_k * f;
}

// The running-sum n-step pop (MGN_NSTEP_POP_RUNNING; within north_star's 1e-6
// of the exact pop): per env, the buffer's discounted sums
// sum_k gamma^k {1, r_k, r_k^2}, split by DDR's sign test (r > 0 / else).
// Every DSR / DDR / PPC / none pop is a function of them
// (nstep_buffer.py:62-91, 128-162, 182-204, 23-27):
//   DSR   sum_k g^k [B (r_k - A) - A (r_k^2 - B) / 2]
//           = B (S_r - A S_1) - A/2 (S_rr - B S_1)
//   DDR   sum_{r>0} g^k (r_k - A/2) / dpos
//           + sum_{r<=0} g^k [B (r_k - A/2) - A r_k^2 / 2] / dneg
//   PPC / none  S_r over the stored values
// An entry appended at position L-1 enters at weight g^(L-1); a pop removes
// the oldest (weight g^0 = 1) and divides the rest by g (every entry moves
// one position forward), so a pop costs O(1) instead of L summands and an
// ordered sum.  The slides' rounding grows by 1/g per pop, so the sums are
// re-formed from the buffer every n pops and the host grants this pop only
// where g^n >= 1e-3 (mgn_api.hip kparams): drift <= n eps g^-n of the sums'
// magnitude, < 1e-11 at n = 64.
struct NstRun {
  double p1, pr, prr, n1, nr, nrr;
};
__device__ __forceinline__ void nrun_zero(NstRun& s) { s.p1 = s.pr = s.prr = s.n1 = s.nr = s.nrr = 0.; }
__device__ __forceinline__ void nrun_add(NstRun& s, double r, double w) {
  const double wr = w * r, wrr = wr * r;
  const bool pos = r > 0.;
  s.p1 += pos ? w : 0.;
  s.pr += pos ? wr : 0.;
  s.prr += pos ? wrr : 0.;
  s.n1 += pos ? 0. : w;
  s.nr += pos ? 0. : wr;
  s.nrr += pos ? 0. : wrr;
}
// the oldest entry r0 leaves; the rest move one position forward
__device__ __forceinline__ void nrun_slide(NstRun& s, double r0, double rg) {
  nrun_add(s, r0, -1.0);
  s.p1 *= rg;
  s.pr *= rg;
  s.prr *= rg;
  s.n1 *= rg;
  s.nr *= rg;
  s.nrr *= rg;
}
// every lane of an S-lane env segment holds part of the sums -> all of them
template <int S>
__device__ __forceinline__ void nrun_allsum(NstRun& s) {
  s.p1 = seg_sum<S>(s.p1);
  s.pr = seg_sum<S>(s.pr);
  s.prr = seg_sum<S>(s.prr);
  s.n1 = seg_sum<S>(s.n1);
  s.nr = seg_sum<S>(s.nr);
  s.nrr = seg_sum<S>(s.nrr);
}
// A pop of a buffer of len entries, split into what the sums give (`base`:
// formed ahead of the step's reward -- the shaper state A, B and len are
// known when the step's evaluation starts) and the term of the entry v
// appended at weight w (nrun_fin).  The quotients by len and by the
// reward-independent denominators are one refined reciprocal per class.
struct NstPre {
  double base, cp, cn, hA, A, B;
};
__device__ __forceinline__ NstPre nrun_pre(int shaper, const NstRun& s, int len, double A, double B) {
  NstPre q;
  q.A = A;
  q.B = B;
  q.hA = A / 2;
  q.cp = q.cn = 0.;
  if (shaper == MGN_SHAPER_DSR) {
    const double S1 = s.p1 + s.n1, Sr = s.pr + s.nr, Srr = s.prr + s.nrr;
    // ((B - A^2)^2)^(3/4) + EPS as dsr_den, its square root and the
    // reciprocal with one refinement each (as DDR's below)
    const double a = fabs(B - A * A);
    const double y = __builtin_amdgcn_rsq(a);
    double gq = a * y;
    gq = __builtin_fma(gq, __builtin_fma(-gq, 0.5 * y, 0.5), gq);
    const double den = (a * (a > 0. ? gq : 0.) + 1.1920928955078125e-07) * len;
    const double r0 = __builtin_amdgcn_rcp(den);
    q.cp = __builtin_fma(r0, __builtin_fma(-den, r0, 1.0), r0);
    q.base = q.cp * (B * (Sr - A * S1) - q.hA * (Srr - B * S1));
  } else if (shaper == MGN_SHAPER_DDR) {
    // (the square root and the reciprocal with one refinement each: within
    // 1e-13 relative, far inside the pop's 1e-6; the exact pop's rt_sqrt /
    // two rt_rcp measured 2.60 against 2.54 us/step at n = 20 DDR,
    // profiles/r06h_ab.txt)
    const double y = __builtin_amdgcn_rsq(B);
    double gq = B * y;
    gq = __builtin_fma(gq, __builtin_fma(-gq, 0.5 * y, 0.5), gq);
    const double sB = B > 0. ? gq : 0.;  // (rsq(0) = inf)
    const double dpos = sB + 1.1920928955078125e-07, dneg = B * sB + 1.1920928955078125e-07;
    const double den = (dpos * dneg) * len;
    const double r0 = __builtin_amdgcn_rcp(den);
    const double r = __builtin_fma(r0, __builtin_fma(-den, r0, 1.0), r0);
    q.cp = dneg * r;
    q.cn = dpos * r;
    q.base = q.cp * (s.pr - q.hA * s.p1) + q.cn * (B * (s.nr - q.hA * s.n1) - q.hA * s.nrr);
  } else if (shaper == MGN_SHAPER_SORTINO_B) {
    q.base = s.p1 - s.n1;
  } else {
    q.base = s.pr + s.nr;
  }
  return q;
}
// the pop with v appended at weight w (sortino_shaperB: its root at weight
// w2); DSR / DDR: clip(sum / len) as __main_func__ (nstep_buffer.py:78, :144)
__device__ __forceinline__ double nrun_fin_sb(const NstPre& q, double v, double root, double w, double w2) {
  return clip1(q.base + ((v > 0.) ? w * v : ((v < 0.) ? -(w2 * root) : 0.)));
}
__device__ __forceinline__ double nrun_fin(int shaper, const NstPre& q, double v, double w) {
  if (shaper == MGN_SHAPER_DSR) return clip1(q.base + q.cp * (w * (q.B * (v - q.A) - q.hA * (v * v - q.B))));
  if (shaper == MGN_SHAPER_DDR) {
    const bool pos = v > 0.;
    const double t = pos ? (v - q.hA) : (q.B * (v - q.hA) - q.hA * (v * v));
    return clip1(q.base + (pos ? q.cp : q.cn) * (w * t));
  }
  return q.base + w * v;
}
// the pop of a buffer of len entries from its sums alone
__device__ __forceinline__ double nrun_pop(int shaper, const NstRun& s, int len, double A, double B) {
  const NstPre q = nrun_pre(shaper, s, len, A, B);
  return (shaper == MGN_SHAPER_DSR || shaper == MGN_SHAPER_DDR || shaper == MGN_SHAPER_SORTINO_B) ? clip1(q.base)
                                                                                                 : q.base;
}

// naive shapers (nstep_buffer.py:207-312), benchmark 0.  x**e and x**(1/e) as
// numpy evaluates them on float64 arrays: exponents 2 and 0.5 take numpy's
// square / sqrt fast paths, others pow (the oracle makes the same split).
__device__ __forceinline__ double pow_e(double x, double e) { return e == 2.0 ? x * x : pow(x, e); }
__device__ __forceinline__ double root_e(double x, double e) {
  return e == 2.0 ? sqrt(x) : pow(x, 1.0 / e);
}
__device__ __forceinline__ double max_m1(double x) { return (x < -1.) ? -1. : x; }          // clip(x, -1, None)
__device__ __forceinline__ double min_0(double x) { return (x < 0. || x != x) ? x : 0.; }  // minimum(x, 0.)

// sortino_shaperB's summand of entry k of a buffer of more than one entry
// (nstep_buffer.py:293-312, naive_n's): the clipped, sign-preserving e-th
// root of the discounted entry; the pop is clip(sum) over the entries in order
__device__ __forceinline__ double sortinoB_term(double r, double disc_k, double ex) {
  const double v = max_m1((r - 0.) * disc_k);
  return (v < 0.) ? -root_e(-v, ex) : v;
}

// sortino_shaperB's running-sum pop (MGN_NSTEP_POP_RUNNING): with
// x_k = gamma^k r_k, the pop is clip(sum_k (x_k >= 0 ? x_k : -(-x_k)^(1/e)))
// and -(-x_k)^(1/e) = -(gamma^k)^(1/e) (-r_k)^(1/e), so two discounted sums
// carry it -- NstRun.p1 = sum_{r>0} gamma^k r_k, .n1 = sum_{r<0}
// (gamma^k)^(1/e) (-r_k)^(1/e) (the entry's root formed once, at its
// append) -- while no entry can reach the per-term clip at -1 (x_k < -1 needs
// r_k < -1: .prr counts those entries, and a pop with any of them is the exact
// one).  A pop removes the oldest entry and divides p1 by gamma, n1 by
// gamma^(1/e).
__device__ __forceinline__ void nrun_add_sb(NstRun& s, double r, double root, double w, double w2) {
  s.p1 += (r > 0.) ? w * r : 0.;
  s.n1 += (r < 0.) ? w2 * root : 0.;
  s.prr += (r < -1. || r != r) ? 1. : 0.;
}
__device__ __forceinline__ void nrun_slide_sb(NstRun& s, double r0, double root0, double rg, double rg2) {
  s.p1 = (s.p1 - ((r0 > 0.) ? r0 : 0.)) * rg;
  s.n1 = (s.n1 - ((r0 < 0.) ? root0 : 0.)) * rg2;
  s.prr -= (r0 < -1. || r0 != r0) ? 1. : 0.;
}

// the len(nstep_buffer) == 1 heuristics (:212-216, :244-249, :286-291)
__device__ __noinline__ double naive1(int shaper, double r, double ex) {
  double diff = r - 0.;
  if (shaper == MGN_SHAPER_SHARPE) {  // no clip; r == 0 gives 0/0 = nan as in the reference
    diff = (diff != 0.) ? diff : 0.;
    return diff / sqrt(diff * diff);
  }
  if (shaper == MGN_SHAPER_SORTINO_A) {
    const double downside = root_e(pow_e(fabs(diff), ex), ex);
    return clip1(0.1 * ((diff != 0.) ? diff / downside : 0.));
  }
  diff = max_m1(diff);
  diff = (diff < 0.) ? -root_e(-diff, ex) : diff;
  return clip1(diff);
}

// L > 1 entries r_k = ring[(head + k) % n][d], diffs_k = (r_k - 0.) * gamma^k
// (sharpe :217-239, sortino_shaperA :251-272, sortino_shaperB :293-312)
__device__ __noinline__ double naive_n(int shaper, const double* ring, int n, int D, int d, int head,
                                       int len, const double* disc, double ex) {
  double s = 0., s2 = 0.;
  for (int k = 0; k < len; ++k) {
    const double x = (ring[(size_t)((head + k) % n) * D + d] - 0.) * disc[k];
    if (shaper == MGN_SHAPER_SHARPE) {
      s += x;
      s2 += x * x;
    } else if (shaper == MGN_SHAPER_SORTINO_A) {
      s += x;
      const double down = max_m1(min_0(x));
      s2 += root_e(pow_e(fabs(down), ex) / (len - 1), ex);
    } else {
      const double v = max_m1(x);
      s += (v < 0.) ? -root_e(-v, ex) : v;
    }
  }
  if (shaper == MGN_SHAPER_SHARPE) {
    const double num = s / len;
    const double denom = sqrt(s2 / (len - 1));
    return clip1(.1 * ((denom != 0.) ? num / denom : 0.));
  }
  if (shaper == MGN_SHAPER_SORTINO_A) {
    const double num = s / len;
    return (s2 != 0.) ? clip1(.1 * (num / s2)) : ((num == 0.) ? 0. : 1.);
  }
  return clip1(s);
}

// one shaper evaluation + parameter update, n = 1 (nstep_buffer.py:62-91, :128-162)
__device__ __forceinline__ double shape(int shaper, double r, double& A, double& B, double eta,
                                        double cos_term, double ex) {
  if (shaper == MGN_SHAPER_DSR) {
    const double out = clip1((0.0 + 1.0 * dsr_one(r, A, B)) / 1);
    A += eta * (r - A);
    B += eta * (r * r - B);
    return out;
  }
  if (shaper == MGN_SHAPER_DDR) {
    const double out = clip1((0.0 + 1.0 * ddr_one(r, A, B)) / 1);
    double m = r < 0. ? r : 0.;
    if (r != r) m = r;
    A += eta * (r - A);
    B += eta * (m * m - B);
    return out;
  }
  if (shaper == MGN_SHAPER_PPC) return 1.0 * (r + cos_term);
  if (shaper >= MGN_SHAPER_SHARPE) return naive1(shaper, r, ex);
  return r;
}

// NStepBuffer.add + pop_nstep_sarsd for reward column d of one env
// (nstep_buffer.py:315-356 as replay_buffer.py:68-80 drives it): append v; pop
// once if the buffer is full, every entry if done.  A pop aggregates the
// whole buffer (L entries, discounts gamma^0..gamma^(L-1)): DSR/DDR
// clip(sum_k gamma^k f(r_k; A, B) / L) and then A, B from the oldest reward
// (:62-91, :128-162); PPC / none: sum_k gamma^k v_k, v = r (+ temp*cos for
// PPC, stored at add time) (:182-204, :23-27).  Ring (n, D) per env, oldest
// at `head`; out: the env's (n, D) row of this step, zero after the pops.
// ring: the env's (n, D) ring (global for k_step, LDS for k_step_duo)
template <typename RingP, typename OutP>
__device__ __forceinline__ void nstep_column(const KParams& p, RingP ring, OutP out, int d, int D,
                                          double v, bool done, int len, int head, double& A,
                                          double& B) {
  const int n = p.nstep;
  ring[(size_t)((head + len) % n) * D + d] = v;
  len += 1;
  const bool sr = p.shaper == MGN_SHAPER_DSR || p.shaper == MGN_SHAPER_DDR;
  const bool naive = p.shaper >= MGN_SHAPER_SHARPE;
  int pops = 0;
  while (len >= n || (done && len > 0)) {
    if (naive) {
      const double res = (len == 1) ? naive1(p.shaper, ring[(size_t)head * D + d], p.sexp)
                                    : naive_n(p.shaper, ring, n, D, d, head, len, p.disc, p.sexp);
      if (out) out[(size_t)pops * D + d] = res;
      head = (head + 1) % n;
      len -= 1;
      pops += 1;
      if (!done && len < n) break;
      continue;
    }
    double acc = 0.0;
    const PopPre c = pop_pre(p.shaper, A, B);
    for (int k = 0, idx = head; k < len; ++k, idx = (idx + 1 == n) ? 0 : idx + 1)
      acc += pop_term(p.shaper, ring[(size_t)idx * D + d], A, B, c, p.disc[k]);
    double res = acc;
    if (sr) {
      res = clip1(acc / len);
      const double r0 = ring[(size_t)head * D + d];
      A += p.eta * (r0 - A);
      if (p.shaper == MGN_SHAPER_DSR) {
        B += p.eta * (r0 * r0 - B);
      } else {
        double m = r0 < 0. ? r0 : 0.;
        if (r0 != r0) m = r0;
        B += p.eta * (m * m - B);
      }
    }
    if (out) out[(size_t)pops * D + d] = res;
    head = (head + 1) % n;
    len -= 1;
    pops += 1;
    if (!done && len < n) break;
  }
  if (out)
    for (int j = pops; j < n; ++j) out[(size_t)j * D + d] = 0.;
}

// ---------------------------------------------------------------------------
// The fused step kernel: K consecutive Env steps per launch, state held in
// registers between steps.  in_kind selects Env::step() / step(units) /
// step(assetIdx, units) / discrete actions via action_to_transaction.
// RQ1: required_margin == 1.0, where x / required_margin == x exactly and the
// divisions are skipped.  NST: n-step aggregation (nstep > 1) compiled in.
// speculative Broker resolution for one asset per lane (defined in mgn_duo.h)
template <int S, bool RQ1, bool ONE = false>
__device__ __forceinline__ void broker_spec(Lane<1>& s, const KParams& p, EnvRecs<S>& er,
                                            double& cash, const double (&uc)[1], double (&tp)[1],
                                            double (&tu)[1], double (&tc)[1], int (&rk)[1], int ls,
                                            Sums& after, int& any_mc);

template <int M, int S, bool RQ1, bool NST>
__global__ __launch_bounds__(BLOCK) void k_step(KParams p, mgn_traj out, int in_kind,
                                                const double* __restrict__ units_in,
                                                const int32_t* __restrict__ aidx_in,
                                                const int8_t* __restrict__ act_in, int K) {
  // loop-invariant fp64 parameters live in VGPRs: the kernel is SGPR-bound
  // (pointers), and an SGPR spill costs a v_readlane per use in the loop
  p.init_cash = in_vgpr(p.init_cash);
  p.reqM = in_vgpr(p.reqM);
  p.mainM = in_vgpr(p.mainM);
  p.slip_rel = in_vgpr(p.slip_rel);
  p.slip_abs = in_vgpr(p.slip_abs);
  p.tc_rel = in_vgpr(p.tc_rel);
  p.tc_abs = in_vgpr(p.tc_abs);
  p.eta = in_vgpr(p.eta);
  p.cos_temp = in_vgpr(p.cos_temp);
  p.unit_size = in_vgpr(p.unit_size);
  constexpr int EPB = BLOCK / S;  // envs per block
  constexpr int APADK = M * S;
  // exchange-form Broker rounds (LDS: M * 28 KB per block)
  constexpr bool XCH = (M * S <= 16) && (M <= 2) && (S >= 2);
  __shared__ EnvRecs<XCH ? M * S : 1> recs[XCH ? EPB : 1];
  // loop-invariant tables read every step (generator parameters, PPC target,
  // n-step discounts) are staged in LDS: a global load in the step loop would
  // expose its full latency to the single resident wave
  __shared__ mgn_asset_source s_src[APADK];  // p.A <= APADK assets
  __shared__ double s_tgt[MGN_MAX_ASSETS + 1];
  __shared__ double s_disc[NST ? MGN_MAX_NSTEP : 1];
  {
    const double* g = reinterpret_cast<const double*>(p.src);
    double* d = reinterpret_cast<double*>(s_src);
    const int n = p.A * (int)(sizeof(mgn_asset_source) / sizeof(double));
    for (int i = threadIdx.x; i < n; i += BLOCK) d[i] = g[i];
    if (p.target)
      for (int i = threadIdx.x; i <= p.A; i += BLOCK) s_tgt[i] = p.target[i];
    if constexpr (NST)
      for (int i = threadIdx.x; i < p.nstep; i += BLOCK) s_disc[i] = p.disc[i];
    __syncthreads();
    p.src = s_src;
    if (p.target) p.target = s_tgt;
    if constexpr (NST) p.disc = s_disc;
  }
  const int tid = threadIdx.x;
  const int ls = tid % S;
  const int env = blockIdx.x * EPB + tid / S;
  if (env >= p.N) return;
  const int A = p.A;
  const int D = p.D;

  Lane<M> s;
  load_lane<M>(s, p, env, ls);
  if (p.replay && p.F <= S) s.fcol = ls;  // one feature column per lane: prefetched
  double cash = p.cash[env];
  uint64_t ts = p.ts[env];
  s.dskip = p.dskip[env];
  double shA[M], shB[M];  // shaper state: slot values for D==A, [0] for D==1
#pragma unroll
  for (int m = 0; m < M; ++m) {
    if (D == 1) {
      shA[m] = p.sA[env];
      shB[m] = p.sB[env];
    } else {
      shA[m] = s.valid[m] ? p.sA[(size_t)env * A + s.asset[m]] : 0.;
      shB[m] = s.valid[m] ? p.sB[(size_t)env * A + s.asset[m]] : 0.;
    }
  }
  double ep_ret = p.ep[(size_t)env * 2], ep_len = p.ep[(size_t)env * 2 + 1];
  int32_t nlen = 0, nhead = 0;  // NStepBuffer fill count / oldest index (n > 1)
  if constexpr (NST) {
    nlen = p.nlen[env];
    nhead = p.nhead[env];
  }
  int32_t head = 0, len = 0;
  if (p.W > 0) {
    head = p.rhead[env];
    len = p.rlen[env];
  }
  // PPC target norm: entry 0 + canonical tree over the assets
  double cos_qn = 0.;
  if (p.shaper == MGN_SHAPER_PPC) {
    double qq[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const double q = s.valid[m] ? p.target[1 + s.asset[m]] : 0.;
      qq[m] = q * q;
    }
    cos_qn = sqrt(p.target[0] * p.target[0] + canon<M, S>(qq));
  }

  // agent-side reward only when it is an output or feeds the shaper
  const bool need_ar = (p.reward_mode != MGN_REWARD_ENV_LOG) || (out.agent_reward != nullptr);
  // Portfolio sums of the current state.  They are carried from the previous
  // step's post-getData sums (same inputs, so bit-identical to a recompute)
  // and recomputed only after a reset.
  Sums s0 = port_sums<M, S>(s.L, s.mep, s.Bm, s.P);
  // discrete actions of the next step are prefetched one step ahead
  int8_t act_next[M];
  if (in_kind == IN_DISCRETE) {
#pragma unroll
    for (int m = 0; m < M; ++m)
      act_next[m] = s.valid[m] ? act_in[(size_t)env * A + s.asset[m]] : 0;
  }

  // Per-segment state machine: a segment either steps (k < K) or runs the
  // source ticks of an auto-reset (Env::reset's getData + initialize_history,
  // `pending` of them), so one inlined getData serves both paths.
  int k = 0;
  int pending = 0;
  int hcnt = p.W;  // next launch-history row
  while (true) {
    const bool stepping = (pending == 0) && (k < K);
    const bool ticking = stepping || (pending > 0);
    if (__ballot(ticking) == 0) break;
    const size_t oN = (size_t)k * p.N, oNA = (size_t)k * p.N * A;
    double uc[M], prevVal[M], tp[M], tu[M], tc[M];
    int rk[M];
    double prevEq = 0.;
    int mcall = 0;
    Sums sa = s0;  // canonical sums after the Broker (ledger unchanged: s0)
    int any_mc = 0;  // exchange form: some order refused with MARGIN_CALL
#pragma unroll
    for (int m = 0; m < M; ++m) {
      tp[m] = 0.;
      tu[m] = 0.;
      tc[m] = 0.;
      rk[m] = MGN_GREEN;
      uc[m] = 0.;
    }
    if (stepping) {
      // ---- action -> units for this lane's slots
      prevEq = (cash + s0.lp) - s0.b;  // Env.h:208
      if (in_kind == IN_DISCRETE) {     // dqn.py:160-179
        const double bp = (cash + s0.sh) + (s0.lp - s0.ml);
        const double avM = RQ1 ? bp : bp / p.reqM;
        const int half = p.atoms / 2;
        int8_t act_cur[M];
#pragma unroll
        for (int m = 0; m < M; ++m) {
          act_cur[m] = act_next[m];
          if (k + 1 < K && s.valid[m])
            act_next[m] = act_in[oNA + (size_t)p.N * A + (size_t)env * A + s.asset[m]];
        }
#pragma unroll
        for (int m = 0; m < M; ++m) {
          if (!s.valid[m]) continue;
          const int a = act_cur[m];
          const double u = p.unit_size * avM / s.P[m];
          uc[m] = (double)(a - half) * u;
          if (a == 0) uc[m] = (s.L[m] != 0) ? -s.L[m] : 0.;
        }
      } else if (in_kind == IN_UNITS) {
#pragma unroll
        for (int m = 0; m < M; ++m)
          uc[m] = s.valid[m] ? units_in[oNA + (size_t)env * A + s.asset[m]] : 0.;
      } else if (in_kind == IN_SINGLE) {
        const int ai = aidx_in[env];
        const double u = units_in[oN + env];
#pragma unroll
        for (int m = 0; m < M; ++m) uc[m] = (s.valid[m] && s.asset[m] == ai) ? u : 0.;
      }
#pragma unroll
      for (int m = 0; m < M; ++m) prevVal[m] = s.L[m] * s.P[m];
      // ---- Broker::handleTransaction(units): serial rounds over assets
      if (in_kind != IN_NONE) {
        if constexpr (XCH) {
          if (!(p.ablate & 1)) {
            if constexpr (M == 1) {
              // one asset per lane: the speculative resolution of the two-role
              // kernel (mgn_duo.h) -- one pass when no order is refused
              broker_spec<S, RQ1>(s, p, recs[tid / S], cash, uc, tp, tu, tc, rk, ls, sa, any_mc);
            } else {
              broker_x<M, S, RQ1>(s, p, recs[tid / S], cash, s0, uc, tp, tu, tc, rk, ls, sa, any_mc);
            }
          }
        } else {
          if (!(p.ablate & 1)) Rounds<M, S, 0>::run(s, p, cash, uc, tp, tu, tc, rk, ls);
          sa = port_sums<M, S>(s.L, s.mep, s.Bm, s.P);
        }
        // BrokerResponse.marginCall (Broker.cpp:156-157)
        mcall = margin_call(sa, cash, p.mainM) ? 1 : 0;
      }
    }
    if (ticking) {
      // ---- dataSource->getData()
      if (!(p.ablate & 2)) gen_tick<M>(s, p, env, ts);
      ts = next_ts<M>(s, p, ts);
    }
    if (stepping) {
      // ---- reward / done (Env.h:211-223).  Only the L*P sum sees the new
      // prices; the ledger sums are the ones after the Broker.
      Sums q = sa;
      {
        double tlp[M];
#pragma unroll
        for (int m = 0; m < M; ++m) tlp[m] = s.L[m] * s.P[m];
        q.lp = canon<M, S>(tlp);
      }
      const double curEq = (cash + q.lp) - q.b;
      const double ratio = curEq / prevEq;
      const double clampv = (in_kind == IN_SINGLE) ? 0.01 : 0.3;
      const double reward = log_ratio((ratio < clampv) ? clampv : ratio);
      int bad = 0;
      if constexpr (XCH) {
        bad = any_mc;  // every lane saw every round's risk
      } else {
#pragma unroll
        for (int m = 0; m < M; ++m) bad |= (rk[m] != MGN_GREEN && rk[m] != MGN_INSUFF_MARGIN) ? 1 : 0;
        bad = seg_or<S>(bad);
      }
      const bool done = bad || margin_call(q, cash, p.mainM) || (curEq < 0.1 * p.init_cash);

      // ---- State.portfolio = ledgerNormedFull (Portfolio.cpp:150-155)
      const double port0 = (cash - q.b) / curEq;
      double portA[M];
#pragma unroll
      for (int m = 0; m < M; ++m) portA[m] = (s.L[m] * s.P[m]) / curEq;

      // ---- agent-side per-asset reward (offpolicy_q.py:152-164)
      double ar[M];
#pragma unroll
      for (int m = 0; m < M; ++m) {
        if (!s.valid[m] || !need_ar) {
          ar[m] = 0.;
          continue;
        }
        double v = (((s.L[m] * s.P[m]) - prevVal[m]) - (tu[m] * tp[m] + tc[m])) / prevEq;
        v += 1;
        v = (v < .35) ? .35 : v;
        ar[m] = (p.ablate & 8) ? v : log_ratio(v);
      }
      // ---- reward shaping
      double cos_term = 0.;
      if (p.shaper == MGN_SHAPER_PPC) {
        double pp[M], pq[M];
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const double qv = s.valid[m] ? p.target[1 + s.asset[m]] : 0.;
          const double pv = s.valid[m] ? portA[m] : 0.;
          pp[m] = pv * pv;
          pq[m] = pv * qv;
        }
        const double np_ = sqrt(port0 * port0 + canon<M, S>(pp));
        const double dot = port0 * p.target[0] + canon<M, S>(pq);
        cos_term = p.cos_temp * (dot / (np_ * cos_qn));
      }
      double shaped_s = 0., rin_s = 0.;
      double shaped_v[M];
      constexpr bool nst = NST;
      if (D == 1) rin_s = (p.reward_mode == MGN_REWARD_AGENT_SUM) ? canon<M, S>(ar) : reward;
      if constexpr (!NST) {
        if (D == 1) {
          shaped_s = shape(p.shaper, rin_s, shA[0], shB[0], p.eta, cos_term, p.sexp);
        } else {
#pragma unroll
          for (int m = 0; m < M; ++m)
            shaped_v[m] = s.valid[m] ? shape(p.shaper, ar[m], shA[m], shB[m], p.eta, cos_term, p.sexp) : 0.;
        }
      } else {
        // NStepBuffer add + pops (replay_buffer.py:68-80); every lane tracks the
        // segment's fill count / oldest index, column owners touch the ring
        const int n = p.nstep;
        const int L1 = nlen + 1;
        const int pops = done ? L1 : (L1 >= n ? 1 : 0);
        const bool ppc = p.shaper == MGN_SHAPER_PPC;
        double* row = (out.shaped && !(p.ablate & 4)) ? out.shaped + (oN + env) * (size_t)n * D : nullptr;
        if (D == 1) {
          if (ls == 0)
            nstep_column(p, p.nring + (size_t)env * n, row, 0, 1, ppc ? rin_s + cos_term : rin_s, done,
                         nlen, nhead, shA[0], shB[0]);
        } else {
#pragma unroll
          for (int m = 0; m < M; ++m)
            if (s.valid[m])
              nstep_column(p, p.nring + (size_t)env * n * D, row, s.asset[m], D,
                           ppc ? ar[m] + cos_term : ar[m], done, nlen, nhead, shA[m], shB[m]);
        }
        if (ls == 0 && out.n_shaped && !(p.ablate & 4)) out.n_shaped[oN + env] = (uint8_t)pops;
        nhead = (nhead + pops) % n;
        nlen = L1 - pops;
      }

      // ---- outputs
#pragma unroll
      for (int m = 0; m < M; ++m) {
        if (!s.valid[m] || (p.ablate & 4)) continue;
        const size_t i = oNA + (size_t)env * A + s.asset[m];
        if (out.tprice) out.tprice[i] = tp[m];
        if (out.tunits) out.tunits[i] = tu[m];
        if (out.tcost) out.tcost[i] = tc[m];
        if (out.risk) out.risk[i] = (uint8_t)rk[m];
        if (out.obs_port) out.obs_port[(size_t)k * p.N * (A + 1) + (size_t)env * (A + 1) + 1 + s.asset[m]] = portA[m];
        if (D != 1) {
          if (out.agent_reward) out.agent_reward[i] = ar[m];
          if (out.shaped && !nst) out.shaped[i] = shaped_v[m];
        }
      }
      if (out.obs_price && !(p.ablate & 4))
        put_feats<M, S>(s, p, ls, out.obs_price + (oN + env) * (size_t)p.F);
      if (ls == 0 && !(p.ablate & 4)) {
        if (out.data_end) out.data_end[oN + env] = p.replay ? p.rp_end[s.row] : 0;
        if (out.reward) out.reward[oN + env] = reward;
        if (out.done) out.done[oN + env] = done ? 1 : 0;
        if (out.timestamp) out.timestamp[oN + env] = ts;
        if (out.margin_call) out.margin_call[oN + env] = (uint8_t)mcall;
        if (!NST && out.n_shaped) out.n_shaped[oN + env] = 1;
        if (out.obs_port) out.obs_port[(size_t)k * p.N * (A + 1) + (size_t)env * (A + 1)] = port0;
        if (D == 1) {
          if (out.agent_reward) out.agent_reward[oN + env] = rin_s;
          if (out.shaped && !nst) out.shaped[oN + env] = shaped_s;
        }
      }

      // ---- episode statistics
      ep_ret += reward;
      ep_len += 1;
      if (done) {
        if (ls == 0) {
          double* st = p.epstats + (size_t)env * 4;
          st[0] = ep_ret;
          st[1] = ep_len;
          st[2] = curEq;
          st[3] = st[3] + 1;
        }
        ep_ret = 0;
        ep_len = 0;
      }
      // ---- window; agent reset (offpolicy_q.py:199-201)
      if (p.W > 0) {
        ring_push<M, S>(s, p, env, ls, cash, ts, head, len, p.hist ? hcnt : -1);
        if (p.hist) hist_mark(p, env, ls, hcnt, len, k);
      }
      s0 = q;
      k += 1;
      if (done && p.auto_reset) {
        // Env::reset (Env.h:181-187): source reset + fresh Broker; its getData
        // and initialize_history's no-action ticks run as pending ticks
        src_reset<M>(s, p, env, ts);
#pragma unroll
        for (int m = 0; m < M; ++m) {
          s.L[m] = 0.;
          s.mep[m] = 0.;
          s.Bm[m] = 0.;
        }
        cash = p.init_cash;
        if (p.W > 0) {
          len = 0;
          head = p.W - 1;
        }
        pending = p.W > 0 ? p.W : 1;
      }
    } else if (pending > 0) {
      // ---- a reset tick: stream the State (preprocessor.py:172-194)
      if (p.W > 0) {
        ring_push<M, S>(s, p, env, ls, cash, ts, head, len, p.hist ? hcnt : -1);
        if (p.hist) hist_mark(p, env, ls, hcnt, len, k - 1);
      }
      pending -= 1;
      if (pending == 0) s0 = port_sums<M, S>(s.L, s.mep, s.Bm, s.P);
    }
  }

  // ---- write back state
  store_lane<M>(s, p, env);
  if (ls == 0) {
    p.cash[env] = cash;
    p.ts[env] = ts;
    p.dskip[env] = s.dskip;
    if (p.replay) p.rcur[env] = s.rcur;
    p.ep[(size_t)env * 2] = ep_ret;
    p.ep[(size_t)env * 2 + 1] = ep_len;
    if (p.W > 0) {
      p.rhead[env] = head;
      p.rlen[env] = len;
    }
    if constexpr (NST) {
      p.nlen[env] = nlen;
      p.nhead[env] = nhead;
    }
    if (D == 1) {
      p.sA[env] = shA[0];
      p.sB[env] = shB[0];
    }
  }
  if (D != 1) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      if (!s.valid[m]) continue;
      p.sA[(size_t)env * A + s.asset[m]] = shA[m];
      p.sB[(size_t)env * A + s.asset[m]] = shB[m];
    }
  }
}

// Env constructor (mode 0: initMembers + initAccountants) or Env::reset for
// masked envs (mode 1), Env.h:139-187.
template <int M, int S>
__global__ __launch_bounds__(BLOCK) void k_init_reset(KParams p, int mode,
                                                      const uint8_t* __restrict__ mask) {
  constexpr int EPB = BLOCK / S;
  const int tid = threadIdx.x;
  const int ls = tid % S;
  const int env = blockIdx.x * EPB + tid / S;
  if (env >= p.N) return;
  if (mode == 1 && mask && !mask[env]) return;
  Lane<M> s;
  double cash;
  uint64_t ts;
  int32_t head = 0, len = 0;
  if (mode == 0) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const int a = ls * M + m;
      s.asset[m] = a;
      s.valid[m] = a < p.A;
      s.L[m] = s.mep[m] = s.Bm[m] = s.P[m] = s.sx[m] = s.oum[m] = s.dy[m] = 0.;
      s.tlen[m] = 0;
      s.tfl[m] = 0;
      s.kind[m] = s.valid[m] ? p.src[a].kind : -1;
      if (!s.valid[m]) continue;
      const double* q = p.src[a].p;
      const int kd = s.kind[m];
      if (kd == MGN_SRC_SINE || kd == MGN_SRC_SAWTOOTH || kd == MGN_SRC_TRIANGLE) s.sx[m] = q[3];
      else if (kd == MGN_SRC_OU) s.P[m] = q[0];
      else if (kd == MGN_SRC_TRENDOU || kd == MGN_SRC_TRENDYOU) {
        s.P[m] = q[5];
        s.oum[m] = q[5];
      } else if (kd == MGN_SRC_SIMPLETREND) s.P[m] = q[4];
      else if (kd == MGN_SRC_GAUSSIAN) s.P[m] = q[0];
      else if (kd == MGN_SRC_OUPAIR) {
        s.P[m] = 10.;
        s.oum[m] = 10.;
      } else if (kd == MGN_SRC_SINEADDER) {  // DataSource.cpp:645-661: x = phase
        double* ax = p.aux + ((size_t)env * p.A + a) * MGN_AUX_WIDTH;
        const int C = (int)q[0];
        for (int c = 0; c < C; ++c) ax[c] = q[3 + 3 * C + c];
      } else if (kd == MGN_SRC_SINEDYNAMIC || kd == MGN_SRC_SINEDYNTREND) {  // :742-792, :925-992
        double* ax = p.aux + ((size_t)env * p.A + a) * MGN_AUX_WIDTH;
        for (int k = 0; k < MGN_AUX_WIDTH; ++k) ax[k] = 0.;
        sd_sample(p.src_g[a].p, ax, p.seed, (uint64_t)(p.env_offset + env), (uint32_t)a, 0);
        ax[16] = 1.;                                    // trendComponent
        for (int t = 0; t < 2; ++t) ax[18 + 3 * t] = 1.;  // currentDirection
      }
    }
    ts = 0;
    s.dskip = 0;
    cash = p.init_cash;
    // replay: env g starts at tape row (g * stride) mod rows
    s.rcur = p.replay ? (int64_t)(((uint64_t)(p.env_offset + env) * (uint64_t)p.rp_stride) %
                                  (uint64_t)p.rp_rows)
                      : 0;
    s.row = 0;
    gen_tick<M>(s, p, env, ts);  // initAccountants' getData (Env.h:160)
    ts = next_ts<M>(s, p, ts);
    if (ls == 0) {
      p.ep[(size_t)env * 2] = 0.;
      p.ep[(size_t)env * 2 + 1] = 0.;
      for (int f = 0; f < 4; ++f) p.epstats[(size_t)env * 4 + f] = 0.;
      if (p.W > 0) {
        p.rhead[env] = p.W - 1;
        p.rlen[env] = 0;
      }
    }
  } else {
    load_lane<M>(s, p, env, ls);
    cash = p.cash[env];
    ts = p.ts[env];
    s.dskip = p.dskip[env];
    if (p.W > 0) {
      head = p.rhead[env];
      len = p.rlen[env];
    }
    env_reset<M, S>(s, p, env, ls, cash, ts, head, len);
    if (ls == 0 && p.W > 0) {
      p.rhead[env] = head;
      p.rlen[env] = len;
    }
  }
  store_lane<M>(s, p, env);
  if (ls == 0) {
    p.cash[env] = cash;
    p.ts[env] = ts;
    p.dskip[env] = s.dskip;
    if (p.replay) p.rcur[env] = s.rcur;
  }
}

// Portfolio accessors (Portfolio.cpp:170-252) for every env, same canonical
// sums as the step: out (N, 10) = {cash, equity, pnl, balance, availableMargin,
// usedMargin, borrowedMargin, borrowedAssetValue, assetValue, checkRisk}.
template <int M, int S>
__global__ __launch_bounds__(BLOCK) void k_valuation(KParams p, double* __restrict__ out) {
  constexpr int EPB = BLOCK / S;
  const int tid = threadIdx.x;
  const int ls = tid % S;
  const int env = blockIdx.x * EPB + tid / S;
  if (env >= p.N) return;
  Lane<M> s;
  load_lane<M>(s, p, env, ls);
  const double cash = p.cash[env];
  const Sums q = port_sums<M, S>(s.L, s.mep, s.Bm, s.P);
  double tu[M], tb[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    tu[m] = fabs(s.L[m]) * s.mep[m];                       // :199-201
    const double mask = (s.L[m] < 0.) ? 1.0 : 0.0;
    tb[m] = s.L[m] * (s.P[m] * mask);                      // :219-223
  }
  const double used = p.reqM * canon<M, S>(tu);
  const double bav = canon<M, S>(tb);
  if (ls != 0) return;
  const double pnl = q.lp - q.ml;
  const double balance = cash + q.sh;
  double* o = out + (size_t)env * 10;
  o[0] = cash;
  o[1] = (cash + q.lp) - q.b;
  o[2] = pnl;
  o[3] = balance;
  o[4] = (balance + pnl) / p.reqM;
  o[5] = used;
  o[6] = q.b;
  o[7] = bav;
  o[8] = q.lp;
  o[9] = margin_call(q, cash, p.mainM) ? (double)MGN_MARGIN_CALL : (double)MGN_GREEN;
}

}  // namespace mgn
