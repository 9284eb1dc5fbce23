// mgn_aux_kernels.h -- non-templated kernels (window ring, action generator);
// included by exactly one translation unit (mgn_api.hip).
#pragma once

#include "mgn_kernels.h"

namespace mgn {

// ---------------------------------------------------------------------------
// Window kernels (StackerDiscrete, preprocessor.py:143-199).  Ring layout
// (N, W, C) with C = F + P columns (price features then portfolio entries).
struct RingDesc {
  int N, F, Pn, W, norm;
  int prelog;  // norm "log" already applied to the price columns at push
  int transform;  // MGN_RING_PAIR_RATIO: pushed price rows have 2 columns, stored p0 / p1
  int ostride, ooff;  // gathered price: row stride and first column in the output
  double* ring;
  uint64_t* ring_ts;
  int32_t* head;
  int32_t* len;
};

// stream_state: one thread per env (rare; the fused step writes its own rows)
__global__ void k_ring_push(RingDesc r, const double* __restrict__ price,
                            const double* __restrict__ port, const uint64_t* __restrict__ ts) {
  const int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= r.N) return;
  const int C = r.F + r.Pn;
  const int h = (r.head[env] + 1) % r.W;
  double* row = r.ring + ((size_t)env * r.W + h) * C;
  if (r.transform == MGN_RING_PAIR_RATIO) {  // (price[:, 0] / price[:, 1]), preprocessor.py:311
    row[0] = price ? price[(size_t)env * 2] / price[(size_t)env * 2 + 1] : 0.;
  } else {
    for (int c = 0; c < r.F; ++c) {
      const double v = price ? price[(size_t)env * r.F + c] : 0.;
      row[c] = r.prelog ? log_norm(v) : v;
    }
  }
  for (int c = 0; c < r.Pn; ++c) row[r.F + c] = port ? port[(size_t)env * r.Pn + c] : 0.;
  r.ring_ts[(size_t)env * r.W + h] = ts ? ts[env] : 0;
  r.head[env] = h;
  if (r.len[env] < r.W) r.len[env] += 1;
}

__global__ void k_ring_clear(RingDesc r, const uint8_t* __restrict__ mask) {
  const int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= r.N) return;
  if (mask && !mask[env]) return;
  r.head[env] = r.W - 1;
  r.len[env] = 0;
}

// current_data: one thread per (env, column); rows oldest -> newest, norm on
// price columns (log_norm :79-81, lookback :63-66, standard_norm :83-92,
// log_standard_norm :95-107: log without the clamp, nan-skipping mean / std).
__device__ __forceinline__ double nan_to_num(double v) {
  if (v != v) return 0.;
  if (v == __builtin_inf()) return 1.7976931348623157e308;
  if (v == -__builtin_inf()) return -1.7976931348623157e308;
  return v;
}

__global__ __launch_bounds__(BLOCK) void k_ring_gather(RingDesc r, double* __restrict__ price_out,
                                                       double* __restrict__ port_out,
                                                       uint64_t* __restrict__ ts_out) {
  const int C = r.F + r.Pn;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (int64_t)r.N * C) return;
  const int env = (int)(gid / C);
  const int c = (int)(gid % C);
  const int W = r.W;
  const int len = r.len[env];
  const int hd = r.head[env];
  const double* base = r.ring + (size_t)env * W * C;
  auto row_of = [&](int w) { return (hd - (len - 1) + w + 2 * W) % W; };
  if (c >= r.F) {
    const int pc = c - r.F;
    if (port_out)
      for (int w = 0; w < W; ++w)
        port_out[((size_t)env * W + w) * r.Pn + pc] = (w < len) ? base[(size_t)row_of(w) * C + c] : 0.;
    return;
  }
  if (c == 0 && ts_out)
    for (int w = 0; w < W; ++w)
      ts_out[(size_t)env * W + w] = (w < len) ? r.ring_ts[(size_t)env * W + row_of(w)] : 0;
  if (!price_out) return;
  double* o = price_out + (size_t)env * W * r.ostride + r.ooff + c;
  const int nt = r.norm;
  if (nt == MGN_NORM_LOG_STANDARD_NORMAL) {
    // np.nanmean / np.nanstd over the window of log(x); log of x <= 0 is nan / -inf
    double sum = 0.;
    int cnt = 0;
    for (int w = 0; w < len; ++w) {
      const double x = log(base[(size_t)row_of(w) * C + c]);
      if (x == x) { sum += x; cnt += 1; }
    }
    const double mean = sum / cnt;
    double ss = 0.;
    for (int w = 0; w < len; ++w) {
      const double x = log(base[(size_t)row_of(w) * C + c]);
      if (x == x) { const double d = x - mean; ss += d * d; }
    }
    const double sd = sqrt(ss / cnt);
    for (int w = 0; w < W; ++w) {
      const double x = (w < len) ? log(base[(size_t)row_of(w) * C + c]) : 0.;
      o[(size_t)w * r.ostride] = (w < len) ? nan_to_num((x - mean) / sd) : 0.;
    }
    return;
  }
  if (nt == MGN_NORM_STANDARD_NORMAL) {
    double sum = 0.;
    for (int w = 0; w < len; ++w) sum += base[(size_t)row_of(w) * C + c];
    const double mean = sum / len;
    double ss = 0.;
    for (int w = 0; w < len; ++w) {
      const double d = base[(size_t)row_of(w) * C + c] - mean;
      ss += d * d;
    }
    const double sd = sqrt(ss / len);
    for (int w = 0; w < W; ++w) {
      double v = 0.;
      if (w < len) v = nan_to_num((base[(size_t)row_of(w) * C + c] - mean) / sd);
      o[(size_t)w * r.ostride] = v;
    }
    return;
  }
  const double last = (len > 0) ? base[(size_t)row_of(len - 1) * C + c] : 1.;
  for (int w = 0; w < W; ++w) {
    double v = 0.;
    if (w < len) {
      v = base[(size_t)row_of(w) * C + c];
      if (nt == MGN_NORM_LOG && !r.prelog) v = log((v < 1e-5) ? 1e-5 : v);
      else if (nt == MGN_NORM_LOOKBACK) v = v / last;
      else if (nt == MGN_NORM_LOOKBACK_LOG) v = log(v / last);
    }
    o[(size_t)w * r.ostride] = v;
  }
}

// current_data for the element-wise normalisers (none / log / lookback /
// lookback_log), in the ring's physical order: the ring of all envs is one
// contiguous array (N, W, C), so lane t of the grid reads 16 B pairs
// 2t, 2t+1 (W even: a pair never straddles two envs), fully coalesced, and
// scatters each element to its logical window row w = (row - head + len - 1)
// mod W of the price (c < F) or portfolio (c >= F) output; rows w >= len are
// written as zeros.  Index math is 32-bit with reciprocal division (exact
// after one correction step).  HBM-bound: per env read W*(C+1)*8 B (ring +
// timestamps), write W*(C+1)*8 B.
__device__ __forceinline__ void divmod_u32(uint32_t n, uint32_t d, double inv, uint32_t& q,
                                           uint32_t& r) {
  q = (uint32_t)((double)n * inv);
  int32_t rr = (int32_t)(n - q * d);
  if (rr < 0) { q -= 1; rr += (int32_t)d; }
  else if (rr >= (int32_t)d) { q += 1; rr -= (int32_t)d; }
  r = (uint32_t)rr;
}

constexpr int GATHER_U = 4;  // 16-B pairs per lane per pass

__global__ __launch_bounds__(BLOCK) void k_ring_gather_elem(RingDesc r, double* __restrict__ price_out,
                                                            double* __restrict__ port_out,
                                                            uint64_t* __restrict__ ts_out,
                                                            uint32_t n_pairs, double inv_wc,
                                                            double inv_c) {
  const int C = r.F + r.Pn;
  const uint32_t WC = (uint32_t)(r.W * C);
  const int W = r.W;
  const d2* src = reinterpret_cast<const d2*>(r.ring);
  const uint32_t p0 = blockIdx.x * (BLOCK * GATHER_U) + threadIdx.x;
  d2 v[GATHER_U];
#pragma unroll
  for (int u = 0; u < GATHER_U; ++u) {
    const uint32_t pi = p0 + u * BLOCK;
    if (pi < n_pairs) v[u] = src[pi];
  }
#pragma unroll
  for (int u = 0; u < GATHER_U; ++u) {
    const uint32_t pi = p0 + u * BLOCK;
    if (pi >= n_pairs) continue;
    uint32_t env, rem, pr, c;
    divmod_u32(2 * pi, WC, inv_wc, env, rem);
    divmod_u32(rem, (uint32_t)C, inv_c, pr, c);
    const int len = r.len[env];
    const int hd = r.head[env];
    const double* base = r.ring + (size_t)env * WC;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      double x = h ? v[u].y : v[u].x;
      const int w = ((int)pr - hd + len - 1 + 2 * W) % W;
      const bool valid = w < len;
      if (!valid) x = 0.;
      if ((int)c >= r.F) {
        if (port_out) port_out[((size_t)env * W + w) * r.Pn + ((int)c - r.F)] = x;
      } else {
        if (c == 0 && ts_out) ts_out[(size_t)env * W + w] = valid ? r.ring_ts[(size_t)env * W + pr] : 0;
        if (price_out) {
          if (valid) {
            const int nt = r.norm;
            if (nt == MGN_NORM_LOG && !r.prelog) {
              x = log((x < 1e-5) ? 1e-5 : x);
            } else if (nt == MGN_NORM_LOOKBACK || nt == MGN_NORM_LOOKBACK_LOG) {
              x = x / base[(size_t)hd * C + c];
              if (nt == MGN_NORM_LOOKBACK_LOG) x = log(x);
            }
          }
          price_out[((size_t)env * W + w) * r.F + c] = x;
        }
      }
      // the pair's second element: next column, or column 0 of the next row
      if (++c == (uint32_t)C) {
        c = 0;
        ++pr;
      }
    }
  }
}

// current_data for the element-wise normalisers, LDS-staged: a workgroup owns
// `epb` consecutive envs, whose ring rows (epb, W, C) and timestamps (epb, W)
// are one contiguous range of the arena each, and whose outputs price
// (epb, W, F), portfolio (epb, W, P) and timestamps (epb, W) are contiguous
// too.  Phase 1 copies the ring range into LDS with 16-B loads (U in flight
// per lane); phase 2 walks the three outputs in 16-B pairs, each element read
// from LDS at its logical row (head - len + 1 + w) mod W, normalised, and
// stored coalesced.  Every HBM byte is read once and written once with full
// 16-B accesses.  Local indices are < 2^24, so the divisions are one fp32
// reciprocal multiply plus a correction.
__device__ __forceinline__ void divmod_small(uint32_t n, uint32_t d, float inv, uint32_t& q,
                                             uint32_t& r) {
  q = (uint32_t)((float)n * inv);
  int32_t rr = (int32_t)(n - q * d);
  while (rr < 0) { q -= 1; rr += (int32_t)d; }
  while (rr >= (int32_t)d) { q += 1; rr -= (int32_t)d; }
  r = (uint32_t)rr;
}

struct GatherLds {
  int epb;                        // envs per workgroup
  float inv_f, inv_p, inv_w;      // 1/F, 1/P, 1/W
};

__global__ __launch_bounds__(BLOCK) void k_ring_gather_lds(RingDesc r, double* __restrict__ price_out,
                                                           double* __restrict__ port_out,
                                                           uint64_t* __restrict__ ts_out,
                                                           GatherLds g) {
  extern __shared__ d2 s_buf[];
  const int F = r.F, P = r.Pn, W = r.W, C = F + P;
  const int env0 = blockIdx.x * g.epb;
  const int ne = min(g.epb, r.N - env0);
  const int ring_pairs = ne * W * C / 2;   // W even: whole pairs
  const int ts_pairs = ne * W / 2;
  d2* s_ring = s_buf;
  d2* s_ts = s_buf + g.epb * W * C / 2;
  __shared__ int s_hd[64], s_len[64];
  if (threadIdx.x < ne) {
    s_hd[threadIdx.x] = r.head[env0 + threadIdx.x];
    s_len[threadIdx.x] = r.len[env0 + threadIdx.x];
  }
  {
    const d2* gr = reinterpret_cast<const d2*>(r.ring + (size_t)env0 * W * C);
    const d2* gt = reinterpret_cast<const d2*>(r.ring_ts + (size_t)env0 * W);
    const int total = ring_pairs + (ts_out ? ts_pairs : 0);
    constexpr int U = 4;
    for (int i0 = threadIdx.x; i0 < total; i0 += U * BLOCK) {
      d2 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * BLOCK;
        if (i < ring_pairs) v[u] = __builtin_nontemporal_load(gr + i);
        else if (i < total) v[u] = __builtin_nontemporal_load(gt + (i - ring_pairs));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * BLOCK;
        if (i < ring_pairs) s_ring[i] = v[u];
        else if (i < total) s_ts[i - ring_pairs] = v[u];
      }
    }
  }
  __syncthreads();
  const double* sr = reinterpret_cast<const double*>(s_ring);
  const int nt = r.norm;
  // one element of the logical window: env-local row R = e*W + w, column c
  auto elem = [&](uint32_t R, int c, bool is_price) -> double {
    uint32_t e, w;
    divmod_small(R, (uint32_t)W, g.inv_w, e, w);
    const int len = s_len[e], hd = s_hd[e];
    if ((int)w >= len) return 0.;
    int row = hd - len + 1 + (int)w;
    if (row < 0) row += W;
    const double* base = sr + (size_t)e * W * C;
    double x = base[row * C + c];
    if (is_price) {
      if (nt == MGN_NORM_LOG && !r.prelog) {
        x = log((x < 1e-5) ? 1e-5 : x);
      } else if (nt == MGN_NORM_LOOKBACK || nt == MGN_NORM_LOOKBACK_LOG) {
        x = x / base[hd * C + c];
        if (nt == MGN_NORM_LOOKBACK_LOG) x = log(x);
      }
    }
    return x;
  };
  if (price_out) {
    d2* o = reinterpret_cast<d2*>(price_out + (size_t)env0 * W * F);
    const int n = ne * W * F / 2;
    for (int q = threadIdx.x; q < n; q += BLOCK) {
      uint32_t R, c;
      divmod_small(2u * q, (uint32_t)F, g.inv_f, R, c);
      d2 v;
      v.x = elem(R, (int)c, true);
      if (++c == (uint32_t)F) { c = 0; ++R; }
      v.y = elem(R, (int)c, true);
      __builtin_nontemporal_store(v, o + q);
    }
  }
  if (port_out) {
    d2* o = reinterpret_cast<d2*>(port_out + (size_t)env0 * W * P);
    const int n = ne * W * P / 2;
    for (int q = threadIdx.x; q < n; q += BLOCK) {
      uint32_t R, c;
      divmod_small(2u * q, (uint32_t)P, g.inv_p, R, c);
      d2 v;
      v.x = elem(R, F + (int)c, false);
      if (++c == (uint32_t)P) { c = 0; ++R; }
      v.y = elem(R, F + (int)c, false);
      __builtin_nontemporal_store(v, o + q);
    }
  }
  if (ts_out) {
    const uint64_t* st = reinterpret_cast<const uint64_t*>(s_ts);
    ulong2* o = reinterpret_cast<ulong2*>(ts_out + (size_t)env0 * W);
    for (int q = threadIdx.x; q < ts_pairs; q += BLOCK) {
      uint64_t t[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        uint32_t e, w;
        divmod_small(2u * q + h, (uint32_t)W, g.inv_w, e, w);
        const int len = s_len[e], hd = s_hd[e];
        int row = hd - len + 1 + (int)w;
        if (row < 0) row += W;
        t[h] = ((int)w < len) ? st[e * W + row] : 0;
      }
      o[q] = make_ulong2(t[0], t[1]);
    }
  }
}

// ---------------------------------------------------------------------------
// Launch history (mgn_rollout_hist / mgn_window_hist): K steps in one launch
// with every step's window.  The step kernel appends each ring push to a
// linear per-env history, so step k's window is the contiguous row range
// [hend - hlen, hend) -- no modulo, no rotation.  Sized W + K*(W+1) rows per
// env (each step pushes one row, plus W refill rows when it ends an episode).
struct HistDesc {
  int N, F, Pn, W, K, hrows, norm, prelog;
  const double* hist;
  const uint64_t* hist_ts;
  const int32_t* hend;
  const int32_t* hlen;
};

// rows [W - len, W) of every env's history := its ring window, oldest first.
// A workgroup per env: the window is at most two contiguous runs of the ring
// (before and after the wrap), so the copy is two coalesced streams, no
// per-element division.
__global__ __launch_bounds__(BLOCK) void k_hist_prefix(RingDesc r, double* __restrict__ hist,
                                                       uint64_t* __restrict__ hist_ts, int hrows) {
  const int C = r.F + r.Pn, W = r.W;
  const int env = blockIdx.x;
  const int len = r.len[env];
  if (len <= 0) return;
  const int first = (r.head[env] - len + 1 + W) % W;  // oldest row
  const int nA = min(len, W - first);                 // rows before the wrap
  const double* src = r.ring + (size_t)env * W * C;
  double* dst = hist + ((size_t)env * hrows + (W - len)) * C;
  const int n = len * C, na = nA * C;
  for (int i = threadIdx.x; i < n; i += BLOCK)
    dst[i] = (i < na) ? src[first * C + i] : src[i - na];
  const uint64_t* tsrc = r.ring_ts + (size_t)env * W;
  uint64_t* tdst = hist_ts + (size_t)env * hrows + (W - len);
  for (int i = threadIdx.x; i < len; i += BLOCK) tdst[i] = (i < nA) ? tsrc[first + i] : tsrc[i - nA];
}

// every step's StackerDiscrete.current_data: a workgroup per (env, ks
// consecutive steps) writes those windows (outputs (K,N,W,F), (K,N,W,P), (K,N,W); element-wise normalisers as
// k_ring_gather_elem).  The history rows the K windows span, [hend[0] -
// hlen[0], hend[K-1]), are staged once into LDS (they are shared by
// consecutive windows: W + K rows when no episode ends), so HBM sees each row
// read once and every output byte written once with 16-B stores; a span
// larger than the LDS budget reads the history directly (L2-resident within
// the workgroup).  Splitting an env's K windows over workgroups of ks keeps
// the grid fine-grained (no tail of a few long workgroups); mgn_window_hist
// sizes ks so that a workgroup still writes >= 80 KB (its two dependent
// memory round trips amortised: narrow rows take more steps per workgroup).
constexpr int HIST_KMAX = 64;

__global__ __launch_bounds__(BLOCK) void k_hist_gather(HistDesc h, double* __restrict__ price_out,
                                                       double* __restrict__ port_out,
                                                       uint64_t* __restrict__ ts_out, int ks, int lds_rows,
                                                       float inv_f, float inv_p, float inv_w,
                                                       float inv_wf, float inv_wp) {
  extern __shared__ double s_rows[];  // (lds_rows, C) then lds_rows timestamps
  const int F = h.F, P = h.Pn, W = h.W, C = F + P;
  // workgroup: env, steps [k0, k0 + K) of the launch (ks steps per workgroup)
  const int kb = (h.K + ks - 1) / ks;
  const int env = blockIdx.x / kb;
  const int k0 = (blockIdx.x - env * kb) * ks;
  const int K = min(ks, h.K - k0);
  __shared__ int s_start[HIST_KMAX], s_len[HIST_KMAX];
  if (threadIdx.x < K) {
    const size_t t = (size_t)(k0 + threadIdx.x) * h.N + env;
    s_start[threadIdx.x] = h.hend[t] - h.hlen[t];
    s_len[threadIdx.x] = h.hlen[t];
  }
  __syncthreads();
  const int r0 = s_start[0];
  const int r1 = s_start[K - 1] + s_len[K - 1];
  const int nrows = r1 - r0;
  const bool staged = nrows <= lds_rows;
  const double* grow = h.hist + ((size_t)env * h.hrows + r0) * C;  // row r0 of this env
  const uint64_t* gts = h.hist_ts + (size_t)env * h.hrows + r0;
  uint64_t* s_ts = reinterpret_cast<uint64_t*>(s_rows + (size_t)lds_rows * C);
  if (staged) {
    constexpr int U = 8;
    const int n = nrows * C;
    for (int i0 = threadIdx.x; i0 < n; i0 += U * BLOCK) {
      double v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = (i0 + u * BLOCK < n) ? grow[i0 + u * BLOCK] : 0.;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (i0 + u * BLOCK < n) s_rows[i0 + u * BLOCK] = v[u];
    }
    if (ts_out)
      for (int i = threadIdx.x; i < nrows; i += BLOCK) s_ts[i] = gts[i];
    __syncthreads();
  }
  const double* rows = staged ? s_rows : grow;
  const int nt = h.norm;
  auto block_out = [&](double* __restrict__ out_base, int ncol, int col0, float inv_n, float inv_wn,
                       bool is_price) {
    const uint32_t WN = (uint32_t)(W * ncol);
    const int n = K * W * ncol / 2;  // pairs (W even: never across windows)
    for (int q = threadIdx.x; q < n; q += BLOCK) {
      uint32_t k, rem, w, c;
      divmod_small(2u * q, WN, inv_wn, k, rem);
      divmod_small(rem, (uint32_t)ncol, inv_n, w, c);
      const int len = s_len[k];
      const int rs = s_start[k] - r0;
      d2 v;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        double x = 0.;
        if ((int)w < len) {
          x = rows[(rs + (int)w) * C + col0 + (int)c];
          if (is_price) {
            if (nt == MGN_NORM_LOG && !h.prelog) {
              x = log((x < 1e-5) ? 1e-5 : x);
            } else if (nt == MGN_NORM_LOOKBACK || nt == MGN_NORM_LOOKBACK_LOG) {
              x = x / rows[(rs + len - 1) * C + col0 + (int)c];
              if (nt == MGN_NORM_LOOKBACK_LOG) x = log(x);
            }
          }
        }
        if (hh) v.y = x; else v.x = x;
        if (++c == (uint32_t)ncol) { c = 0; ++w; }
      }
      d2* o = reinterpret_cast<d2*>(out_base + ((size_t)(k0 + k) * h.N + env) * WN);
      __builtin_nontemporal_store(v, o + (rem >> 1));
    }
  };
  if (price_out) block_out(price_out, F, 0, inv_f, inv_wf, true);
  if (port_out) block_out(port_out, P, F, inv_p, inv_wp, false);
  if (ts_out) {
    const uint64_t* tsrc = staged ? s_ts : gts;
    const int n = K * W / 2;
    for (int q = threadIdx.x; q < n; q += BLOCK) {
      uint32_t k, w;
      divmod_small(2u * q, (uint32_t)W, inv_w, k, w);
      const int len = s_len[k];
      const int rs = s_start[k] - r0;
      const uint64_t a = ((int)w < len) ? tsrc[rs + (int)w] : 0;
      const uint64_t b = ((int)w + 1 < len) ? tsrc[rs + (int)w + 1] : 0;
      ulong2* o = reinterpret_cast<ulong2*>(ts_out + ((size_t)(k0 + k) * h.N + env) * W);
      o[w >> 1] = make_ulong2(a, b);
    }
  }
}

// StackerDiscreteReturns' np.diff along the last axis: out (rows, cols-1)
__global__ __launch_bounds__(BLOCK) void k_feat_diff(const double* __restrict__ in,
                                                     double* __restrict__ out, int64_t rows,
                                                     int cols) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int co = cols - 1;
  if (gid >= rows * co) return;
  const int64_t rw = gid / co;
  const int c = (int)(gid % co);
  out[gid] = in[rw * cols + c + 1] - in[rw * cols + c];
}

// Philox discrete actions U{0..atoms-1}: counter (k, env, asset, 0xAC7)
__global__ void k_gen_actions(int8_t* __restrict__ out, int K, int N, int A, int atoms,
                              uint64_t seed, int64_t env_offset) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)K * N * A;
  if (gid >= total) return;
  const int a = (int)(gid % A);
  const int64_t ke = gid / A;
  const int env = (int)(ke % N);
  const uint32_t k = (uint32_t)(ke / N);
  const u4 x = philox4x32_10(k, (uint32_t)(env_offset + env), (uint32_t)a, 0xAC7u, (uint32_t)seed,
                             (uint32_t)(seed >> 32));
  out[gid] = (int8_t)(((uint64_t)x.x * (uint32_t)atoms) >> 32);
}

// Attainable-bandwidth probe ("measure attainable bandwidth on
// the box with a device-copy kernel"): a grid-stride 16-B-per-lane copy,
// 4 loads in flight per lane, non-temporal stores
typedef double probe_v2 __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ void probe_st(probe_v2* q, probe_v2 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, q);
  else *q = v;
}
// ONESHOT: one U x 4-KiB chunk per workgroup (U x 16 B per lane, each
// coalesced), grid = bytes / chunk; else a grid-stride loop over 16 waves per
// CU with 4 loads in flight.  NT: nontemporal stores.
template <bool NT, bool ONESHOT, int U = 4>
__global__ __launch_bounds__(BLOCK) void k_copy_probe(const probe_v2* __restrict__ src,
                                                      probe_v2* __restrict__ dst, int64_t n) {
  if constexpr (ONESHOT) {
    const int64_t base = (int64_t)blockIdx.x * (U * BLOCK) + threadIdx.x;
    if (base + (U - 1) * BLOCK < n) {
      probe_v2 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = src[base + u * BLOCK];
#pragma unroll
      for (int u = 0; u < U; ++u) probe_st<NT>(dst + base + u * BLOCK, v[u]);
    } else {
      for (int u = 0; u < U; ++u)
        if (base + u * BLOCK < n) probe_st<NT>(dst + base + u * BLOCK, src[base + u * BLOCK]);
    }
  } else {
    const int64_t stride = (int64_t)gridDim.x * BLOCK;
    int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
      const probe_v2 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
      probe_st<NT>(dst + i, a);
      probe_st<NT>(dst + i + stride, b);
      probe_st<NT>(dst + i + 2 * stride, c);
      probe_st<NT>(dst + i + 3 * stride, d);
    }
    for (; i < n; i += stride) probe_st<NT>(dst + i, src[i]);
  }
}

// ---------------------------------------------------------------------------
// Broker / Portfolio operations outside a step (the drop-in's env.broker and
// env.portfolio objects): no tick, no reward, only the ledger and the
// responses.  One thread per env; the assets in the reference's serial order,
// every risk check re-evaluating the canonical sums from the current ledger
// (Portfolio.cpp:170-279), as the step kernels' serial form does.  Off the
// step path (one call per Python-level Broker / Portfolio method).
struct LedgerOp {
  int op;  // MGN_OP_*
  const int32_t* aidx;   // (N) asset index (single-asset ops)
  const double* units;   // (N, A) BROKER_UNITS, else (N)
  const double* tprice;  // (N) PORT_TXN / PORT_CLOSE transaction price
  const double* tcost;   // (N) PORT_TXN / PORT_CLOSE transaction cost
  double *o_tp, *o_tu, *o_tc;  // responses: (N, A) BROKER_UNITS, else (N)
  uint8_t *o_risk, *o_mc;      // risk (N, A) / (N); marginCall (N)
};

// the canonical pairwise tree of v[0..A) padded with +0.0 to APAD
__device__ double lop_canon(const double* v, int A, int apad) {
  double t[MGN_MAX_ASSETS];
  for (int i = 0; i < apad; ++i) t[i] = i < A ? v[i] : 0.0;
  for (int w = apad; w > 1; w >>= 1)
    for (int i = 0; i < w / 2; ++i) t[i] = t[2 * i] + t[2 * i + 1];
  return t[0];
}
__device__ Sums lop_sums(const double* L, const double* mep, const double* Bm, const double* P, int A,
                         int apad) {
  double a[MGN_MAX_ASSETS], b[MGN_MAX_ASSETS], c[MGN_MAX_ASSETS];
  for (int i = 0; i < A; ++i) {
    a[i] = L[i] * P[i];
    b[i] = mep[i] * L[i];
    const double mask = (L[i] < 0.) ? 1.0 : 0.0;
    c[i] = L[i] * (mep[i] * mask);
  }
  Sums s;
  s.lp = lop_canon(a, A, apad);
  s.ml = lop_canon(b, A, apad);
  s.sh = lop_canon(c, A, apad);
  s.b = lop_canon(Bm, A, apad);
  return s;
}
// Portfolio::checkRisk(assetIdx, units), Portfolio.cpp:254-279
__device__ int lop_check_order(const KParams& p, const double* L, const double* mep, const double* Bm,
                               const double* P, double cash, int A, int apad, int i, double u) {
  const Sums q = lop_sums(L, mep, Bm, P, A, apad);
  const double pnl = q.lp - q.ml;
  const double balance = cash + q.sh;
  const double availM = (balance + pnl) / p.reqM;
  const double cur = L[i];
  if (signbit(u) != signbit(cur)) {
    if (u > -1 * cur) {
      const double excess = u + cur;
      if (availM <= fabs(P[i] * excess) || balance <= 0.) return MGN_INSUFF_MARGIN;
    }
    return MGN_GREEN;
  }
  if (margin_call(q, cash, p.mainM)) return MGN_MARGIN_CALL;
  if (availM <= fabs(P[i] * u) || balance <= 0.) return MGN_INSUFF_MARGIN;
  return MGN_GREEN;
}
// Portfolio::handleTransaction, Portfolio.cpp:284-323
__device__ void lop_txn(const KParams& p, double* L, double* mep, double* Bm, double& cash, int i,
                        double tp, double u, double cost) {
  double& cur = L[i];
  double& me = mep[i];
  if (signbit(cur) != signbit(u)) {
    if (fabs(u) > fabs(cur)) {
      u += cur;
      cash += cur * tp;
      cur = 0.;
      me = tp;
    }
  } else {
    me += (tp - me) * (u / (u + cur));
  }
  const double amt = tp * u;
  const double use = amt * p.reqM;
  const double brw = amt - use;
  Bm[i] += brw;
  cash -= (use + cost);
  cur += u;
  if (fabs(cur) < 0.000001) {
    me = 0.;
    if (Bm[i] > 0.) {
      cash -= Bm[i];
      Bm[i] = 0.;
    }
  }
  if (Bm[i] < 0.) {
    cash -= Bm[i];
    Bm[i] = 0.;
  }
}
// Broker::applySlippage / getTransactionCost (Broker.cpp:171-178)
__device__ double lop_slip(const KParams& p, double price, double u) {
  const double slippage = (price * p.slip_rel) + p.slip_abs;
  return u < 0 ? (price - slippage) : (price + slippage);
}
__device__ double lop_cost(const KParams& p, double amount) { return fabs(amount) * p.tc_rel + p.tc_abs; }

__global__ __launch_bounds__(BLOCK) void k_ledger_op(KParams p, LedgerOp o) {
  const int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= p.N) return;
  const int A = p.A;
  int apad = 1;
  while (apad < A) apad <<= 1;
  double L[MGN_MAX_ASSETS], mep[MGN_MAX_ASSETS], Bm[MGN_MAX_ASSETS], P[MGN_MAX_ASSETS];
  const size_t b = (size_t)env * A;
  for (int i = 0; i < A; ++i) {
    L[i] = p.L[b + i];
    mep[i] = p.mep[b + i];
    Bm[i] = p.Bm[b + i];
    P[i] = p.P[b + i];
  }
  double cash = p.cash[env];
  if (o.op != MGN_OP_BROKER_UNITS && (o.aidx[env] < 0 || o.aidx[env] >= A)) {
    // an asset index out of range (the Python layer raises IndexError first,
    // as the reference's std::out_of_range): the env is left untouched, its
    // response zero with risk code 0xFF
    if (o.op != MGN_OP_PORT_TXN && o.op != MGN_OP_PORT_CLOSE) {
      if (o.o_tp) o.o_tp[env] = 0.;
      if (o.o_tu) o.o_tu[env] = 0.;
      if (o.o_tc) o.o_tc[env] = 0.;
      if (o.o_risk) o.o_risk[env] = (uint8_t)0xFF;
    }
    if (o.o_mc) o.o_mc[env] = 0;
    return;
  }
  if (o.op == MGN_OP_BROKER_UNITS) {
    // Broker::handleTransaction(port, units), Broker.cpp:144-158
    for (int i = 0; i < A; ++i) {
      const double u = o.units[b + i];
      double tp = 0., tu = 0., tc = 0.;
      int risk = MGN_GREEN;
      if (u != 0.) {
        risk = lop_check_order(p, L, mep, Bm, P, cash, A, apad, i, u);
        if (risk == MGN_GREEN) {
          tp = lop_slip(p, P[i], u);
          tc = lop_cost(p, u * P[i]);
          tu = u;
          lop_txn(p, L, mep, Bm, cash, i, tp, u, tc);
        }
      }
      if (o.o_tp) o.o_tp[b + i] = tp;
      if (o.o_tu) o.o_tu[b + i] = tu;
      if (o.o_tc) o.o_tc[b + i] = tc;
      if (o.o_risk) o.o_risk[b + i] = (uint8_t)risk;
    }
  } else if (o.op == MGN_OP_BROKER_SINGLE || o.op == MGN_OP_CHECK_ORDER) {
    // Broker::handleTransaction(port, assetIdx, units), Broker.cpp:124-142;
    // CHECK_ORDER: Portfolio::checkRisk(assetIdx, units) alone
    const int i = o.aidx[env];
    const double u = o.units[env];
    double tp = 0., tu = 0., tc = 0.;
    int risk = MGN_GREEN;
    if (o.op == MGN_OP_CHECK_ORDER) {
      risk = lop_check_order(p, L, mep, Bm, P, cash, A, apad, i, u);
    } else if (u != 0.) {
      risk = lop_check_order(p, L, mep, Bm, P, cash, A, apad, i, u);
      if (risk == MGN_GREEN) {
        tp = lop_slip(p, P[i], u);
        tc = lop_cost(p, u * P[i]);
        tu = u;
        lop_txn(p, L, mep, Bm, cash, i, tp, u, tc);
      }
    }
    if (o.o_tp) o.o_tp[env] = tp;
    if (o.o_tu) o.o_tu[env] = tu;
    if (o.o_tc) o.o_tc[env] = tc;
    if (o.o_risk) o.o_risk[env] = (uint8_t)risk;
  } else if (o.op == MGN_OP_BROKER_CLOSE) {
    // Broker::close(assetIdx), Broker.cpp:160-169: units = -ledger, slippage and
    // cost as an order, Portfolio::close, always green
    const int i = o.aidx[env];
    const double u = -(L[i]);
    const double tp = lop_slip(p, P[i], u);
    const double tc = lop_cost(p, P[i] * u);
    if (L[i] != 0.) lop_txn(p, L, mep, Bm, cash, i, tp, -1 * L[i], tc);  // Portfolio.cpp:327-333
    if (o.o_tp) o.o_tp[env] = tp;
    if (o.o_tu) o.o_tu[env] = u;
    if (o.o_tc) o.o_tc[env] = tc;
    if (o.o_risk) o.o_risk[env] = (uint8_t)MGN_GREEN;
  } else if (o.op == MGN_OP_PORT_TXN) {
    // Portfolio::handleTransaction(assetIdx, transactionPrice, units, cost)
    lop_txn(p, L, mep, Bm, cash, o.aidx[env], o.tprice[env], o.units[env], o.tcost ? o.tcost[env] : 0.);
  } else if (o.op == MGN_OP_PORT_CLOSE) {
    // Portfolio::close(assetIdx, transactionPrice, cost), Portfolio.cpp:327-333
    const int i = o.aidx[env];
    if (L[i] != 0.) lop_txn(p, L, mep, Bm, cash, i, o.tprice[env], -1 * L[i], o.tcost ? o.tcost[env] : 0.);
  }
  if (o.o_mc) o.o_mc[env] = margin_call(lop_sums(L, mep, Bm, P, A, apad), cash, p.mainM) ? 1 : 0;
  if (o.op == MGN_OP_CHECK_ORDER) return;
  for (int i = 0; i < A; ++i) {
    p.L[b + i] = L[i];
    p.mep[b + i] = mep[i];
    p.Bm[b + i] = Bm[i];
  }
  p.cash[env] = cash;
}

}  // namespace mgn
