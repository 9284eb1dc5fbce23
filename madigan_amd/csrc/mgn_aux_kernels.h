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

}  // namespace mgn
