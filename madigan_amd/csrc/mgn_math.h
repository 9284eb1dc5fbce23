// mgn_math.h -- device-side RNG and deterministic math for the generators.
//
// The reference draws its noise from std::default_random_engine seeded with
// the wall clock (madigan/environments/cpp/DataSource.cpp:472, :1131, :1407),
// so its streams cannot be replayed.  This framework's variates are a fixed
// specification instead: Philox4x32-10 keyed by (seed), counter
// (tick, env, asset|slot<<16), Box-Muller (53-bit radius, 32-bit angle), with fdlibm's
// log/sin/cos kernels evaluated in plain IEEE binary64 (compiled with
// -ffp-contract=off) so every host restatement reproduces the device bits.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mgn {

__device__ __forceinline__ double bits_to_d(uint64_t u) { return __longlong_as_double((long long)u); }
__device__ __forceinline__ uint64_t d_to_bits(double d) { return (uint64_t)__double_as_longlong(d); }

struct u4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                            uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one v_mad_u64_u32 per product gives both halves
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return u4{c0, c1, c2, c3};
}

__device__ __forceinline__ u4 block(uint64_t seed, uint64_t env, uint32_t asset, uint32_t slot,
                                    uint64_t tick) {
  return philox4x32_10((uint32_t)tick, (uint32_t)env, asset | (slot << 16),
                       (uint32_t)(tick >> 32) ^ (uint32_t)(env >> 32), (uint32_t)seed,
                       (uint32_t)(seed >> 32));
}

// two 53-bit integers from one Philox block
__device__ __forceinline__ void draw53(uint64_t seed, uint64_t env, uint32_t asset, uint32_t slot,
                                       uint64_t tick, uint64_t& a, uint64_t& b) {
  const u4 x = block(seed, env, asset, slot, tick);
  a = (((uint64_t)x.y << 32) | x.x) >> 11;
  b = (((uint64_t)x.w << 32) | x.z) >> 11;
}

constexpr double TWO_M53 = 1.1102230246251565404e-16;

__device__ __forceinline__ void uniform2(uint64_t seed, uint64_t env, uint32_t asset,
                                         uint32_t slot, uint64_t tick, double& u0, double& u1) {
  uint64_t a, b;
  draw53(seed, env, asset, slot, tick, a, b);
  u0 = (double)a * TWO_M53;
  u1 = (double)b * TWO_M53;
}

// fdlibm e_log.c, normal positive arguments
__device__ __forceinline__ double det_log(double x) {
  const double ln2_hi = bits_to_d(0x3fe62e42fee00000ull);
  const double ln2_lo = bits_to_d(0x3dea39ef35793c76ull);
  const double Lg1 = bits_to_d(0x3FE5555555555593ull), Lg2 = bits_to_d(0x3FD999999997FA04ull),
               Lg3 = bits_to_d(0x3FD2492494229359ull), Lg4 = bits_to_d(0x3FCC71C51D8E78AFull),
               Lg5 = bits_to_d(0x3FC7466496CB03DEull), Lg6 = bits_to_d(0x3FC39A09D078C69Full),
               Lg7 = bits_to_d(0x3FC2F112DF3E5244ull);
  const uint64_t ix = d_to_bits(x);
  int32_t hx = (int32_t)(ix >> 32);
  int32_t k = ((hx >> 20) & 0x7ff) - 1023;
  hx &= 0x000fffff;
  const int32_t i = (hx + 0x95f64) & 0x100000;
  k += (i >> 20);
  const uint64_t mb = ((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (ix & 0xffffffffull);
  const double f = bits_to_d(mb) - 1.0;
  const double s = f / (2.0 + f);
  const double dk = (double)k;
  const double z = s * s;
  const double w = z * z;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

__device__ __forceinline__ double k_sin(double x, double y, bool tail) {
  const double S1 = bits_to_d(0xBFC5555555555549ull), S2 = bits_to_d(0x3F8111111110F8A6ull),
               S3 = bits_to_d(0xBF2A01A019C161D5ull), S4 = bits_to_d(0x3EC71DE357B1FE7Dull),
               S5 = bits_to_d(0xBE5AE5E68A2B9CEBull), S6 = bits_to_d(0x3DE5D93A5ACFD57Cull);
  const double z = x * x;
  const double v = z * x;
  const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  if (!tail) return x + v * (S1 + z * r);
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

__device__ __forceinline__ double k_cos(double x, double y) {
  const double C1 = bits_to_d(0x3FA555555555554Cull), C2 = bits_to_d(0xBF56C16C16C15177ull),
               C3 = bits_to_d(0x3EFA01A019CB1590ull), C4 = bits_to_d(0xBE927E4F809C52ADull),
               C5 = bits_to_d(0x3E21EE9EBDB4B1C4ull), C6 = bits_to_d(0xBDA8FAE9BE8838D4ull);
  const double z = x * x;
  const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  const double hz = 0.5 * z;
  const double w = 1.0 - hz;
  return w + (((1.0 - w) - hz) + (z * r - x * y));
}

// sin(x) with fdlibm's medium Cody-Waite reduction; det_sin is its called
// form (the multi-slot kernels), det_sin_inl the inlined one (the pipelined
// kernels' generator role: a call there spilled live registers to scratch
// around every Sine tick)
__device__ __forceinline__ double det_sin_inl(double x) {
  const double invpio2 = bits_to_d(0x3FE45F306DC9C883ull);
  const double pio2_1 = bits_to_d(0x3FF921FB54400000ull), pio2_1t = bits_to_d(0x3DD0B4611A626331ull);
  const double pio2_2 = bits_to_d(0x3DD0B4611A600000ull), pio2_2t = bits_to_d(0x3BA3198A2E037073ull);
  const double pio2_3 = bits_to_d(0x3BA3198A2E000000ull), pio2_3t = bits_to_d(0x397B839A252049C1ull);
  const double ax = fabs(x);
  if (ax <= 0.78539816339744827900) return k_sin(x, 0.0, false);
  if (!(ax < __builtin_inf())) return x - x;
  const double fn = floor(x * invpio2 + 0.5);
  const int32_t n = (int32_t)(int64_t)fn;
  double r = x - fn * pio2_1;
  double w = fn * pio2_1t;
  double y0 = r - w;
  const int32_t j = (int32_t)((d_to_bits(x) >> 52) & 0x7ff);
  int32_t i = j - (int32_t)((d_to_bits(y0) >> 52) & 0x7ff);
  if (i > 16) {
    double t = r;
    w = fn * pio2_2;
    r = t - w;
    w = fn * pio2_2t - ((t - r) - w);
    y0 = r - w;
    i = j - (int32_t)((d_to_bits(y0) >> 52) & 0x7ff);
    if (i > 49) {
      t = r;
      w = fn * pio2_3;
      r = t - w;
      w = fn * pio2_3t - ((t - r) - w);
      y0 = r - w;
    }
  }
  const double y1 = (r - y0) - w;
  const int q = n & 3;
  const double v = (q & 1) ? k_cos(y0, y1) : k_sin(y0, y1, true);
  return (q >= 2) ? -v : v;
}
__device__ __noinline__ double det_sin(double x) { return det_sin_inl(x); }

constexpr double TWO_M32 = 2.3283064365386962890625e-10;

// Arithmetic of the reward shaping (DSR / DDR quotients and square roots, and
// the quotient inside log_ratio, whose residual term absorbs its last bits):
// outputs compared at a relative tolerance (rtol 1e-6, tests
// 1e-12) whose error stays relative to the output itself, and which never
// feed the ledger, the prices, done or State.  a / b as a times the
// reciprocal of b refined by two Newton steps (<= 2 ulp; 6 VALU instead of
// the IEEE sequence's 11), sqrt x from v_rsq_f64 with one Goldschmidt
// refinement (<= 1 ulp; 8 VALU instead of 17).  Operands outside the normal
// class (zero, denormal, inf, NaN, negative square-root arguments) take the
// IEEE operation.  The reward ratio curEq / prevEq stays IEEE: a small log
// reward would carry its last-bit error at a large relative size.  Every step
// kernel uses these helpers, so the schedules stay bit-identical.
constexpr int kNormalClass = (1 << 3) | (1 << 8);  // v_cmp_class: -normal | +normal

// IEEE binary64 x / y split at the reciprocal.  The compiler's division
// (v_div_scale twice, v_rcp, four Newton fma, mul, fma, v_div_fmas,
// v_div_fixup) forms a refined reciprocal of y that depends on y alone
// wherever v_div_scale leaves both operands unscaled -- y and x / y normal,
// the exponent of x above 53 - 1023 and at most 767 above y's -- and there
// v_div_fmas is a plain fma and v_div_fixup the identity.  rcp_refined(y) is
// that reciprocal for |y| in [2^-150, 2^150] (0 outside); div_by_rcp(x, y, r)
// finishes the quotient with the sequence's last three operations for |x| in
// [2^-600, 2^600] and falls back to the division elsewhere: the IEEE
// quotient, bit for bit.  (The three-role kernel's generator forms the
// reciprocal of each price it publishes, off the ledger's chain.)
__device__ __forceinline__ double rcp_refined(double y) {
  const double ay = fabs(y);
  if (!(ay >= 0x1p-150 && ay <= 0x1p150)) return 0.;
  const double r = __builtin_amdgcn_rcp(y);
  const double f1 = __builtin_fma(r, __builtin_fma(-y, r, 1.0), r);
  return __builtin_fma(f1, __builtin_fma(-y, f1, 1.0), f1);
}
__device__ __forceinline__ double div_by_rcp(double x, double y, double r) {
  const double ax = fabs(x);
  const bool fast = r != 0. && ax >= 0x1p-600 && ax <= 0x1p600;
  double q = x * r;
  q = __builtin_fma(__builtin_fma(-y, q, x), r, q);
  if (!fast) {
    // (the empty volatile asm keeps the division in its branch: speculated,
    // as the compiler otherwise does with a lone fdiv, every lane would run
    // it beside the finish above)
    double xs = x;
    asm volatile("" : "+v"(xs));
    q = xs / y;
  }
  return q;
}
__device__ __forceinline__ double rt_div(double a, double b) {
  if (!__builtin_amdgcn_class(b, kNormalClass)) return a / b;
  double r = __builtin_amdgcn_rcp(b);
  r = __builtin_fma(r, __builtin_fma(-b, r, 1.0), r);
  r = __builtin_fma(r, __builtin_fma(-b, r, 1.0), r);
  return a * r;
}
__device__ __forceinline__ double rt_sqrt(double x) {
  if (!__builtin_amdgcn_class(x, 1 << 8)) return sqrt(x);
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double r = __builtin_fma(-g, h, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  return __builtin_fma(__builtin_fma(-g, g, x), h, g);
}

// Variates, specification v3 (this framework's own: the reference's streams
// are seeded from the wall clock and cannot be replayed).  Every tick of an
// (env, asset) has a draw index d = timestamp + resets (Lane.dskip: each
// Env::reset skips one index, so an auto-reset keeps d's parity in step with
// the other envs').  Ticks come in pairs P = d >> 1 that share one
// Box-Muller transform of block A = Philox4x32-10(key seed, counter (P, env,
// asset | 0 << 16)):
//   u1 = ((xA1:xA0 >> 11) + 1) 2^-53 in (0,1],  u2 = xA2 2^-32 in [0,1)
//   r  = sqrt(-2 log u1)
//   d even: z = r cos(2 pi u2),  ut = xA3 2^-32,  dbit = xA0 & 1 (a bit u1 drops)
//   d odd:  z = r sin(2 pi u2),  ut = xB3 2^-32,  dbit = xB0 & 1 from block B
//           (counter slot 3 of the same pair)
// (z: the normal variate; ut: the TrendOU regime-switch uniform; dbit: the
// trend direction.)  The other blocks -- slot 1 (trend length and slope),
// OUPair's slot 2, SineAdder's slot c, SineDynamic's 0 and 16 + c -- are keyed
// by d itself.  log, cos and sin are fdlibm's algorithms with their
// polynomials in fused multiply-add Horner form (v_log2pi / v_sincos2pi;
// fma is correctly rounded, so the host restatement reproduces every bit).
// A lane keeps the odd half of its last pair (zc, tagged P + 1): in a kernel
// whose lanes tick in step the pair's transform runs on even ticks only and
// an odd tick draws block B alone.
struct Draw {
  double z, ut;
  uint32_t dbit;
};

// fdlibm e_log.c for the variate's u1 in (0, 1] (normal, positive), the
// polynomial in fma form
__device__ __forceinline__ double v_log(double x) {
  const double ln2_hi = bits_to_d(0x3fe62e42fee00000ull);
  const double ln2_lo = bits_to_d(0x3dea39ef35793c76ull);
  const double Lg1 = bits_to_d(0x3FE5555555555593ull), Lg2 = bits_to_d(0x3FD999999997FA04ull),
               Lg3 = bits_to_d(0x3FD2492494229359ull), Lg4 = bits_to_d(0x3FCC71C51D8E78AFull),
               Lg5 = bits_to_d(0x3FC7466496CB03DEull), Lg6 = bits_to_d(0x3FC39A09D078C69Full),
               Lg7 = bits_to_d(0x3FC2F112DF3E5244ull);
  const uint64_t ix = d_to_bits(x);
  int32_t hx = (int32_t)(ix >> 32);
  int32_t k = ((hx >> 20) & 0x7ff) - 1023;
  hx &= 0x000fffff;
  const int32_t i = (hx + 0x95f64) & 0x100000;
  k += (i >> 20);
  const uint64_t mb = ((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (ix & 0xffffffffull);
  const double f = bits_to_d(mb) - 1.0;
  const double s = f / (2.0 + f);
  const double dk = (double)k;
  const double z = s * s;
  const double w = z * z;
  const double t1 = w * __builtin_fma(w, __builtin_fma(w, Lg6, Lg4), Lg2);
  const double t2 = z * __builtin_fma(w, __builtin_fma(w, __builtin_fma(w, Lg7, Lg5), Lg3), Lg1);
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

// cos(2 pi u) and sin(2 pi u), u in [0,1): t = 4u, q = floor(t + 1/2),
// r = (t - q) pi/2, fdlibm's __kernel_cos / __kernel_sin (y = 0) on r in fma
// form, placed by the quadrant q mod 4
__device__ __forceinline__ void v_sincos2pi(double u, double& sn, double& cs) {
  const double S1 = bits_to_d(0xBFC5555555555549ull), S2 = bits_to_d(0x3F8111111110F8A6ull),
               S3 = bits_to_d(0xBF2A01A019C161D5ull), S4 = bits_to_d(0x3EC71DE357B1FE7Dull),
               S5 = bits_to_d(0xBE5AE5E68A2B9CEBull), S6 = bits_to_d(0x3DE5D93A5ACFD57Cull);
  const double C1 = bits_to_d(0x3FA555555555554Cull), C2 = bits_to_d(0xBF56C16C16C15177ull),
               C3 = bits_to_d(0x3EFA01A019CB1590ull), C4 = bits_to_d(0xBE927E4F809C52ADull),
               C5 = bits_to_d(0x3E21EE9EBDB4B1C4ull), C6 = bits_to_d(0xBDA8FAE9BE8838D4ull);
  const double pio2 = bits_to_d(0x3FF921FB54442D18ull);
  const double t = 4.0 * u;
  const double q = floor(t + 0.5);
  const double x = (t - q) * pio2;
  const int iq = ((int)q) & 3;
  const double z = x * x;
  // __kernel_sin: x + x^3 (S1 + z r)
  const double rs = __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, S6, S5), S4), S3), S2);
  const double ks = __builtin_fma(z * x, __builtin_fma(z, rs, S1), x);
  // __kernel_cos: w + (((1 - w) - z/2) + z r), w = 1 - z/2
  const double rc =
      z * __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, C6, C5), C4), C3), C2), C1);
  const double hz = 0.5 * z;
  const double w = 1.0 - hz;
  const double kc = w + (((1.0 - w) - hz) + z * rc);
  // cos(q pi/2 + x), sin(q pi/2 + x) for q mod 4 = 0, 1, 2, 3
  const double c0 = (iq & 1) ? ks : kc, s0 = (iq & 1) ? kc : ks;
  cs = (iq == 1 || iq == 2) ? -c0 : c0;
  sn = (iq >= 2) ? -s0 : s0;
}

// the radius and angle uniform of pair block A
__device__ __forceinline__ double v_radius(const u4& x) {
  const uint64_t a = (((uint64_t)x.y << 32) | x.x) >> 11;
  const double u1 = (double)(a + 1) * TWO_M53;
  return sqrt(-2.0 * v_log(u1));
}

// the variate of draw index d (v3 above); zc / ztag: the lane's cached odd
// half (ztag = P + 1 when zc holds pair P's r sin(2 pi u2))
__device__ __forceinline__ Draw draw_d(uint64_t seed, uint64_t env, uint32_t asset, uint64_t d, double& zc,
                                       uint64_t& ztag) {
  const uint64_t P = d >> 1;
  Draw r;
#ifdef MGN_ABL_DRAW  // diagnostic timing build: a cheap stand-in for the variate (wrong values)
  const uint32_t h = ((uint32_t)d * 0x9E3779B1u) ^ ((uint32_t)env * 0x85EBCA6Bu) ^ (asset * 0xC2B2AE35u);
  r.z = (double)(int32_t)(h & 0xffffu) * (1.0 / 32768.0) - 1.0;
  r.ut = (double)(h >> 16) * (1.0 / 65536.0);
  r.dbit = h & 1u;
  (void)P;
  (void)zc;
  (void)ztag;
  return r;
#else
  if (d & 1) {
    if (ztag != P + 1) {  // the pair's transform did not run here (first tick, or out of step)
      const u4 x = block(seed, env, asset, 0, P);
      double sn, cs;
      v_sincos2pi((double)x.z * TWO_M32, sn, cs);
      zc = v_radius(x) * sn;
    }
    const u4 y = block(seed, env, asset, 3, P);
    r.z = zc;
    r.ut = (double)y.w * TWO_M32;
    r.dbit = y.x & 1u;
  } else {
    const u4 x = block(seed, env, asset, 0, P);
    double sn, cs;
    v_sincos2pi((double)x.z * TWO_M32, sn, cs);
    const double rad = v_radius(x);
    r.z = rad * cs;
    zc = rad * sn;
    ztag = P + 1;
    r.ut = (double)x.w * TWO_M32;
    r.dbit = x.x & 1u;
  }
  return r;
#endif
}

// the normal variate alone of a full block (the per-tick blocks: OUPair's
// mean walk, SineAdder's components, SineDynamic's noise): r cos(2 pi u2)
__device__ __forceinline__ double normal_of(const u4& x) {
  double sn, cs;
  v_sincos2pi((double)x.z * TWO_M32, sn, cs);
  return v_radius(x) * cs;
}

// std::modf's fractional part: x - trunc(x) is exact; its sign follows x (modf(-3.0) = -0.0)
// natural log of a reward ratio (Env.h:211-212, offpolicy_q.py:152-164), an
// output that never feeds the ledger.  Within 1/32 of 1 -- every step that is
// not a blow-up -- by the atanh series log x = 2 (s + s^3/3 + ... + s^9/9),
// s = (x - 1) / (x + 1) carried as s_hi + s_lo (x + 1 = u + e exactly, the
// division's residual by fma), so the result is rounded once from a value
// within ~2^-60 relative: it agrees with a correctly rounded log except in
// rare last-bit cases (36 of 3e5 random ratios against glibc).  |s| < 1/63,
// so the dropped s^11/11 term is < 2^-66 relative.  Elsewhere the library log.
// Compared with the oracle (glibc log) at rtol 1e-12.
__device__ __forceinline__ double log_ratio(double x) {
  const double d = x - 1.0;
  if (fabs(d) <= 0.03125) {
    const double u = x + 1.0;
    const double e = x - (u - 1.0);  // x + 1 == u + e exactly
    const double sh = rt_div(d, u);
    const double r = __fma_rn(-sh, u, d);  // d - sh * u exactly
    const double sl = (r - sh * e) * 0.5;  // 1/u ~ 1/2 to 2 %: s_lo needs few bits
    const double s2 = sh * sh;
    const double t =
        s2 * (0.3333333333333333 + s2 * (0.2 + s2 * (0.14285714285714285 + s2 * 0.1111111111111111)));
    const double s_2 = sh + sh;
    return s_2 + ((sl + sl) + s_2 * t);
  }
  return log(x);
}

__device__ __forceinline__ double frac_part(double x) { return copysign(x - trunc(x), x); }

// fdlibm e_asin.c on |x| <= 1 (same statements as the oracle's orc_asin)
__device__ __noinline__ double det_asin(double x) {
  const double pio2_hi = bits_to_d(0x3FF921FB54442D18ull), pio2_lo = bits_to_d(0x3C91A62633145C07ull),
               pio4_hi = bits_to_d(0x3FE921FB54442D18ull);
  const double pS0 = bits_to_d(0x3FC5555555555555ull), pS1 = bits_to_d(0xBFD4D61203EB6F7Dull),
               pS2 = bits_to_d(0x3FC9C1550E884455ull), pS3 = bits_to_d(0xBFA48228B5688F3Bull),
               pS4 = bits_to_d(0x3F49EFE07501B288ull), pS5 = bits_to_d(0x3F023DE10DFDF709ull),
               qS1 = bits_to_d(0xC0033A271C8A2D4Bull), qS2 = bits_to_d(0x40002AE59C598AC8ull),
               qS3 = bits_to_d(0xBFE6066C1B8D0159ull), qS4 = bits_to_d(0x3FB3B8C5B12E9282ull);
  const uint64_t bx = d_to_bits(x);
  const int32_t hx = (int32_t)(bx >> 32);
  const int32_t ix = hx & 0x7fffffff;
  if (ix >= 0x3ff00000) {
    if (((ix - 0x3ff00000) | (int32_t)(uint32_t)bx) == 0) return x * pio2_hi + x * pio2_lo;
    return (x - x) / (x - x);
  }
  if (ix < 0x3fe00000) {
    if (ix < 0x3e400000) return x;
    const double t = x * x;
    const double p = t * (pS0 + t * (pS1 + t * (pS2 + t * (pS3 + t * (pS4 + t * pS5)))));
    const double q = 1.0 + t * (qS1 + t * (qS2 + t * (qS3 + t * qS4)));
    const double w = p / q;
    return x + x * w;
  }
  double w = 1.0 - fabs(x);
  double t = w * 0.5;
  double p = t * (pS0 + t * (pS1 + t * (pS2 + t * (pS3 + t * (pS4 + t * pS5)))));
  double q = 1.0 + t * (qS1 + t * (qS2 + t * (qS3 + t * qS4)));
  const double sr = sqrt(t);
  if (ix >= 0x3FEF3333) {
    w = p / q;
    t = pio2_hi - (2.0 * (sr + sr * w) - pio2_lo);
  } else {
    w = bits_to_d(d_to_bits(sr) & 0xffffffff00000000ull);
    const double c = (t - w * w) / (sr + w);
    const double r = p / q;
    p = 2.0 * sr * r - (pio2_lo - 2.0 * c);
    q = pio4_hi - 2.0 * w;
    t = pio4_hi - (p - q);
  }
  return (hx > 0) ? t : -t;
}

}  // namespace mgn
