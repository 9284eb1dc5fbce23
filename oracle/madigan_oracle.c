/*
 * madigan_oracle.c -- CPU restatement of madigan's market-simulation step.
 *
 * TEST INFRASTRUCTURE ONLY (see madigan_oracle.h).  Restates, statement by
 * statement and in the reference's operation order:
 *   Portfolio   madigan/environments/cpp/Portfolio.cpp:150-323
 *   Broker      madigan/environments/cpp/Broker.cpp:124-178
 *   Env         madigan/environments/cpp/Env.h:150-256
 *   Sine        madigan/environments/cpp/DataSource.cpp:455-543
 *   OU          madigan/environments/cpp/DataSource.cpp:1118-1180
 *   TrendOU     madigan/environments/cpp/DataSource.cpp:1364-1502
 *   Composite   madigan/environments/cpp/DataSource.cpp:411-451
 *   DSR/DDR/PPC madigan/utils/buffers/nstep_buffer.py:20-204
 *   Stacker     madigan/utils/preprocessor.py:53-107, :143-199
 *   agent step  madigan/modelling/algorithm/dqn.py:160-179,
 *               madigan/modelling/algorithm/offpolicy_q.py:138-164
 *
 * Build strict IEEE: gcc -O2 -ffp-contract=off (oracle/Makefile).  The same
 * source built with -O3 -march=native -ffast-math (the reference's own flags,
 * madigan/environments/cpp/CMakeLists.txt:5) is the CPU-baseline timing build.
 */
#include "madigan_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define MAXA ORC_MAX_ASSETS

/* ------------------------------------------------------------------------ */
/* Deterministic math: the random-variate transform is this framework's own */
/* specification (the reference seeds std::default_random_engine from the   */
/* wall clock, DataSource.cpp:472/1131/1407, so its stream is not            */
/* reproducible).  Device code implements the identical algorithms.          */
/* ------------------------------------------------------------------------ */

static inline double from_bits(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
static inline uint64_t to_bits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }

void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c0 = hi1 ^ c1 ^ k0;
    c1 = lo1;
    c2 = hi0 ^ c3 ^ k1;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static void draw(uint64_t seed, uint64_t env, uint32_t asset, uint32_t slot, uint64_t tick,
                 uint64_t *a, uint64_t *b) {
  uint32_t ctr[4] = {(uint32_t)tick, (uint32_t)env, asset | (slot << 16),
                     (uint32_t)(tick >> 32) ^ (uint32_t)(env >> 32)};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t x[4];
  orc_philox4x32_10(ctr, key, x);
  *a = (((uint64_t)x[1] << 32) | x[0]) >> 11;
  *b = (((uint64_t)x[3] << 32) | x[2]) >> 11;
}

static const double TWO_M53 = 1.1102230246251565404e-16; /* 2^-53 */

void orc_uniform2(uint64_t seed, uint64_t env, uint32_t asset, uint32_t slot, uint64_t tick,
                  double *u0, double *u1) {
  uint64_t a, b;
  draw(seed, env, asset, slot, tick, &a, &b);
  *u0 = (double)a * TWO_M53;
  *u1 = (double)b * TWO_M53;
}

/* fdlibm e_log.c algorithm (public domain, Sun Microsystems) for normal x>0 */
double orc_log(double x) {
  const double ln2_hi = from_bits(0x3fe62e42fee00000ull);
  const double ln2_lo = from_bits(0x3dea39ef35793c76ull);
  const double Lg1 = from_bits(0x3FE5555555555593ull), Lg2 = from_bits(0x3FD999999997FA04ull),
               Lg3 = from_bits(0x3FD2492494229359ull), Lg4 = from_bits(0x3FCC71C51D8E78AFull),
               Lg5 = from_bits(0x3FC7466496CB03DEull), Lg6 = from_bits(0x3FC39A09D078C69Full),
               Lg7 = from_bits(0x3FC2F112DF3E5244ull);
  uint64_t ix = to_bits(x);
  int32_t hx = (int32_t)(ix >> 32);
  int32_t k = ((hx >> 20) & 0x7ff) - 1023;
  hx &= 0x000fffff;
  int32_t i = (hx + 0x95f64) & 0x100000; /* normalize m into [sqrt(2)/2, sqrt(2)) */
  k += (i >> 20);
  uint64_t mb = ((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (ix & 0xffffffffull);
  double f = from_bits(mb) - 1.0;
  double s = f / (2.0 + f);
  double dk = (double)k;
  double z = s * s;
  double w = z * z;
  double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  double R = t2 + t1;
  double hfsq = 0.5 * f * f;
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

/* fdlibm k_sin.c / k_cos.c kernels on |x| <= pi/4 with tail y */
static double k_sin(double x, double y, int iy) {
  const double S1 = from_bits(0xBFC5555555555549ull), S2 = from_bits(0x3F8111111110F8A6ull),
               S3 = from_bits(0xBF2A01A019C161D5ull), S4 = from_bits(0x3EC71DE357B1FE7Dull),
               S5 = from_bits(0xBE5AE5E68A2B9CEBull), S6 = from_bits(0x3DE5D93A5ACFD57Cull);
  double z = x * x;
  double v = z * x;
  double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  if (iy == 0) return x + v * (S1 + z * r);
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}
static double k_cos(double x, double y) {
  const double C1 = from_bits(0x3FA555555555554Cull), C2 = from_bits(0xBF56C16C16C15177ull),
               C3 = from_bits(0x3EFA01A019CB1590ull), C4 = from_bits(0xBE927E4F809C52ADull),
               C5 = from_bits(0x3E21EE9EBDB4B1C4ull), C6 = from_bits(0xBDA8FAE9BE8838D4ull);
  double z = x * x;
  double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  double hz = 0.5 * z;
  double w = 1.0 - hz;
  return w + (((1.0 - w) - hz) + (z * r - x * y));
}

/* The variates' math (specification v3, the device's mgn_math.h v_log /
 * v_sincos2pi): fdlibm's log and __kernel_sin / __kernel_cos with their
 * polynomials in fused multiply-add Horner form.  C99 fma() is correctly
 * rounded, as the device's v_fma_f64, so every bit is reproduced. */
double orc_vlog(double x) {
  const double ln2_hi = from_bits(0x3fe62e42fee00000ull);
  const double ln2_lo = from_bits(0x3dea39ef35793c76ull);
  const double Lg1 = from_bits(0x3FE5555555555593ull), Lg2 = from_bits(0x3FD999999997FA04ull),
               Lg3 = from_bits(0x3FD2492494229359ull), Lg4 = from_bits(0x3FCC71C51D8E78AFull),
               Lg5 = from_bits(0x3FC7466496CB03DEull), Lg6 = from_bits(0x3FC39A09D078C69Full),
               Lg7 = from_bits(0x3FC2F112DF3E5244ull);
  uint64_t ix = to_bits(x);
  int32_t hx = (int32_t)(ix >> 32);
  int32_t k = ((hx >> 20) & 0x7ff) - 1023;
  hx &= 0x000fffff;
  int32_t i = (hx + 0x95f64) & 0x100000;
  k += (i >> 20);
  uint64_t mb = ((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (ix & 0xffffffffull);
  double f = from_bits(mb) - 1.0;
  double s = f / (2.0 + f);
  double dk = (double)k;
  double z = s * s;
  double w = z * z;
  double t1 = w * fma(w, fma(w, Lg6, Lg4), Lg2);
  double t2 = z * fma(w, fma(w, fma(w, Lg7, Lg5), Lg3), Lg1);
  double R = t2 + t1;
  double hfsq = 0.5 * f * f;
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

/* cos(2 pi u) and sin(2 pi u), u in [0,1): t = 4u, q = floor(t + 1/2),
 * x = (t - q) pi/2 (|x| <= pi/4), the kernels placed by the quadrant q mod 4 */
void orc_vsincos2pi(double u, double *sn, double *cs) {
  const double S1 = from_bits(0xBFC5555555555549ull), S2 = from_bits(0x3F8111111110F8A6ull),
               S3 = from_bits(0xBF2A01A019C161D5ull), S4 = from_bits(0x3EC71DE357B1FE7Dull),
               S5 = from_bits(0xBE5AE5E68A2B9CEBull), S6 = from_bits(0x3DE5D93A5ACFD57Cull);
  const double C1 = from_bits(0x3FA555555555554Cull), C2 = from_bits(0xBF56C16C16C15177ull),
               C3 = from_bits(0x3EFA01A019CB1590ull), C4 = from_bits(0xBE927E4F809C52ADull),
               C5 = from_bits(0x3E21EE9EBDB4B1C4ull), C6 = from_bits(0xBDA8FAE9BE8838D4ull);
  const double pio2 = from_bits(0x3FF921FB54442D18ull);
  double t = 4.0 * u;
  double q = floor(t + 0.5);
  double x = (t - q) * pio2;
  int iq = ((int)q) & 3;
  double z = x * x;
  double rs = fma(z, fma(z, fma(z, fma(z, S6, S5), S4), S3), S2);
  double ks = fma(z * x, fma(z, rs, S1), x);               /* __kernel_sin, y = 0 */
  double rc = z * fma(z, fma(z, fma(z, fma(z, fma(z, C6, C5), C4), C3), C2), C1);
  double hz = 0.5 * z;
  double w = 1.0 - hz;
  double kc = w + (((1.0 - w) - hz) + z * rc);            /* __kernel_cos, y = 0 */
  switch (iq) {
    case 0: *cs = kc; *sn = ks; break;
    case 1: *cs = -ks; *sn = kc; break;
    case 2: *cs = -kc; *sn = -ks; break;
    default: *cs = ks; *sn = -kc; break;
  }
}

/* sin(x): fdlibm medium-range Cody-Waite reduction (e_rem_pio2.c), kernels above. */
double orc_sin(double x) {
  const double invpio2 = from_bits(0x3FE45F306DC9C883ull);
  const double pio2_1 = from_bits(0x3FF921FB54400000ull), pio2_1t = from_bits(0x3DD0B4611A626331ull);
  const double pio2_2 = from_bits(0x3DD0B4611A600000ull), pio2_2t = from_bits(0x3BA3198A2E037073ull);
  const double pio2_3 = from_bits(0x3BA3198A2E000000ull), pio2_3t = from_bits(0x397B839A252049C1ull);
  double ax = fabs(x);
  if (ax <= 0.78539816339744827900) return k_sin(x, 0.0, 0);
  if (!(ax < INFINITY)) return x - x;
  double fn = floor(x * invpio2 + 0.5);
  int32_t n = (int32_t)(int64_t)fn;
  double r = x - fn * pio2_1;
  double w = fn * pio2_1t;
  double y0 = r - w;
  int32_t j = (int32_t)((to_bits(x) >> 52) & 0x7ff);
  int32_t i = j - (int32_t)((to_bits(y0) >> 52) & 0x7ff);
  if (i > 16) { /* 2nd iteration, good to 118 bits */
    double t = r;
    w = fn * pio2_2;
    r = t - w;
    w = fn * pio2_2t - ((t - r) - w);
    y0 = r - w;
    i = j - (int32_t)((to_bits(y0) >> 52) & 0x7ff);
    if (i > 49) { /* 3rd iteration, 151 bits */
      t = r;
      w = fn * pio2_3;
      r = t - w;
      w = fn * pio2_3t - ((t - r) - w);
      y0 = r - w;
    }
  }
  double y1 = (r - y0) - w;
  switch (n & 3) {
    case 0: return k_sin(y0, y1, 1);
    case 1: return k_cos(y0, y1);
    case 2: return -k_sin(y0, y1, 1);
    default: return -k_cos(y0, y1);
  }
}

static const double TWO_M32 = 2.3283064365386962890625e-10; /* 2^-32 */

/* the raw Philox block of counter slot `slot` at counter value c */
static void block_at(uint64_t seed, uint64_t env, uint32_t asset, uint32_t slot, uint64_t c,
                     uint32_t x[4]) {
  uint32_t ctr[4] = {(uint32_t)c, (uint32_t)env, asset | (slot << 16),
                     (uint32_t)(c >> 32) ^ (uint32_t)(env >> 32)};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  orc_philox4x32_10(ctr, key, x);
}

/* Box-Muller radius sqrt(-2 log u1), u1 = ((x1:x0 >> 11) + 1) 2^-53 */
static double radius_of(const uint32_t x[4]) {
  uint64_t a = (((uint64_t)x[1] << 32) | x[0]) >> 11;
  double u1 = (double)(a + 1) * TWO_M53;
  return sqrt(-2.0 * orc_vlog(u1));
}

/* Variates of draw index d (specification v3; d = timestamp + resets of the
 * env).  Ticks pair up: P = d >> 1, block A = slot 0 at counter P:
 *   u2 = xA2 2^-32, r = radius_of(A)
 *   d even: z = r cos(2 pi u2), ut = xA3 2^-32, dbit = xA0 & 1
 *   d odd:  z = r sin(2 pi u2), ut = xB3 2^-32, dbit = xB0 & 1, block B = slot 3 at P
 * (z: the normal variate, ut: the TrendOU regime-switch uniform, dbit: the
 * trend direction) */
void orc_draw0(uint64_t seed, uint64_t env, uint32_t asset, uint64_t d, double *z, double *ut,
               uint32_t *dbit) {
  uint32_t x[4];
  const uint64_t P = d >> 1;
  block_at(seed, env, asset, 0, P, x);
  double sn, cs;
  orc_vsincos2pi((double)x[2] * TWO_M32, &sn, &cs);
  const double r = radius_of(x);
  if ((d & 1) == 0) {
    *z = r * cs;
    *ut = (double)x[3] * TWO_M32;
    *dbit = x[0] & 1u;
  } else {
    uint32_t y[4];
    block_at(seed, env, asset, 3, P, y);
    *z = r * sn;
    *ut = (double)y[3] * TWO_M32;
    *dbit = y[0] & 1u;
  }
}

/* the normal variate of a full block (per-tick blocks: OUPair's mean walk,
 * SineAdder's components, SineDynamic's noise): r cos(2 pi u2) */
static double normal_of(const uint32_t x[4]) {
  double sn, cs;
  orc_vsincos2pi((double)x[2] * TWO_M32, &sn, &cs);
  return radius_of(x) * cs;
}

/* fdlibm e_asin.c (Sun Microsystems) on |x| <= 1, plain binary64 */
double orc_asin(double x) {
  const double pio2_hi = from_bits(0x3FF921FB54442D18ull), pio2_lo = from_bits(0x3C91A62633145C07ull),
               pio4_hi = from_bits(0x3FE921FB54442D18ull);
  const double pS0 = from_bits(0x3FC5555555555555ull), pS1 = from_bits(0xBFD4D61203EB6F7Dull),
               pS2 = from_bits(0x3FC9C1550E884455ull), pS3 = from_bits(0xBFA48228B5688F3Bull),
               pS4 = from_bits(0x3F49EFE07501B288ull), pS5 = from_bits(0x3F023DE10DFDF709ull),
               qS1 = from_bits(0xC0033A271C8A2D4Bull), qS2 = from_bits(0x40002AE59C598AC8ull),
               qS3 = from_bits(0xBFE6066C1B8D0159ull), qS4 = from_bits(0x3FB3B8C5B12E9282ull);
  uint64_t bx = to_bits(x);
  int32_t hx = (int32_t)(bx >> 32);
  int32_t ix = hx & 0x7fffffff;
  if (ix >= 0x3ff00000) {
    if (((ix - 0x3ff00000) | (int32_t)(uint32_t)bx) == 0) return x * pio2_hi + x * pio2_lo;
    return (x - x) / (x - x);
  }
  if (ix < 0x3fe00000) {                  /* |x| < 0.5 */
    if (ix < 0x3e400000) return x;        /* |x| < 2^-27 */
    double t = x * x;
    double p = t * (pS0 + t * (pS1 + t * (pS2 + t * (pS3 + t * (pS4 + t * pS5)))));
    double q = 1.0 + t * (qS1 + t * (qS2 + t * (qS3 + t * qS4)));
    double w = p / q;
    return x + x * w;
  }
  double w = 1.0 - fabs(x);
  double t = w * 0.5;
  double p = t * (pS0 + t * (pS1 + t * (pS2 + t * (pS3 + t * (pS4 + t * pS5)))));
  double q = 1.0 + t * (qS1 + t * (qS2 + t * (qS3 + t * qS4)));
  double sr = sqrt(t);
  if (ix >= 0x3FEF3333) {                 /* |x| > 0.975 */
    w = p / q;
    t = pio2_hi - (2.0 * (sr + sr * w) - pio2_lo);
  } else {
    w = from_bits(to_bits(sr) & 0xffffffff00000000ull);
    double c = (t - w * w) / (sr + w);
    double r = p / q;
    p = 2.0 * sr * r - (pio2_lo - 2.0 * c);
    q = pio4_hi - 2.0 * w;
    t = pio4_hi - (p - q);
  }
  return (hx > 0) ? t : -t;
}

double orc_normal(uint64_t seed, uint64_t env, uint32_t asset, uint64_t tick) {
  double z, ut;
  uint32_t b;
  orc_draw0(seed, env, asset, tick, &z, &ut, &b);
  return z;
}

/* Canonical reduction: pairwise tree over v[0..n-1], padded with +0.0 to the
 * next power of two.  The HIP kernels use the same tree. */
double orc_canon_sum(const double *v, int n) {
  double t[2 * MAXA + 2];
  int p = 1;
  while (p < n) p <<= 1;
  for (int i = 0; i < p; ++i) t[i] = (i < n) ? v[i] : 0.0;
  for (int w = p; w > 1; w >>= 1)
    for (int i = 0; i < w / 2; ++i) t[i] = t[2 * i] + t[2 * i + 1];
  return t[0];
}

/* ------------------------------------------------------------------------ */
/* Environment state                                                        */
/* ------------------------------------------------------------------------ */

typedef struct {
  /* Portfolio (Portfolio.h:109-130) */
  double L[MAXA], mep[MAXA], Bm[MAXA];
  double cash;
  /* DataSource state */
  double P[MAXA];
  double x[MAXA];       /* Synth phase accumulator (DataSource.h:246) */
  double ouMean[MAXA];  /* TrendOU (DataSource.h:670) */
  double dY[MAXA];
  int32_t tlen[MAXA];
  uint8_t trending[MAXA];
  int8_t dir[MAXA];
  uint64_t ts;
  uint64_t dskip;  /* resets so far: the variates' draw index is ts + dskip (v3) */
  /* HDFSourceSingle (DataSource.h:136-148): currentData_, currentIdx_,
   * currentCacheIdx_, currentCacheSize_, first file row of the cache */
  double feat[MAXA];
  int64_t h_idx, h_cidx, h_ccs, h_cstart;
  /* shaper state (nstep_buffer.py:38-60): index 0 for scalar */
  double sA[MAXA], sB[MAXA];
  /* episode statistics */
  double ep_ret, ep_len, last_ret, last_len, last_eq, n_done;
} orc_env;

struct orc_batch {
  orc_config cfg;
  orc_asset_src src[MAXA];
  int N, A;
  orc_env *envs;
  double *ext;  /* (N,A) external prices */
  double *aux;  /* (N,A,ORC_AUX_WIDTH) multi-component source state, or NULL */
  orc_ring ring; /* StackerDiscrete deques (preprocessor.py:150-152), F, P = A+1 */
  int F;         /* State.price width: A, or the replay source's feature count */
  int replay;
  /* replay file arrays and bounds (HDFSourceSingle) */
  double *rp_price, *rp_feat;
  uint64_t *rp_ts;
  int64_t rp_T, rp_first, rp_second, rp_cs;
  /* NStepBuffer per env (nstep_buffer.py:315-356), oldest first: (N, n, D) values
   * (raw reward; PPC: reward + temp*cos), fill count (N), discounts gamma^i */
  double *nring;
  int32_t *nlen;
  double disc[ORC_MAX_NSTEP];
};

/* ---- Portfolio valuation (Portfolio.cpp:170-235) ------------------------ */

static double p_asset_value(const orc_env *s, int A) {           /* :180-182 */
  double t[MAXA];
  for (int i = 0; i < A; ++i) t[i] = s->L[i] * s->P[i];
  return orc_canon_sum(t, A);
}
static double p_pnl(const orc_env *s, int A) {                   /* :184-186 */
  double t[MAXA];
  for (int i = 0; i < A; ++i) t[i] = s->mep[i] * s->L[i];
  return p_asset_value(s, A) - orc_canon_sum(t, A);
}
static double p_balance(const orc_env *s, int A) {               /* :192-197 */
  double t[MAXA];
  for (int i = 0; i < A; ++i) {
    double mask = (s->L[i] < 0.) ? 1.0 : 0.0;
    t[i] = s->L[i] * (s->mep[i] * mask);
  }
  return s->cash + orc_canon_sum(t, A);
}
static double p_borrowed_margin(const orc_env *s, int A) {       /* :207-209 */
  return orc_canon_sum(s->Bm, A);
}
static double p_equity(const orc_env *s, int A) {                /* :211-213 */
  return s->cash + p_asset_value(s, A) - p_borrowed_margin(s, A);
}
static double p_available_margin(const orc_env *s, int A, double reqM) { /* :229-231 */
  return (p_balance(s, A) + p_pnl(s, A)) / reqM;
}
static double p_used_margin(const orc_env *s, int A, double reqM) {      /* :199-201 */
  double t[MAXA];
  for (int i = 0; i < A; ++i) t[i] = fabs(s->L[i]) * s->mep[i];
  return reqM * orc_canon_sum(t, A);
}
static double p_borrowed_asset_value(const orc_env *s, int A) {  /* :219-223 */
  double t[MAXA];
  for (int i = 0; i < A; ++i) {
    double mask = (s->L[i] < 0.) ? 1.0 : 0.0;
    t[i] = s->L[i] * (s->P[i] * mask);
  }
  return orc_canon_sum(t, A);
}

/* Portfolio::checkRisk() -- Portfolio.cpp:243-252 */
static int p_check_risk(const orc_env *s, int A, double mainM) {
  double marginRequired = mainM * p_pnl(s, A);
  if (p_equity(s, A) <= -marginRequired) return ORC_MARGIN_CALL;
  if ((p_balance(s, A) + p_pnl(s, A)) <= -marginRequired) return ORC_MARGIN_CALL;
  return ORC_GREEN;
}

/* Portfolio::checkRisk(assetIdx, units) -- Portfolio.cpp:254-279 */
static int p_check_risk_order(const orc_env *s, int A, double reqM, double mainM, int i,
                              double units) {
  double cashAmount = s->P[i] * units;
  double currentUnits = s->L[i];
  if (signbit(units) != signbit(currentUnits)) {
    if (units > -1 * currentUnits) {
      double excess = units + currentUnits;
      if (p_available_margin(s, A, reqM) <= fabs(s->P[i] * excess) || p_balance(s, A) <= 0.)
        return ORC_INSUFF_MARGIN;
    }
    return ORC_GREEN;
  }
  if (p_check_risk(s, A, mainM) == ORC_MARGIN_CALL) return ORC_MARGIN_CALL;
  if (p_available_margin(s, A, reqM) <= fabs(cashAmount) || p_balance(s, A) <= 0.)
    return ORC_INSUFF_MARGIN;
  return ORC_GREEN;
}

/* Portfolio::handleTransaction -- Portfolio.cpp:284-323 */
static void p_handle_transaction(orc_env *s, double reqM, int i, double transactionPrice,
                                 double units, double transactionCost) {
  double *currentUnits = &s->L[i];
  double *meanEntryPrice = &s->mep[i];
  if (signbit(*currentUnits) != signbit(units)) {
    if (fabs(units) > fabs(*currentUnits)) {
      units += *currentUnits;
      s->cash += *currentUnits * transactionPrice;
      *currentUnits = 0.;
      *meanEntryPrice = transactionPrice;
    }
  } else {
    *meanEntryPrice += (transactionPrice - *meanEntryPrice) * (units / (units + *currentUnits));
  }
  double amount_in_base_currency = transactionPrice * units;
  double marginToUse = amount_in_base_currency * reqM;
  double marginToBorrow = amount_in_base_currency - marginToUse;
  double *borrowedMarginRef = &s->Bm[i];
  *borrowedMarginRef += marginToBorrow;
  s->cash -= (marginToUse + transactionCost);
  *currentUnits += units;
  if (fabs(*currentUnits) < 0.000001) {
    *meanEntryPrice = 0.;
    if (*borrowedMarginRef > 0.) {
      s->cash -= *borrowedMarginRef;
      *borrowedMarginRef = 0.;
    }
  }
  if (*borrowedMarginRef < 0.) {
    s->cash -= *borrowedMarginRef;
    *borrowedMarginRef = 0.;
  }
}

/* Portfolio::ledgerNormedFull -- Portfolio.cpp:150-155 */
static void p_ledger_normed_full(const orc_env *s, int A, double *out) {
  double eq = p_equity(s, A);
  out[0] = (s->cash - p_borrowed_margin(s, A)) / eq;
  for (int i = 0; i < A; ++i) out[1 + i] = (s->L[i] * s->P[i]) / eq;
}

/* Broker::handleTransaction(port, i, u) -- Broker.cpp:124-142, :171-178 */
static void b_handle_transaction(const orc_config *c, orc_env *s, int A, int i, double units,
                                 double *tp_o, double *u_o, double *cost_o, int *risk_o) {
  *tp_o = 0.; *u_o = 0.; *cost_o = 0.; *risk_o = ORC_GREEN;
  if (units != 0.) {
    int risk = p_check_risk_order(s, A, c->required_margin, c->maintenance_margin, i, units);
    *risk_o = risk;
    if (risk == ORC_GREEN) {
      double currentPrice = s->P[i];
      double slippage = (currentPrice * c->slippage_rel) + c->slippage_abs;  /* :172 */
      double transactionPrice = units < 0 ? (currentPrice - slippage) : (currentPrice + slippage);
      double transactionCost = fabs(units * currentPrice) * c->tc_rel + c->tc_abs; /* :131,:176 */
      p_handle_transaction(s, c->required_margin, i, transactionPrice, units, transactionCost);
      *tp_o = transactionPrice; *u_o = units; *cost_o = transactionCost;
    }
  }
}

/* ---- DataSource::getData ------------------------------------------------ */

/* HDFSourceSingle::loadData (DataSource.cpp:368-379) */
static void h_load(const orc_batch *b, orc_env *s) {
  if (s->h_idx >= b->rp_second - 1) s->h_idx = b->rp_first;
  int64_t rest = b->rp_second - s->h_idx;
  s->h_ccs = b->rp_cs < rest ? b->rp_cs : rest;
  s->h_cstart = s->h_idx;
}

/* HDFSourceSingle::getData with iterCache (DataSource.cpp:381-408) */
static void h_get_data(const orc_batch *b, orc_env *s) {
  const int64_t full = b->rp_second - b->rp_first;
  if (s->h_cidx == s->h_ccs || s->h_idx == b->rp_second) {
    if (s->h_ccs >= full) {
      s->h_idx = b->rp_first;
      s->h_cidx = 0;
    } else {
      h_load(b, s);
      s->h_cidx = 0;
    }
  }
  const int64_t row = s->h_cstart + s->h_cidx;
  for (int i = 0; i < b->A; ++i) s->P[i] = b->rp_price[row * b->A + i];
  for (int f = 0; f < b->F; ++f) s->feat[f] = b->rp_feat[row * b->F + f];
  s->ts = b->rp_ts[row];
  s->h_idx++;
  s->h_cidx++;
}

static int h_data_end(const orc_batch *b, const orc_env *s) { /* DataSource.h:126 */
  return b->replay && s->h_idx == b->rp_second;
}

/* State.price of the current tick: currentData (features) */
static const double *state_price(const orc_batch *b, const orc_env *s) {
  return b->replay ? s->feat : s->P;
}

/* WaveTableOsc<double> of setSineOsc (WaveTableOsc.h:104-174): every table of
 * the oscillator holds the same len samples sin(i*2*pi/len) (scale stays 1),
 * with sample len = sample 0; the interpolated read of getOutput (:84-95)
 * after updatePhase (:31).  Samples are evaluated where read, with the
 * statement the table was built from. */
static double wt_sample(int i, int len) {
  if (i == len) i = 0;
  return 1.0 * orc_sin((double)i * 2. * 3.14159265358979323846 / len);
}
static double wt_process(double *phasor, double incr, int len) {
  *phasor += incr;
  if (*phasor >= 1.) *phasor -= 1.;
  double temp = *phasor * len;
  int ip = (int)temp;
  double frac = temp - ip;
  double s0 = wt_sample(ip, len), s1 = wt_sample(ip + 1, len);
  return s0 + (s1 - s0) * frac;
}
static double clampd(double lo, double hi, double v) { /* std::max(lo, std::min(hi, v)) */
  double m = (v < hi) ? v : hi;
  return (lo < m) ? m : lo;
}

/* SineDynamic(Trend)::updateParams (DataSource.cpp:802-813, :1002-1015): a
 * +-step random walk of mu, amp, freq per component, clamped to the ranges;
 * the steps' signs are bits 3c, 3c+1, 3c+2 of the slot-0 block's word 3 */
static void sd_update(const double *p, double *ax, uint32_t bits) {
  int C = (int)p[0];
  for (int c = 0; c < C; ++c) {
    const double *r = p + 3 + C + 9 * c;  /* freqRange, muRange, ampRange */
    double *a = ax + 4 * c;             /* phasor, freq, mu, amp */
    a[2] = clampd(r[3], r[4], a[2] + (((bits >> (3 * c)) & 1) ? r[5] : -r[5]));
    a[3] = clampd(r[6], r[7], a[3] + (((bits >> (3 * c + 1)) & 1) ? r[8] : -r[8]));
    a[1] = clampd(r[0], r[1], a[1] + (((bits >> (3 * c + 2)) & 1) ? r[2] : -r[2]));
  }
}
/* freq, mu, amp of every component ~ U[lo, hi] (initParams :777-782, reset
 * :794-800), from the slot 16 + c block of the tick */
static void sd_sample(const double *p, double *ax, uint64_t seed, uint64_t env, uint32_t asset,
                      uint64_t tick) {
  int C = (int)p[0];
  for (int c = 0; c < C; ++c) {
    const double *r = p + 3 + C + 9 * c;
    uint32_t x[4];
    block_at(seed, env, asset, 16u + (uint32_t)c, tick, x);
    ax[4 * c + 1] = (r[1] - r[0]) * ((double)x[0] * TWO_M32) + r[0];
    ax[4 * c + 2] = (r[4] - r[3]) * ((double)x[1] * TWO_M32) + r[3];
    ax[4 * c + 3] = (r[7] - r[6]) * ((double)x[2] * TWO_M32) + r[6];
  }
}
static void src_get_data(orc_batch *b, int e) {
  orc_env *s = &b->envs[e];
  if (b->replay) {
    h_get_data(b, s);
    return;
  }
  uint64_t genv = (uint64_t)(b->cfg.env_offset + e);
  uint64_t seed = b->cfg.seed;
  uint64_t tick = s->ts + s->dskip;  /* the draw index (variates v3) */
  for (int i = 0; i < b->A; ++i) {
    const double *p = b->src[i].p;
    switch (b->src[i].kind) {
      case ORC_SRC_SINE: { /* Synth::getData, DataSource.cpp:535-543 */
        double noise = 0.0;
        if (p[5] != 0.0) noise = orc_normal(seed, genv, (uint32_t)i, tick) * p[5] + 0.0;
        const double PI2 = 3.141592653589793238463 * 2;
        s->P[i] = noise + p[1] + p[2] * orc_sin(PI2 * s->x[i] * p[0]);
        s->x[i] += p[4];
        break;
      }
      case ORC_SRC_OU: { /* OU::getData, DataSource.cpp:1173-1180 */
        double z = orc_normal(seed, genv, (uint32_t)i, tick) * 1.0 + 0.0;
        double x = s->P[i];
        x += (p[1] * (p[0] - x)) + p[0] * p[2] * z;
        s->P[i] = x;
        break;
      }
      case ORC_SRC_TRENDOU: { /* TrendOU::getData, DataSource.cpp:1457-1493 */
        double y = s->P[i];
        double z, u_trend;
        uint32_t dbit;
        orc_draw0(seed, genv, (uint32_t)i, tick, &z, &u_trend, &dbit);
        if (s->trending[i]) {
          double n = z * p[8] + 0.0;
          y += y * (s->dY[i] * (double)s->dir[i] + n);
          s->tlen[i] -= 1;
          if (s->tlen[i] == 0) {
            s->trending[i] = 0;
            s->ouMean[i] = y;
          }
          y = (0.01 < y) ? y : 0.01;   /* std::max(0.01, y) */
          if (y <= .1) s->dir[i] = 1;
        } else {
          double n = z * p[7] + 0.0;
          double ou_noise = y * n;
          double ou_reverting_component = p[6] * (s->ouMean[i] - y);
          y += ou_reverting_component + ou_noise;
          if (u_trend < p[0]) {
            double u_len, u_dy;
            orc_uniform2(seed, genv, (uint32_t)i, 1, tick, &u_len, &u_dy);
            s->trending[i] = 1;
            s->dir[i] = dbit ? -1 : 1;
            int32_t lo = (int32_t)p[1], hi = (int32_t)p[2];
            int32_t len = lo + (int32_t)(u_len * (double)(hi - lo + 1));
            if (len > hi) len = hi;
            s->tlen[i] = len;
            s->dY[i] = (p[4] - p[3]) * u_dy + p[3];
          }
        }
        s->P[i] = y;
        break;
      }
      case ORC_SRC_SIMPLETREND: { /* SimpleTrend::getData, DataSource.cpp:1322-1347 */
        double y = s->P[i];
        double z, u_trend;
        uint32_t dbit;
        orc_draw0(seed, genv, (uint32_t)i, tick, &z, &u_trend, &dbit);
        if (s->trending[i]) {
          y += y * s->dY[i] * (double)s->dir[i];
          if (--s->tlen[i] == 0) s->trending[i] = 0;
        } else if (u_trend < p[0]) {
          double u_len, u_dy;
          orc_uniform2(seed, genv, (uint32_t)i, 1, tick, &u_len, &u_dy);
          s->trending[i] = 1;
          s->dir[i] = dbit ? -1 : 1;
          int32_t lo = (int32_t)p[1], hi = (int32_t)p[2];
          int32_t len = lo + (int32_t)(u_len * (double)(hi - lo + 1));
          if (len > hi) len = hi;
          s->tlen[i] = len;
          s->dY[i] = (p[6] - p[5]) * u_dy + p[5];
        }
        if (y <= .1) s->dir[i] = 1;
        y += y * (z * p[3] + 0.0);
        s->P[i] = (0.01 < y) ? y : 0.01;   /* std::max(0.01, y) */
        break;
      }
      case ORC_SRC_TRENDYOU: { /* TrendyOU::getData, DataSource.cpp:1608-1640;
                                  x = ouComponent, ouMean = trendComponent */
        double z, u_trend;
        uint32_t dbit;
        orc_draw0(seed, genv, (uint32_t)i, tick, &z, &u_trend, &dbit);
        double ou_noise = s->ouMean[i] * (z * p[7] + 0.0);
        double ou_rev = p[6] * (-s->x[i]);
        s->x[i] += ou_rev + ou_noise;
        int32_t lo = (int32_t)p[1], hi = (int32_t)p[2];
        if (s->trending[i]) {
          double tc = s->ouMean[i];
          tc += tc * (s->dY[i] * (double)s->dir[i]);
          tc = (0.1 < tc) ? tc : 0.1;       /* std::max(0.1, .) */
          if (tc <= .1) {                    /* floored: restart the up-trend */
            double u_len, u_dy;
            orc_uniform2(seed, genv, (uint32_t)i, 1, tick, &u_len, &u_dy);
            s->dir[i] = 1;
            s->trending[i] = 1;
            int32_t len = lo + (int32_t)(u_len * (double)(hi - lo + 1));
            s->tlen[i] = len > hi ? hi : len;
          }
          s->ouMean[i] = tc;
          if (--s->tlen[i] == 0) s->trending[i] = 0;
        } else if (u_trend < p[0]) {
          double u_len, u_dy;
          orc_uniform2(seed, genv, (uint32_t)i, 1, tick, &u_len, &u_dy);
          s->trending[i] = 1;
          s->dir[i] = dbit ? -1 : 1;
          int32_t len = lo + (int32_t)(u_len * (double)(hi - lo + 1));
          s->tlen[i] = len > hi ? hi : len;
          s->dY[i] = (p[4] - p[3]) * u_dy + p[3];
        }
        s->P[i] = s->x[i] + s->ouMean[i];
        break;
      }
      case ORC_SRC_GAUSSIAN: /* Gaussian::getData, DataSource.cpp:1108-1114 */
        s->P[i] = orc_normal(seed, genv, (uint32_t)i, tick) * p[1] + p[0];
        break;
      case ORC_SRC_SAWTOOTH: { /* SawTooth::getData, DataSource.cpp:557-566 */
        double noise = 0.0;
        if (p[5] != 0.0) noise = orc_normal(seed, genv, (uint32_t)i, tick) * p[5] + 0.0;
        double ip;
        s->P[i] = noise + p[1] + p[2] * modf(s->x[i] * p[0], &ip);
        s->x[i] += p[4];
        break;
      }
      case ORC_SRC_TRIANGLE: { /* Triangle::getData, DataSource.cpp:568-577 */
        double noise = 0.0;
        if (p[5] != 0.0) noise = orc_normal(seed, genv, (uint32_t)i, tick) * p[5] + 0.0;
        const double PI2 = 3.141592653589793238463 * 2;
        s->P[i] = noise + p[1] + 4 * p[2] / PI2 * orc_asin(orc_sin(PI2 * s->x[i] / p[0]));
        s->x[i] += p[4];
        break;
      }
      case ORC_SRC_OUPAIR: { /* OUPair::getData, DataSource.cpp:1236-1244: both assets
                                share mean (kept in ouMean of each; the mean's variate is
                                keyed by the pair's first asset, counter slot 2) */
        if (p[3] == 0.0) {
          const uint32_t a0 = (uint32_t)i;
          uint32_t xm[4];
          block_at(seed, genv, a0, 2, tick, xm);
          const double zm = normal_of(xm);
          double mean = s->ouMean[i];
          mean += mean * (zm * p[2] + 0.0);
          for (int j = 0; j < 2; ++j) {
            const double *pj = b->src[i + j].p;
            double zj = orc_normal(seed, genv, (uint32_t)(i + j), tick) * pj[1] + 0.0;
            double x = s->P[i + j];
            x += (pj[0] * (mean - x)) + mean * zj;
            s->P[i + j] = x;
            s->ouMean[i + j] = mean;
          }
        }
        break;
      }
      case ORC_SRC_SINEADDER: { /* SineAdder::getData, DataSource.cpp:663-673 */
        double *ax = b->aux + ((size_t)e * b->A + i) * ORC_AUX_WIDTH;
        const int C = (int)p[0];
        const double PI2 = 3.141592653589793238463 * 2;
        double sum = 0.;
        for (int c = 0; c < C; ++c) {
          double nz = 0.0;  /* component c's noise: the block of counter slot c */
          if (p[2] != 0.0) {
            uint32_t xc[4];
            block_at(seed, genv, (uint32_t)i, (uint32_t)c, tick, xc);
            nz = normal_of(xc) * p[2] + 0.0;
          }
          sum += (nz + p[3 + C + c]) + p[3 + 2 * C + c] * orc_sin(PI2 * ax[c] * p[3 + c]);
          ax[c] += p[1];
        }
        s->P[i] = sum;
        break;
      }
      case ORC_SRC_SINEDYNAMIC:    /* SineDynamic::getData, DataSource.cpp:829-841 */
      case ORC_SRC_SINEDYNTREND: { /* SineDynamicTrend::getData, :1017-1047 */
        double *ax = b->aux + ((size_t)e * b->A + i) * ORC_AUX_WIDTH;
        const int C = (int)p[0];
        const int trend = b->src[i].kind == ORC_SRC_SINEDYNTREND;
        uint32_t x0[4];
        block_at(seed, genv, (uint32_t)i, 0, tick, x0);
        sd_update(p, ax, x0[3]);
        double tc = ax[16];
        double sum = 0.;
        for (int c = 0; c < C; ++c) {
          double *a = ax + 4 * c;
          double out = wt_process(&a[0], a[1] / p[1], (int)p[3 + c]);  /* setFreq(freq / sampleRate) */
          if (trend) sum += tc * (a[2] + a[3] * out);
          else sum += a[2] + a[3] * out;
        }
        double nz = 0.0;
        if (p[2] != 0.0) nz = normal_of(x0) * p[2] + 0.0;
        if (!trend) {
          s->P[i] = sum + nz;
          break;
        }
        const double *tp = p + 3 + 10 * C;  /* T, then per trend {minLen, maxLen, incr, prob} */
        const int T = (int)tp[0];
        uint32_t x1[4];
        int have1 = 0;
        for (int t = 0; t < T; ++t) {
          const double *q = tp + 1 + 4 * t;
          double *st = ax + 17 + 3 * t;  /* trending, direction, length */
          if (st[0] != 0.) {
            tc += (tc * q[2]) * st[1];
            st[2] -= 1.;
            if (st[2] == 0.) st[0] = 0.;
          } else {
            if (!have1) { block_at(seed, genv, (uint32_t)i, 1, tick, x1); have1 = 1; }
            double u = (double)x1[t] * TWO_M32;
            if (u < q[3]) {
              st[0] = 1.;
              st[1] = ((x0[3] >> (12 + t)) & 1) ? -1. : 1.;
              int lo = (int)q[0], hi = (int)q[1];
              int len = lo + (int)(((double)x1[2 + t] * TWO_M32) * (double)(hi - lo + 1));
              st[2] = (double)(len > hi ? hi : len);
            }
          }
          if (tc <= .1) st[1] = 1.;
          tc = (0.01 < tc) ? tc : 0.01;
        }
        ax[16] = tc;
        s->P[i] = (sum + tc) + tc * nz;
        break;
      }
      default: /* external replay: prices supplied via orc_set_prices */
        s->P[i] = b->ext[(size_t)e * b->A + i];
        break;
    }
  }
  s->ts += 1;  /* timestamp_ += 1 (Composite and children tick together) */
}

/* DataSource::reset: OU no-op (DataSource.h:466), Synth no-op (:232),
 * TrendOU restores start (DataSource.cpp:1495-1502). */
static void src_reset(orc_batch *b, int e) {
  orc_env *s = &b->envs[e];
  s->dskip += 1;  /* every Env::reset skips one draw index (variates v3) */
  for (int i = 0; i < b->A; ++i) {
    const double *p = b->src[i].p;
    switch (b->src[i].kind) {
      case ORC_SRC_TRENDOU:
        s->trending[i] = 0;
        s->P[i] = p[5];
        s->tlen[i] = 0;
        s->ouMean[i] = p[5];
        break;
      case ORC_SRC_SIMPLETREND: /* DataSource.cpp:1349-1356 */
        s->P[i] = p[4]; s->trending[i] = 0; s->dir[i] = 1; s->tlen[i] = 0;
        break;
      case ORC_SRC_TRENDYOU:    /* DataSource.cpp:1642-1653 */
        s->x[i] = 0.; s->ouMean[i] = p[5]; s->trending[i] = 0; s->P[i] = p[5]; s->tlen[i] = 0;
        break;
      case ORC_SRC_OUPAIR:      /* DataSource.cpp:1246-1250 */
        s->P[i] = 10.; s->ouMean[i] = 10.;
        break;
      case ORC_SRC_SINEDYNAMIC: case ORC_SRC_SINEDYNTREND:  /* :794-800, :994-1000 */
        sd_sample(p, b->aux + ((size_t)e * b->A + i) * ORC_AUX_WIDTH, b->cfg.seed,
                  (uint64_t)(b->cfg.env_offset + e), (uint32_t)i, s->ts + s->dskip);
        break;
      default: break;           /* Synth family, SineAdder, OU, Gaussian: no-op */
    }
  }
}

/* source construction (initParams) */
static void src_init(orc_batch *b, int e) {
  orc_env *s = &b->envs[e];
  for (int i = 0; i < b->A; ++i) {
    const double *p = b->src[i].p;
    s->dir[i] = 1;
    switch (b->src[i].kind) {
      case ORC_SRC_SINE: s->x[i] = p[3]; s->P[i] = 0.0; break;        /* :466 */
      case ORC_SRC_OU: s->P[i] = p[0]; break;                           /* :1128 */
      case ORC_SRC_TRENDOU:                                             /* :1380-1400, quirk 1 fixed */
        s->P[i] = p[5]; s->ouMean[i] = p[5]; s->dir[i] = 1; s->tlen[i] = 0;
        s->dY[i] = 0.; s->trending[i] = 0; break;
      case ORC_SRC_SIMPLETREND:                                         /* :1262-1276 */
        s->P[i] = p[4]; s->tlen[i] = 0; s->dY[i] = 0.; s->trending[i] = 0; break;
      case ORC_SRC_TRENDYOU:                                            /* :1528-1545, quirk 1 fixed */
        s->P[i] = p[5]; s->ouMean[i] = p[5]; s->x[i] = 0.; s->tlen[i] = 0;
        s->dY[i] = 0.; s->trending[i] = 0; break;
      case ORC_SRC_GAUSSIAN: s->P[i] = p[0]; break;                     /* :1067 */
      case ORC_SRC_SAWTOOTH: case ORC_SRC_TRIANGLE: s->x[i] = p[3]; s->P[i] = 0.0; break;
      case ORC_SRC_OUPAIR: s->P[i] = 10.; s->ouMean[i] = 10.; break;   /* :1191-1196 */
      case ORC_SRC_SINEADDER: {                                         /* :645-661: x = phase */
        double *ax = b->aux + ((size_t)e * b->A + i) * ORC_AUX_WIDTH;
        const int C = (int)p[0];
        for (int c = 0; c < C; ++c) ax[c] = p[3 + 3 * C + c];
        s->P[i] = 0.0;
        break;
      }
      case ORC_SRC_SINEDYNAMIC: case ORC_SRC_SINEDYNTREND: {            /* :742-792, :925-992 */
        double *ax = b->aux + ((size_t)e * b->A + i) * ORC_AUX_WIDTH;
        for (int k = 0; k < ORC_AUX_WIDTH; ++k) ax[k] = 0.;
        sd_sample(p, ax, b->cfg.seed, (uint64_t)(b->cfg.env_offset + e), (uint32_t)i, 0);
        ax[16] = 1.;                                                    /* trendComponent */
        for (int t = 0; t < 2; ++t) ax[18 + 3 * t] = 1.;                /* currentDirection */
        s->P[i] = 0.0;
        break;
      }
      default: s->P[i] = 0.0; break;
    }
  }
  s->ts = 0;
  s->dskip = 0;
}

/* Env::initAccountants -- Env.h:150-165: fresh Broker/Portfolio, one getData */
static void env_init_accountants(orc_batch *b, int e) {
  orc_env *s = &b->envs[e];
  for (int i = 0; i < b->A; ++i) { s->L[i] = 0.; s->mep[i] = 0.; s->Bm[i] = 0.; }
  s->cash = b->cfg.init_cash;
  src_get_data(b, e);
}

/* ---- window (StackerDiscrete) ------------------------------------------- */

/* deque.append on env e's ring (preprocessor.py:172-175) */
static void ring_push_one(const orc_ring *r, int e, const double *price, const double *port,
                          uint64_t ts) {
  int W = r->window, C = r->n_price + r->n_port;
  int h = (r->head[e] + 1) % W;
  double *row = r->ring + ((size_t)e * W + h) * C;
  for (int i = 0; i < r->n_price; ++i) row[i] = price ? price[i] : 0.;
  for (int i = 0; i < r->n_port; ++i) row[r->n_price + i] = port ? port[i] : 0.;
  r->ring_ts[(size_t)e * W + h] = ts;
  r->head[e] = h;
  if (r->len[e] < W) r->len[e]++;
}

static void ring_clear_one(const orc_ring *r, int e) { /* reset_state, preprocessor.py:196-199 */
  r->len[e] = 0;
  r->head[e] = r->window - 1;
}

static void window_stream(orc_batch *b, int e) {
  if (b->cfg.window <= 0) return;
  orc_env *s = &b->envs[e];
  double port[MAXA + 1];
  p_ledger_normed_full(s, b->A, port);
  ring_push_one(&b->ring, e, state_price(b, s), port, s->ts);
}

static void window_clear(orc_batch *b, int e) {
  if (b->cfg.window > 0) ring_clear_one(&b->ring, e);
}

/* Agent reset: env.reset(); preprocessor.reset_state(); stream_state(state);
 * initialize_history(env) -- offpolicy_q.py:93-99, preprocessor.py:191-194 */
static void env_reset_one(orc_batch *b, int e) {
  src_reset(b, e);
  env_init_accountants(b, e);
  if (b->cfg.window > 0) {
    window_clear(b, e);
    window_stream(b, e);
    while (b->ring.len[e] < b->cfg.window) {
      src_get_data(b, e);  /* Env::step() with no action: only the tick matters */
      window_stream(b, e);
    }
  }
}

/* ---- shapers (nstep_buffer.py) ------------------------------------------ */

static const double ORC_EPS = 1.1920928955078125e-07; /* np.finfo(np.float32).eps, :20 */

static double dsr_one(double r, double A, double B) { /* _DSR.calculate_dsr :80-85 */
  double dA = r - A;
  double dB = r * r - B;
  double t = B - A * A;
  return (B * dA - (A * dB) / 2) / (pow(t * t, 3.0 / 4.0) + ORC_EPS);
}
static double ddr_one(double r, double A, double B) { /* _DDR.calculate_ddr :146-156 */
  if (r > 0.) return (r - A / 2) / (sqrt(B) + ORC_EPS);
  return (B * (r - A / 2) - (A * (r * r)) / 2) / (pow(B, 3.0 / 2.0) + ORC_EPS);
}
static double clip1(double v) { /* np.clip(v, -1, 1) */
  if (v < -1.) return -1.;
  if (v > 1.) return 1.;
  return v;
}

void orc_dsr(const double *rewards, int L, int D, const double *discounts, double eta,
             double *A, double *B, double *out) {
  for (int d = 0; d < D; ++d) {
    double acc = 0.0;
    for (int k = 0; k < L; ++k) acc += discounts[k] * dsr_one(rewards[k * D + d], A[d], B[d]);
    out[d] = clip1(acc / L);
    double r0 = rewards[d];                     /* update_parameters :87-91 */
    A[d] += eta * (r0 - A[d]);
    B[d] += eta * (r0 * r0 - B[d]);
  }
}

void orc_ddr(const double *rewards, int L, int D, const double *discounts, double eta,
             double *A, double *B, double *out) {
  for (int d = 0; d < D; ++d) {
    double acc = 0.0;
    for (int k = 0; k < L; ++k) acc += discounts[k] * ddr_one(rewards[k * D + d], A[d], B[d]);
    out[d] = clip1(acc / L);
    double r0 = rewards[d];                     /* update_parameters :158-162 */
    double m = r0 < 0. ? r0 : 0.;               /* np.minimum(r, 0.) */
    if (r0 != r0) m = r0;
    A[d] += eta * (r0 - A[d]);
    B[d] += eta * (m * m - B[d]);
  }
}

/* cosine_similarity (nstep_buffer.py:173-178) over the A+1 entries of
 * ledgerNormedFull: canonical order = entry 0 (cash) + tree over the A assets. */
static double sum_full(const double *v, int n) { return v[0] + orc_canon_sum(v + 1, n - 1); }
static double cosine_sim(const double *p, const double *q, int n) {
  double pp[MAXA + 1], qq[MAXA + 1], pq[MAXA + 1];
  for (int i = 0; i < n; ++i) { pp[i] = p[i] * p[i]; qq[i] = q[i] * q[i]; pq[i] = p[i] * q[i]; }
  double norm_p = sqrt(sum_full(pp, n));
  double norm_q = sqrt(sum_full(qq, n));
  return sum_full(pq, n) / (norm_p * norm_q);
}

/* cosine_port_shaper (nstep_buffer.py:182-204) over an n-step window:
 * rewards (L,D), ports (L,P) = next_state.portfolio[-1] rows, target (P). */
void orc_ppc(const double *rewards, const double *ports, int L, int D, int P, const double *target,
             double temp, const double *discounts, double *out) {
  for (int d = 0; d < D; ++d) out[d] = 0.0;
  for (int k = 0; k < L; ++k) {
    double cs = cosine_sim(ports + (size_t)k * P, target, P);
    for (int d = 0; d < D; ++d) out[d] += discounts[k] * (rewards[k * D + d] + temp * cs);
  }
}

/* ---- naive n-step shapers (nstep_buffer.py:207-312), benchmark = 0. -------- */

/* x**e and x**(1/e) as numpy evaluates them on float64 arrays: the scalar
 * exponents 2 and 0.5 take numpy's square / sqrt fast paths (equal to the
 * correctly rounded pow); other exponents go through pow. */
static double pow_e(double x, double e) { return e == 2.0 ? x * x : pow(x, e); }
static double root_e(double x, double e) { return e == 2.0 ? sqrt(x) : pow(x, 1.0 / e); }
static double max_m1(double x) { return (x < -1.) ? -1. : x; }           /* np.clip(x, -1, None) */
static double min_0(double x) { return (x < 0. || x != x) ? x : 0.; }   /* np.minimum(x, 0.) */

void orc_naive(int shaper, const double *rewards, int L, int D, const double *discounts,
               double ex, double *out) {
  for (int d = 0; d < D; ++d) {
    if (L == 1) {  /* the len(nstep_buffer) == 1 heuristics */
      double diff = rewards[d] - 0.;
      if (shaper == ORC_SHAPER_SHARPE) {                     /* :212-216 (no clip; r = 0 -> nan) */
        diff = (diff != 0.) ? diff : 0.;
        out[d] = diff / sqrt(diff * diff);
      } else if (shaper == ORC_SHAPER_SORTINO_A) {           /* :244-249 */
        double downside = root_e(pow_e(fabs(diff), ex), ex);
        out[d] = clip1(0.1 * ((diff != 0.) ? diff / downside : 0.));
      } else {                                               /* sortino_shaperB :286-291 */
        diff = max_m1(diff);
        diff = (diff < 0.) ? -root_e(-diff, ex) : diff;
        out[d] = clip1(diff);
      }
      continue;
    }
    double diffs[ORC_MAX_NSTEP];
    for (int k = 0; k < L; ++k) diffs[k] = (rewards[(size_t)k * D + d] - 0.) * discounts[k];
    if (shaper == ORC_SHAPER_SHARPE) {                       /* :217-239 */
      double s = 0., s2 = 0.;
      for (int k = 0; k < L; ++k) s += diffs[k];
      for (int k = 0; k < L; ++k) s2 += diffs[k] * diffs[k];
      double num = s / L;
      double denom = sqrt(s2 / (L - 1));
      double o = (denom != 0.) ? num / denom : 0.;           /* np.divide(..., where=denom != 0) */
      out[d] = clip1(.1 * o);
    } else if (shaper == ORC_SHAPER_SORTINO_A) {             /* :251-272 */
      double s = 0., den = 0.;
      for (int k = 0; k < L; ++k) s += diffs[k];
      double num = s / L;
      for (int k = 0; k < L; ++k) {
        double down = max_m1(min_0(diffs[k]));
        den += root_e(pow_e(fabs(down), ex) / (L - 1), ex);
      }
      out[d] = (den != 0.) ? clip1(.1 * (num / den)) : ((num == 0.) ? 0. : 1.);
    } else {                                                 /* sortino_shaperB :293-312 */
      double s = 0.;
      for (int k = 0; k < L; ++k) {
        double v = max_m1(diffs[k]);
        s += (v < 0.) ? -root_e(-v, ex) : v;
      }
      out[d] = clip1(s);
    }
  }
}

static int is_naive(int shaper) {
  return shaper == ORC_SHAPER_SHARPE || shaper == ORC_SHAPER_SORTINO_A ||
         shaper == ORC_SHAPER_SORTINO_B;
}

/* ---- public API ---------------------------------------------------------- */

orc_batch *orc_create(const orc_config *cfg, const orc_asset_src *srcs) {
  if (cfg->n_assets < 1 || cfg->n_assets > MAXA || cfg->n_envs < 1) return NULL;
  if (cfg->nstep < 1 || cfg->nstep > ORC_MAX_NSTEP) return NULL;
  orc_batch *b = (orc_batch *)calloc(1, sizeof(orc_batch));
  b->cfg = *cfg;
  b->N = cfg->n_envs;
  b->A = cfg->n_assets;
  memcpy(b->src, srcs, sizeof(orc_asset_src) * (size_t)b->A);
  b->envs = (orc_env *)calloc((size_t)b->N, sizeof(orc_env));
  b->replay = srcs[0].kind == ORC_SRC_REPLAY;
  b->F = (b->replay && cfg->n_feats > 0) ? cfg->n_feats : b->A;
  b->ext = (double *)calloc((size_t)b->N * b->A, sizeof(double));
  for (int i = 0; i < b->A; ++i)
    if (srcs[i].kind >= ORC_SRC_SINEADDER && !b->aux)
      b->aux = (double *)calloc((size_t)b->N * b->A * ORC_AUX_WIDTH, sizeof(double));
  {
    int D = (cfg->reward_mode == ORC_REWARD_AGENT_PER_ASSET) ? b->A : 1;
    b->nring = (double *)calloc((size_t)b->N * cfg->nstep * D, sizeof(double));
    b->nlen = (int32_t *)calloc((size_t)b->N, sizeof(int32_t));
    for (int i = 0; i < cfg->nstep; ++i) b->disc[i] = pow(cfg->discount, (double)i); /* :328 */
  }
  int W = cfg->window;
  if (W > 0) {
    orc_ring *r = &b->ring;
    r->n_envs = b->N; r->n_price = b->F; r->n_port = b->A + 1; r->window = W;
    r->norm_type = cfg->norm_type;
    r->ring = (double *)calloc((size_t)b->N * W * (b->F + b->A + 1), sizeof(double));
    r->ring_ts = (uint64_t *)calloc((size_t)b->N * W, sizeof(uint64_t));
    r->head = (int32_t *)calloc((size_t)b->N, sizeof(int32_t));
    r->len = (int32_t *)calloc((size_t)b->N, sizeof(int32_t));
  }
  for (int e = 0; e < b->N; ++e) {
    window_clear(b, e);
    src_init(b, e);               /* Env::initMembers -> makeDataSource (Env.h:139-148) */
    if (!b->replay) env_init_accountants(b, e);   /* -> initAccountants (one getData) */
  }
  return b;
}

int64_t orc_set_replay(orc_batch *b, const double *price, const double *feats, const uint64_t *ts,
                       int64_t T, int64_t first, int64_t second, int64_t cache_size,
                       int64_t stride) {
  if (!b->replay || T < 1 || first < 0 || second > T || second - first < 1) return -1;
  free(b->rp_price); free(b->rp_feat); free(b->rp_ts);
  b->rp_price = (double *)malloc(sizeof(double) * (size_t)T * b->A);
  b->rp_feat = (double *)malloc(sizeof(double) * (size_t)T * b->F);
  b->rp_ts = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)T);
  memcpy(b->rp_price, price, sizeof(double) * (size_t)T * b->A);
  memcpy(b->rp_feat, feats, sizeof(double) * (size_t)T * b->F);
  memcpy(b->rp_ts, ts, sizeof(uint64_t) * (size_t)T);
  b->rp_T = T; b->rp_first = first; b->rp_second = second;
  int64_t full = second - first;
  b->rp_cs = cache_size < full ? (cache_size < 1 ? 1 : cache_size) : full; /* :299 */
  /* the period: getData calls until the source is back in its init() state */
  orc_env probe;
  memset(&probe, 0, sizeof probe);
  probe.h_idx = first; probe.h_cidx = 0;
  h_load(b, &probe);
  int64_t period = 0, prev = -1;
  for (;;) {
    orc_env t = probe;
    h_get_data(b, &t);
    int64_t row = t.h_cstart + t.h_cidx - 1;
    if (row <= prev) break;
    prev = row;
    probe = t;
    period++;
  }
  for (int e = 0; e < b->N; ++e) {
    orc_env *s = &b->envs[e];
    s->h_idx = first; s->h_cidx = 0;      /* HDFSourceSingle::init -> loadData */
    h_load(b, s);
    uint64_t g = (uint64_t)(b->cfg.env_offset + e);
    int64_t skip = (int64_t)((g * (uint64_t)stride) % (uint64_t)period);
    for (int64_t j = 0; j < skip; ++j) h_get_data(b, s);
    env_init_accountants(b, e);
  }
  return period;
}

void orc_destroy(orc_batch *b) {
  if (!b) return;
  free(b->ring.ring); free(b->ring.ring_ts); free(b->ring.head); free(b->ring.len);
  free(b->envs);
  free(b->ext);
  free(b->aux);
  free(b->rp_price); free(b->rp_feat); free(b->rp_ts);
  free(b->nring);
  free(b->nlen);
  free(b);
}

void orc_reset(orc_batch *b, const uint8_t *mask) {
  for (int e = 0; e < b->N; ++e)
    if (!mask || mask[e]) env_reset_one(b, e);
}

void orc_set_prices(orc_batch *b, const double *prices) {
  memcpy(b->ext, prices, sizeof(double) * (size_t)b->N * b->A);
}

/* Env::setDataSource (Env.h:174-179): the new source replaces the old one;
 * the Broker / Portfolio stay, and the Broker's price map now points at the
 * new source's currentPrices() (Broker.cpp:68-76), loaded here as P. */
void orc_set_sources(orc_batch *b, const orc_asset_src *srcs, const double *prices) {
  memcpy(b->src, srcs, sizeof(orc_asset_src) * (size_t)b->A);
  if (prices)
    for (int e = 0; e < b->N; ++e)
      memcpy(b->envs[e].P, prices + (size_t)e * b->A, sizeof(double) * (size_t)b->A);
}

/* agent per-asset reward: offpolicy_q.py:152-164 */
static void agent_reward(const orc_env *s, int A, const double *prevVal, double prevEq,
                         const double *tp, const double *tu, const double *tc, double *r) {
  for (int i = 0; i < A; ++i) {
    double curr = s->L[i] * s->P[i];
    double mar_diff = tu[i] * tp[i] + tc[i];
    double v = ((curr - prevVal[i]) - mar_diff) / prevEq;
    v += 1;
    v = (v < .35) ? .35 : v;  /* np.maximum(reward, .35) */
    if (v != v) v = NAN;
    r[i] = log(v);
  }
}

/* NStepBuffer semantics as ReplayBuffer.add drives them (replay_buffer.py:68-80):
 * append; if full (len >= n) pop one; if done pop until empty.  Each pop
 * aggregates the whole buffer (len L) with discounts[:L]
 * (nstep_buffer.py:337-356) -- DSR/DDR: clip(sum_k gamma^k f(r_k) / L) then
 * update A,B from the oldest reward (:62-77, :128-142); PPC: sum_k gamma^k
 * (r_k + temp*cos_k) (:182-204); none: sum_k r_k gamma^k (:23-27) -- and
 * drops the oldest entry.  Returns the number of pops; out is (pops, D). */
static int nstep_add(orc_batch *b, int e, int D, const double *rin, const double *port, int done,
                     double *out) {
  const orc_config *c = &b->cfg;
  orc_env *s = &b->envs[e];
  int n = c->nstep;
  double *ring = b->nring + (size_t)e * n * D;
  int L = b->nlen[e];
  double cs = 0.;
  if (c->shaper == ORC_SHAPER_PPC) cs = cosine_sim(port, c->desired_portfolio, b->A + 1);
  for (int d = 0; d < D; ++d)
    ring[(size_t)L * D + d] = (c->shaper == ORC_SHAPER_PPC) ? rin[d] + c->cosine_temp * cs : rin[d];
  L += 1;
  int pops = 0;
  while (L >= n || (done && L > 0)) {
    double *o = out + (size_t)pops * D;
    if (c->shaper == ORC_SHAPER_DSR) orc_dsr(ring, L, D, b->disc, c->adaptation_rate, s->sA, s->sB, o);
    else if (c->shaper == ORC_SHAPER_DDR) orc_ddr(ring, L, D, b->disc, c->adaptation_rate, s->sA, s->sB, o);
    else if (is_naive(c->shaper)) orc_naive(c->shaper, ring, L, D, b->disc, c->sortino_exp, o);
    else {
      for (int d = 0; d < D; ++d) {
        double acc = 0.0;
        for (int k = 0; k < L; ++k) acc += b->disc[k] * ring[(size_t)k * D + d];
        o[d] = acc;
      }
    }
    memmove(ring, ring + D, sizeof(double) * (size_t)(L - 1) * D);
    L -= 1;
    pops += 1;
    if (!done && L < n) break;
  }
  b->nlen[e] = L;
  return pops;
}

static void step_one(orc_batch *b, int e, int kind, const double *units, int32_t single_idx,
                     double single_u, const orc_out *o) {
  const orc_config *c = &b->cfg;
  orc_env *s = &b->envs[e];
  const int A = b->A;
  double tp[MAXA], tu[MAXA], tc[MAXA], prevVal[MAXA];
  int risk[MAXA];
  for (int i = 0; i < A; ++i) { tp[i] = 0.; tu[i] = 0.; tc[i] = 0.; risk[i] = ORC_GREEN; }
  for (int i = 0; i < A; ++i) prevVal[i] = s->L[i] * s->P[i];

  double prevEq = p_equity(s, A);                                      /* Env.h:208 */
  if (kind == ORC_STEP_UNITS) {                                        /* Broker.cpp:144-158 */
    for (int i = 0; i < A; ++i) {
      int r;
      b_handle_transaction(c, s, A, i, units[i], &tp[i], &tu[i], &tc[i], &r);
      risk[i] = r;
    }
  } else if (kind == ORC_STEP_SINGLE) {                                /* Env.h:235 */
    int r;
    int i = single_idx;
    b_handle_transaction(c, s, A, i, single_u, &tp[i], &tu[i], &tc[i], &r);
    risk[i] = r;
  }
  /* BrokerResponse.marginCall (Broker.cpp:156-157); Env::step() has none (Env.h:199) */
  int marginCall = (kind != ORC_STEP_NONE) &&
                   p_check_risk(s, A, c->maintenance_margin) == ORC_MARGIN_CALL;
  src_get_data(b, e);                                                  /* Env.h:210 */
  double currentEq = p_equity(s, A);                                   /* :211 */
  double ratio = currentEq / prevEq;
  double clampv = (kind == ORC_STEP_SINGLE) ? 0.01 : 0.3;              /* :212, :238 */
  double reward = log((ratio < clampv) ? clampv : ratio);
  int done = 0;
  int prisk = p_check_risk(s, A, c->maintenance_margin);              /* :215 */
  for (int i = 0; i < A; ++i)
    if (risk[i] != ORC_GREEN && risk[i] != ORC_INSUFF_MARGIN) done = 1;
  if (prisk != ORC_GREEN || p_equity(s, A) < 0.1 * c->init_cash) done = 1;

  /* agent-side reward (offpolicy_q.py:152-164) */
  double ar[MAXA];
  agent_reward(s, A, prevVal, prevEq, tp, tu, tc, ar);
  double ar_sum = orc_canon_sum(ar, A);

  /* State.portfolio */
  double port[MAXA + 1];
  p_ledger_normed_full(s, A, port);

  /* reward shaping, n = 1 (nstep_buffer.py; replay_buffer.py:68-80) */
  int D = (c->reward_mode == ORC_REWARD_AGENT_PER_ASSET) ? A : 1;
  double rin[MAXA];
  if (c->reward_mode == ORC_REWARD_ENV_LOG) rin[0] = reward;
  else if (c->reward_mode == ORC_REWARD_AGENT_SUM) rin[0] = ar_sum;
  else for (int i = 0; i < A; ++i) rin[i] = ar[i];
  double shaped[ORC_MAX_NSTEP * MAXA];
  int n_shaped = 1;
  if (c->nstep == 1) {
    const double one = 1.0;
    if (c->shaper == ORC_SHAPER_DSR) orc_dsr(rin, 1, D, &one, c->adaptation_rate, s->sA, s->sB, shaped);
    else if (c->shaper == ORC_SHAPER_DDR) orc_ddr(rin, 1, D, &one, c->adaptation_rate, s->sA, s->sB, shaped);
    else if (is_naive(c->shaper)) orc_naive(c->shaper, rin, 1, D, &one, c->sortino_exp, shaped);
    else if (c->shaper == ORC_SHAPER_PPC) {  /* cosine_port_shaper :182-204 */
      double cs = cosine_sim(port, c->desired_portfolio, A + 1);
      for (int d = 0; d < D; ++d) shaped[d] = 1.0 * (rin[d] + c->cosine_temp * cs);
    } else for (int d = 0; d < D; ++d) shaped[d] = rin[d];
  } else {
    n_shaped = nstep_add(b, e, D, rin, port, done, shaped);
  }

  /* outputs */
  size_t eA = (size_t)e * A;
  if (o->reward) o->reward[e] = reward;
  if (o->agent_reward) {
    if (D == 1) o->agent_reward[e] = rin[0];
    else for (int i = 0; i < A; ++i) o->agent_reward[eA + i] = ar[i];
  }
  if (o->shaped) {
    size_t nD = (size_t)c->nstep * D;
    for (size_t j = 0; j < nD; ++j) o->shaped[(size_t)e * nD + j] = j < (size_t)n_shaped * D ? shaped[j] : 0.;
  }
  if (o->n_shaped) o->n_shaped[e] = (uint8_t)n_shaped;
  if (o->done) o->done[e] = (uint8_t)done;
  if (o->obs_price) {
    const double *sp = state_price(b, s);
    for (int f = 0; f < b->F; ++f) o->obs_price[(size_t)e * b->F + f] = sp[f];
  }
  if (o->data_end) o->data_end[e] = (uint8_t)h_data_end(b, s);
  if (o->obs_port) for (int i = 0; i <= A; ++i) o->obs_port[(size_t)e * (A + 1) + i] = port[i];
  if (o->timestamp) o->timestamp[e] = s->ts;
  for (int i = 0; i < A; ++i) {
    if (o->tprice) o->tprice[eA + i] = tp[i];
    if (o->tunits) o->tunits[eA + i] = tu[i];
    if (o->tcost) o->tcost[eA + i] = tc[i];
    if (o->risk) o->risk[eA + i] = (uint8_t)risk[i];
  }
  if (o->margin_call) o->margin_call[e] = (uint8_t)marginCall;

  /* episode statistics */
  s->ep_ret += reward;
  s->ep_len += 1;
  if (done) {
    s->last_ret = s->ep_ret; s->last_len = s->ep_len; s->last_eq = currentEq;
    s->n_done += 1; s->ep_ret = 0; s->ep_len = 0;
  }
  window_stream(b, e);                       /* agent streams next_state (:193) */
  if (done && c->auto_reset) env_reset_one(b, e);  /* agent reset_state (:199-201) */
}

void orc_step(orc_batch *b, int kind, const double *units, const int32_t *asset_idx,
              const orc_out *out) {
  for (int e = 0; e < b->N; ++e) {
    if (kind == ORC_STEP_UNITS) step_one(b, e, kind, units + (size_t)e * b->A, 0, 0., out);
    else if (kind == ORC_STEP_SINGLE) step_one(b, e, kind, NULL, asset_idx[e], units[e], out);
    else step_one(b, e, kind, NULL, 0, 0., out);
  }
}

/* DQN.action_to_transaction -- dqn.py:160-179 */
static void action_to_units_one(const orc_batch *b, int e, const int8_t *act, double *units) {
  const orc_env *s = &b->envs[e];
  int A = b->A;
  double avM = p_available_margin(s, A, b->cfg.required_margin);
  int half = b->cfg.action_atoms / 2;
  for (int i = 0; i < A; ++i) {
    double u = b->cfg.unit_size * avM / s->P[i];
    double centered = (double)(act[i] - half);
    units[i] = centered * u;
    if (act[i] == 0) units[i] = (s->L[i] != 0) ? -s->L[i] : 0.;
  }
}

void orc_action_to_units(orc_batch *b, const int8_t *actions, double *units) {
  for (int e = 0; e < b->N; ++e)
    action_to_units_one(b, e, actions + (size_t)e * b->A, units + (size_t)e * b->A);
}

static double *offs_d(double *p, size_t off) { return p ? p + off : NULL; }
static uint8_t *offs_u8(uint8_t *p, size_t off) { return p ? p + off : NULL; }

static orc_out out_at_step(const orc_batch *b, const orc_out *out, int k) {
  int N = b->N, A = b->A;
  int D = (b->cfg.reward_mode == ORC_REWARD_AGENT_PER_ASSET) ? A : 1;
  size_t nA = (size_t)k * N * A, nN = (size_t)k * N;
  orc_out o = *out;
  o.reward = offs_d(out->reward, nN);
  o.agent_reward = offs_d(out->agent_reward, nN * D);
  o.shaped = offs_d(out->shaped, nN * D * (size_t)b->cfg.nstep);
  o.done = offs_u8(out->done, nN);
  o.obs_price = offs_d(out->obs_price, (size_t)k * N * b->F);
  o.data_end = offs_u8(out->data_end, nN);
  o.obs_port = offs_d(out->obs_port, (size_t)k * N * (A + 1));
  o.timestamp = out->timestamp ? out->timestamp + nN : NULL;
  o.tprice = offs_d(out->tprice, nA);
  o.tunits = offs_d(out->tunits, nA);
  o.tcost = offs_d(out->tcost, nA);
  o.risk = offs_u8(out->risk, nA);
  o.margin_call = offs_u8(out->margin_call, nN);
  o.n_shaped = offs_u8(out->n_shaped, nN);
  return o;
}

/* Envs are independent, so each env runs its k steps on its own; with
 * threads > 1 the envs are split statically over OpenMP threads (CPU
 * baseline on all host cores; results identical to threads == 1). */
void orc_rollout_mt(orc_batch *b, const int8_t *actions, int k_steps, const orc_out *out,
                    int threads) {
  int N = b->N, A = b->A;
#pragma omp parallel for schedule(static) num_threads(threads > 0 ? threads : 1) if (threads > 1)
  for (int e = 0; e < N; ++e) {
    double units[MAXA];
    for (int k = 0; k < k_steps; ++k) {
      orc_out o = out_at_step(b, out, k);
      action_to_units_one(b, e, actions + (size_t)k * N * A + (size_t)e * A, units);
      step_one(b, e, ORC_STEP_UNITS, units, 0, 0., &o);
    }
  }
}

void orc_rollout(orc_batch *b, const int8_t *actions, int k_steps, const orc_out *out) {
  orc_rollout_mt(b, actions, k_steps, out, 1);
}

/* ---- state access -------------------------------------------------------- */

void orc_get_field(const orc_batch *b, int field, double *out) {
  for (int e = 0; e < b->N; ++e) {
    const orc_env *s = &b->envs[e];
    for (int i = 0; i < b->A; ++i) {
      double v = 0.;
      switch (field) {
        case ORC_F_LEDGER: v = s->L[i]; break;
        case ORC_F_MEP: v = s->mep[i]; break;
        case ORC_F_BORROWED: v = s->Bm[i]; break;
        case ORC_F_PRICE: v = s->P[i]; break;
        case ORC_F_SINE_X: v = s->x[i]; break;
        case ORC_F_OU_MEAN: v = s->ouMean[i]; break;
        case ORC_F_DY: v = s->dY[i]; break;
        case ORC_F_TLEN: v = s->tlen[i]; break;
        case ORC_F_TRENDING: v = s->trending[i]; break;
        case ORC_F_DIR: v = s->dir[i]; break;
        case ORC_F_SHAPER_A: v = s->sA[i]; break;
        case ORC_F_SHAPER_B: v = s->sB[i]; break;
      }
      out[(size_t)e * b->A + i] = v;
    }
  }
}

void orc_set_field(orc_batch *b, int field, const double *in) {
  for (int e = 0; e < b->N; ++e) {
    orc_env *s = &b->envs[e];
    for (int i = 0; i < b->A; ++i) {
      double v = in[(size_t)e * b->A + i];
      switch (field) {
        case ORC_F_LEDGER: s->L[i] = v; break;
        case ORC_F_MEP: s->mep[i] = v; break;
        case ORC_F_BORROWED: s->Bm[i] = v; break;
        case ORC_F_PRICE: s->P[i] = v; break;
        case ORC_F_SINE_X: s->x[i] = v; break;
        case ORC_F_OU_MEAN: s->ouMean[i] = v; break;
        case ORC_F_DY: s->dY[i] = v; break;
        case ORC_F_TLEN: s->tlen[i] = (int32_t)v; break;
        case ORC_F_TRENDING: s->trending[i] = (uint8_t)v; break;
        case ORC_F_DIR: s->dir[i] = (int8_t)v; break;
        case ORC_F_SHAPER_A: s->sA[i] = v; break;
        case ORC_F_SHAPER_B: s->sB[i] = v; break;
      }
    }
  }
}

void orc_get_scalar(const orc_batch *b, int which, double *out) {
  const int A = b->A;
  for (int e = 0; e < b->N; ++e) {
    const orc_env *s = &b->envs[e];
    double v = 0.;
    switch (which) {
      case ORC_S_CASH: v = s->cash; break;
      case ORC_S_EQUITY: v = p_equity(s, A); break;
      case ORC_S_PNL: v = p_pnl(s, A); break;
      case ORC_S_BALANCE: v = p_balance(s, A); break;
      case ORC_S_AVAILABLE_MARGIN: v = p_available_margin(s, A, b->cfg.required_margin); break;
      case ORC_S_USED_MARGIN: v = p_used_margin(s, A, b->cfg.required_margin); break;
      case ORC_S_BORROWED_MARGIN: v = p_borrowed_margin(s, A); break;
      case ORC_S_BORROWED_ASSET_VALUE: v = p_borrowed_asset_value(s, A); break;
      case ORC_S_ASSET_VALUE: v = p_asset_value(s, A); break;
      case ORC_S_TIMESTAMP: v = (double)s->ts; break;
      case ORC_S_CHECK_RISK: v = p_check_risk(s, A, b->cfg.maintenance_margin); break;
      case ORC_S_SHAPER_A: v = s->sA[0]; break;
      case ORC_S_SHAPER_B: v = s->sB[0]; break;
      case ORC_S_EP_RET: v = s->ep_ret; break;
      case ORC_S_EP_LEN: v = s->ep_len; break;
      case ORC_S_LAST_RET: v = s->last_ret; break;
      case ORC_S_LAST_LEN: v = s->last_len; break;
      case ORC_S_LAST_EQUITY: v = s->last_eq; break;
      case ORC_S_N_DONE: v = s->n_done; break;
      case ORC_S_DSKIP: v = (double)s->dskip; break;
    }
    out[e] = v;
  }
}

void orc_set_cash(orc_batch *b, const double *cash) {
  for (int e = 0; e < b->N; ++e) b->envs[e].cash = cash[e];
}

void orc_port_handle_transaction(orc_batch *b, int e, int asset, double tprice, double units,
                                 double cost) {
  p_handle_transaction(&b->envs[e], b->cfg.required_margin, asset, tprice, units, cost);
}
int orc_port_check_risk(const orc_batch *b, int e) {
  return p_check_risk(&b->envs[e], b->A, b->cfg.maintenance_margin);
}
int orc_port_check_risk_order(const orc_batch *b, int e, int asset, double units) {
  return p_check_risk_order(&b->envs[e], b->A, b->cfg.required_margin, b->cfg.maintenance_margin,
                            asset, units);
}
void orc_port_ledger_normed_full(const orc_batch *b, int e, double *out) {
  p_ledger_normed_full(&b->envs[e], b->A, out);
}
void orc_broker_handle_transaction(orc_batch *b, int e, int asset, double units, double *resp) {
  int r;
  b_handle_transaction(&b->cfg, &b->envs[e], b->A, asset, units, &resp[0], &resp[1], &resp[2], &r);
  resp[3] = r;
}

/* Broker::close(assetIdx) -- Broker.cpp:160-169: units = -ledger, slippage
 * and cost as for an order (:171-178), Portfolio::close (Portfolio.cpp:327-333);
 * the response is always green */
void orc_broker_close(orc_batch *b, int e, int asset, double *resp) {
  const orc_config *c = &b->cfg;
  orc_env *s = &b->envs[e];
  double units = -(s->L[asset]);
  double currentPrice = s->P[asset];
  double slippage = (currentPrice * c->slippage_rel) + c->slippage_abs;
  double transactionPrice = units < 0 ? (currentPrice - slippage) : (currentPrice + slippage);
  double transactionCost = fabs(currentPrice * units) * c->tc_rel + c->tc_abs;
  if (s->L[asset] != 0.)
    p_handle_transaction(s, c->required_margin, asset, transactionPrice, -1 * s->L[asset], transactionCost);
  resp[0] = transactionPrice;
  resp[1] = units;
  resp[2] = transactionCost;
  resp[3] = ORC_GREEN;
}

/* Portfolio::close(assetIdx, transactionPrice, transactionCost) -- Portfolio.cpp:327-333 */
void orc_port_close(orc_batch *b, int e, int asset, double tprice, double cost) {
  orc_env *s = &b->envs[e];
  if (s->L[asset] != 0.)
    p_handle_transaction(s, b->cfg.required_margin, asset, tprice, -1 * s->L[asset], cost);
}

/* ---- window output (StackerDiscrete.current_data, preprocessor.py:177-185) */

void orc_window_stream(orc_batch *b) {
  for (int e = 0; e < b->N; ++e) window_stream(b, e);
}

void orc_ring_push(const orc_ring *r, const double *price, const double *port,
                   const uint64_t *ts) {
  for (int e = 0; e < r->n_envs; ++e)
    ring_push_one(r, e, price ? price + (size_t)e * r->n_price : NULL,
                  port ? port + (size_t)e * r->n_port : NULL, ts ? ts[e] : 0);
}

void orc_ring_clear(const orc_ring *r, const uint8_t *mask) {
  for (int e = 0; e < r->n_envs; ++e)
    if (!mask || mask[e]) ring_clear_one(r, e);
}

/* current_data for every env: rows oldest -> newest; an underfull deque yields
 * len rows (the rest zero); normaliser on the price block only. */
void orc_ring_gather(const orc_ring *r, double *price, double *port, uint64_t *ts) {
  const int W = r->window, F = r->n_price, P = r->n_port, C = F + P;
  for (int e = 0; e < r->n_envs; ++e) {
    const int len = r->len[e];
    const double *base = r->ring + (size_t)e * W * C;
    double *xp = price ? price + (size_t)e * W * F : NULL;
    for (int w = 0; w < W; ++w) {
      int valid = w < len;
      int h = (r->head[e] - (len - 1) + w + W * 2) % W;
      const double *row = base + (size_t)h * C;
      if (xp)
        for (int i = 0; i < F; ++i) xp[(size_t)w * F + i] = valid ? row[i] : 0.;
      if (port)
        for (int i = 0; i < P; ++i) port[((size_t)e * W + w) * P + i] = valid ? row[F + i] : 0.;
      if (ts) ts[(size_t)e * W + w] = valid ? r->ring_ts[(size_t)e * W + h] : 0;
    }
    if (!xp || len == 0) continue;
    int nt = r->norm_type;
    if (nt == ORC_NORM_LOG) {                       /* log_norm :79-81 */
      for (int w = 0; w < len; ++w)
        for (int i = 0; i < F; ++i) {
          double v = xp[(size_t)w * F + i];
          xp[(size_t)w * F + i] = log((v < 1e-5) ? 1e-5 : v);
        }
    } else if (nt == ORC_NORM_LOOKBACK || nt == ORC_NORM_LOOKBACK_LOG) { /* :63-66 */
      for (int i = 0; i < F; ++i) {
        double last = xp[(size_t)(len - 1) * F + i];
        for (int w = 0; w < len; ++w) {
          double v = xp[(size_t)w * F + i] / last;
          xp[(size_t)w * F + i] = (nt == ORC_NORM_LOOKBACK_LOG) ? log(v) : v;
        }
      }
    } else if (nt == ORC_NORM_STANDARD_NORMAL) {    /* standard_norm :83-92 */
      for (int i = 0; i < F; ++i) {
        double sum = 0.;
        for (int w = 0; w < len; ++w) sum += xp[(size_t)w * F + i];
        double mean = sum / len;
        double ss = 0.;
        for (int w = 0; w < len; ++w) {
          double d = xp[(size_t)w * F + i] - mean;
          ss += d * d;
        }
        double sd = sqrt(ss / len);
        for (int w = 0; w < len; ++w) {
          double v = (xp[(size_t)w * F + i] - mean) / sd;
          if (v != v) v = 0.;                       /* np.nan_to_num */
          else if (v == INFINITY) v = 1.7976931348623157e308;
          else if (v == -INFINITY) v = -1.7976931348623157e308;
          xp[(size_t)w * F + i] = v;
        }
      }
    } else if (nt == ORC_NORM_LOG_STANDARD_NORMAL) { /* log_standard_norm :95-107 */
      for (int i = 0; i < F; ++i) {
        double sum = 0.;
        int cnt = 0;                                /* np.nanmean / np.nanstd skip nan */
        for (int w = 0; w < len; ++w) {
          double x = log(xp[(size_t)w * F + i]);
          if (x == x) { sum += x; cnt += 1; }
        }
        double mean = sum / cnt;
        double ss = 0.;
        for (int w = 0; w < len; ++w) {
          double x = log(xp[(size_t)w * F + i]);
          if (x == x) { double d = x - mean; ss += d * d; }
        }
        double sd = sqrt(ss / cnt);
        for (int w = 0; w < len; ++w) {
          double v = (log(xp[(size_t)w * F + i]) - mean) / sd;
          if (v != v) v = 0.;
          else if (v == INFINITY) v = 1.7976931348623157e308;
          else if (v == -INFINITY) v = -1.7976931348623157e308;
          xp[(size_t)w * F + i] = v;
        }
      }
    }
  }
}

void orc_window(const orc_batch *b, double *price, double *port, uint64_t *ts) {
  if (b->cfg.window > 0) orc_ring_gather(&b->ring, price, port, ts);
}
