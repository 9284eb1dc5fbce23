/* ASan / UBSan driver for the oracle (TEST INFRASTRUCTURE ONLY; SURVEY 5,
 * "ASan/UBSan on the host cpu_ref").  Built by `make -C oracle sanitize` with
 * -fsanitize=address,undefined -fno-sanitize-recover=all and run by
 * tests/test_sanitizers.py: every entry point of madigan_oracle.h over the
 * configurations the parity tests use (C1..C5 families, every generator,
 * shaper, reward mode, window normaliser, n-step, replay, host sources,
 * auto-reset, Portfolio / Broker hooks).  Any finding aborts with a report. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "madigan_oracle.h"

#define MAXK 40

static orc_asset_src src_of(int kind, const double *p, int np) {
  orc_asset_src s;
  memset(&s, 0, sizeof s);
  s.kind = kind;
  for (int i = 0; i < np; ++i) s.p[i] = p[i];
  return s;
}

typedef struct {
  double *reward, *agent_reward, *shaped, *obs_price, *obs_port, *tprice, *tunits, *tcost;
  uint8_t *done, *risk, *mc, *nsh, *dend;
  uint64_t *ts;
  orc_out o;
} outbuf;

static void out_alloc(outbuf *b, int K, int N, int A, int F, int n) {
  const size_t NK = (size_t)K * N, NA = NK * A;
  b->reward = calloc(NK, 8);
  b->agent_reward = calloc(NA, 8);
  b->shaped = calloc(NA * n, 8);
  b->obs_price = calloc(NK * F, 8);
  b->obs_port = calloc(NK * (A + 1), 8);
  b->tprice = calloc(NA, 8);
  b->tunits = calloc(NA, 8);
  b->tcost = calloc(NA, 8);
  b->done = calloc(NK, 1);
  b->risk = calloc(NA, 1);
  b->mc = calloc(NK, 1);
  b->nsh = calloc(NK, 1);
  b->dend = calloc(NK, 1);
  b->ts = calloc(NK, 8);
  orc_out o = {b->reward, b->agent_reward, b->shaped, b->done, b->obs_price, b->obs_port, b->ts,
               b->tprice, b->tunits, b->tcost, b->risk, b->mc, b->nsh, b->dend};
  b->o = o;
}

static void out_free(outbuf *b) {
  free(b->reward); free(b->agent_reward); free(b->shaped); free(b->obs_price); free(b->obs_port);
  free(b->tprice); free(b->tunits); free(b->tcost); free(b->done); free(b->risk); free(b->mc);
  free(b->nsh); free(b->dend); free(b->ts);
}

static orc_config base_cfg(int N, int A) {
  orc_config c;
  memset(&c, 0, sizeof c);
  c.n_envs = N;
  c.n_assets = A;
  c.seed = 1234;
  c.init_cash = 1e5;
  c.required_margin = 0.02;
  c.maintenance_margin = 0.25;
  c.slippage_rel = 1e-4;
  c.tc_rel = 0.02;
  c.adaptation_rate = 0.01;
  c.desired_portfolio[0] = 1.0;
  c.action_atoms = 3;
  c.unit_size = 0.9;
  c.auto_reset = 1;
  c.nstep = 1;
  c.discount = 0.97;
  c.sortino_exp = 2.0;
  return c;
}

static int run_case(const char *name, orc_config c, const orc_asset_src *srcs, int K) {
  orc_batch *b = orc_create(&c, srcs);
  if (!b) { fprintf(stderr, "%s: orc_create rejected the config\n", name); return 1; }
  const int N = c.n_envs, A = c.n_assets, F = (c.n_feats > 0 ? c.n_feats : A);
  outbuf ob;
  out_alloc(&ob, K, N, A, F, c.nstep);
  int8_t *acts = malloc((size_t)K * N * A);
  for (size_t i = 0; i < (size_t)K * N * A; ++i) acts[i] = (int8_t)((i * 2654435761u >> 7) % 3);
  orc_rollout(b, acts, K / 2, &ob.o);
  orc_rollout_mt(b, acts + (size_t)(K / 2) * N * A, K - K / 2, &ob.o, 1);
  double *u = calloc((size_t)N * A, 8);
  for (int i = 0; i < N * A; ++i) u[i] = (i % 5 - 2) * 300.0;
  outbuf one;
  out_alloc(&one, 1, N, A, F, c.nstep);
  orc_step(b, ORC_STEP_UNITS, u, NULL, &one.o);
  int32_t *idx = calloc((size_t)N, 4);
  for (int e = 0; e < N; ++e) idx[e] = e % A;
  orc_step(b, ORC_STEP_SINGLE, u, idx, &one.o);
  orc_step(b, ORC_STEP_NONE, NULL, NULL, &one.o);
  orc_action_to_units(b, acts, u);
  double *f = calloc((size_t)N * A, 8), *s = calloc((size_t)N, 8);
  for (int fld = ORC_F_LEDGER; fld <= ORC_F_SHAPER_B; ++fld) orc_get_field(b, fld, f);
  for (int w = ORC_S_CASH; w <= ORC_S_N_DONE; ++w) orc_get_scalar(b, w, s);
  if (c.window > 0) {
    double *wp = calloc((size_t)N * c.window * F, 8), *wo = calloc((size_t)N * c.window * (A + 1), 8);
    uint64_t *wt = calloc((size_t)N * c.window, 8);
    orc_window(b, wp, wo, wt);
    orc_window_stream(b);
    orc_window(b, wp, wo, wt);
    free(wp); free(wo); free(wt);
  }
  uint8_t *mask = calloc((size_t)N, 1);
  for (int e = 0; e < N; e += 2) mask[e] = 1;
  orc_reset(b, mask);
  orc_reset(b, NULL);
  if (srcs[0].kind != ORC_SRC_REPLAY) {
    orc_asset_src ext[ORC_MAX_ASSETS];
    for (int i = 0; i < A; ++i) ext[i] = src_of(ORC_SRC_EXTERNAL, NULL, 0);
    for (int i = 0; i < N * A; ++i) f[i] = 5.0 + (i % 7) * 0.1;
    orc_set_sources(b, ext, f);
    orc_set_prices(b, f);
    orc_step(b, ORC_STEP_UNITS, u, NULL, &one.o);
  }
  double lnf[ORC_MAX_ASSETS + 1], resp[4];
  orc_port_handle_transaction(b, 0, 0, 10.0, 100.0, 1.0);
  (void)orc_port_check_risk(b, 0);
  (void)orc_port_check_risk_order(b, 0, 0, -50.0);
  orc_port_ledger_normed_full(b, 0, lnf);
  orc_broker_handle_transaction(b, 0, A - 1, 25.0, resp);
  orc_set_cash(b, s);
  orc_destroy(b);
  out_free(&ob);
  out_free(&one);
  free(acts); free(u); free(idx); free(f); free(s); free(mask);
  fprintf(stderr, "ok %s\n", name);
  return 0;
}

int main(void) {
  int bad = 0;
  const double trend[10] = {0.2, 2, 6, 0.05, 0.2, 5.0, 0.15, 0.3, 0.2, 0.99};
  const double ou[3] = {10.0, 0.08, 0.04};
  const double sine[6] = {1.0, 2.0, 1.0, 0.0, 0.01, 0.05};
  const double strend[7] = {0.2, 2, 6, 0.01, 10.0, 0.01, 0.05};
  const double gauss[2] = {5.0, 1.0};
  orc_asset_src s[ORC_MAX_ASSETS];

  /* C3 family over every shaper / reward mode / n-step */
  for (int sh = ORC_SHAPER_NONE; sh <= ORC_SHAPER_SORTINO_B; ++sh)
    for (int rm = 0; rm <= ORC_REWARD_AGENT_PER_ASSET; ++rm)
      for (int n = 1; n <= 5; n += 4) {
        orc_config c = base_cfg(7, 8);
        c.shaper = sh;
        c.reward_mode = rm;
        c.nstep = n;
        c.cosine_temp = 0.05;
        for (int i = 0; i < 8; ++i) s[i] = src_of(ORC_SRC_TRENDOU, trend, 10);
        char name[64];
        snprintf(name, sizeof name, "trendou shaper %d mode %d n %d", sh, rm, n);
        bad |= run_case(name, c, s, MAXK);
      }
  /* C2 / C4 families: windows under every normaliser, composite sources */
  for (int norm = ORC_NORM_NONE; norm <= ORC_NORM_LOG_STANDARD_NORMAL; ++norm) {
    orc_config c = base_cfg(5, 8);
    c.window = 6;
    c.norm_type = norm;
    c.shaper = ORC_SHAPER_PPC;
    c.cosine_temp = 0.01;
    s[0] = src_of(ORC_SRC_SINE, sine, 6);
    s[1] = src_of(ORC_SRC_SAWTOOTH, sine, 6);
    s[2] = src_of(ORC_SRC_OU, ou, 3);
    s[3] = src_of(ORC_SRC_TRIANGLE, sine, 6);
    s[4] = src_of(ORC_SRC_SIMPLETREND, strend, 7);
    s[5] = src_of(ORC_SRC_TRENDYOU, trend, 10);
    s[6] = src_of(ORC_SRC_GAUSSIAN, gauss, 2);
    s[7] = src_of(ORC_SRC_TRENDOU, trend, 10);
    char name[64];
    snprintf(name, sizeof name, "composite window norm %d", norm);
    bad |= run_case(name, c, s, 24);
  }
  /* OUPair (adjacent roles) and 16 / 1 assets */
  {
    orc_config c = base_cfg(4, 2);
    const double p0[4] = {0.015, 0.01, 0.03, 0.0}, p1[4] = {0.015, 0.01, 0.03, 1.0};
    s[0] = src_of(ORC_SRC_OUPAIR, p0, 4);
    s[1] = src_of(ORC_SRC_OUPAIR, p1, 4);
    bad |= run_case("oupair", c, s, 16);
    orc_config c16 = base_cfg(3, 16);
    for (int i = 0; i < 16; ++i) s[i] = src_of(ORC_SRC_OU, ou, 3);
    bad |= run_case("ou x16", c16, s, 16);
    orc_config c1 = base_cfg(1, 1);
    c1.required_margin = 1.0;
    s[0] = src_of(ORC_SRC_SINE, sine, 6);
    bad |= run_case("C1 sine x1", c1, s, 16);
  }
  /* multi-component sources (SineAdder, SineDynamic, SineDynamicTrend) */
  {
    orc_config c = base_cfg(3, 3);
    double add[3 + 4 * 2] = {2, 0.01, 0.02, 1.0, 0.5, 2.0, 2.5, 1.0, 0.5, 0.0, 1.0};
    double dyn[64];
    memset(dyn, 0, sizeof dyn);
    dyn[0] = 2; dyn[1] = 100.0; dyn[2] = 0.01; dyn[3] = 64; dyn[4] = 32;
    for (int k = 0; k < 2; ++k) {
      double *r = dyn + 3 + 2 + 9 * k;
      const double v[9] = {0.1, 1.0, 0.01, 1.0, 5.0, 0.02, 1.0, 5.0, 0.01};
      memcpy(r, v, sizeof v);
    }
    double dtr[64];
    memcpy(dtr, dyn, sizeof dtr);
    dtr[3 + 10 * 2] = 2;
    const double tr[8] = {5, 20, 0.001, 0.1, 5, 30, 0.01, 0.2};
    memcpy(dtr + 3 + 10 * 2 + 1, tr, sizeof tr);
    s[0] = src_of(ORC_SRC_SINEADDER, add, 11);
    s[1] = src_of(ORC_SRC_SINEDYNAMIC, dyn, 64);
    s[2] = src_of(ORC_SRC_SINEDYNTREND, dtr, 64);
    bad |= run_case("multi-component", c, s, 24);
  }
  /* C5 family: replay over in-memory arrays (HDFSourceSingle) */
  {
    const int T = 50, A = 4, F = 3;
    double *price = malloc(sizeof(double) * T * A), *feats = malloc(sizeof(double) * T * F);
    uint64_t *ts = malloc(sizeof(uint64_t) * T);
    for (int t = 0; t < T; ++t) {
      ts[t] = (uint64_t)(1000 + 60 * t);
      for (int a = 0; a < A; ++a) price[t * A + a] = 10.0 + 0.01 * t + a;
      for (int j = 0; j < F; ++j) feats[t * F + j] = 0.1 * t - j;
    }
    orc_config c = base_cfg(6, A);
    c.n_feats = F;
    c.window = 4;
    c.shaper = ORC_SHAPER_DDR;
    for (int i = 0; i < A; ++i) s[i] = src_of(ORC_SRC_REPLAY, NULL, 0);
    orc_batch *b = orc_create(&c, s);
    if (!b || orc_set_replay(b, price, feats, ts, T, 3, 41, 7, 5) <= 0) {
      fprintf(stderr, "replay setup failed\n");
      bad = 1;
    } else {
      outbuf ob;
      out_alloc(&ob, 30, c.n_envs, A, F, 1);
      int8_t acts[30 * 6 * 4];
      for (size_t i = 0; i < sizeof acts; ++i) acts[i] = (int8_t)(i % 3);
      orc_rollout(b, acts, 30, &ob.o);
      out_free(&ob);
      fprintf(stderr, "ok replay\n");
    }
    orc_destroy(b);
    free(price); free(feats); free(ts);
  }
  /* stand-alone ring + shaper functions */
  {
    const int N = 3, P = 2, W = 5;
    orc_ring r;
    memset(&r, 0, sizeof r);
    r.n_envs = N; r.n_price = P; r.n_port = 3; r.window = W; r.norm_type = ORC_NORM_STANDARD_NORMAL;
    r.ring = calloc((size_t)N * W * (P + 3), 8);
    r.ring_ts = calloc((size_t)N * W, 8);
    r.head = calloc(N, 4);
    r.len = calloc(N, 4);
    orc_ring_clear(&r, NULL);
    double pr[6] = {1, 2, 3, 4, 5, 6}, po[9] = {0}, out_p[N * W * P], out_o[N * W * 3];
    uint64_t ts[3] = {1, 2, 3}, out_t[N * W];
    for (int k = 0; k < 7; ++k) orc_ring_push(&r, pr, po, ts);
    orc_ring_gather(&r, out_p, out_o, out_t);
    free(r.ring); free(r.ring_ts); free(r.head); free(r.len);
    double rw[20 * 2], disc[20], A0[2] = {0, 0}, B0[2] = {0, 0}, out[2], ports[20 * 3], tgt[3] = {1, 0, 0};
    for (int i = 0; i < 40; ++i) rw[i] = ((i * 7) % 11 - 5) * 0.01;
    for (int i = 0; i < 20; ++i) disc[i] = 1.0;
    for (int i = 0; i < 60; ++i) ports[i] = (i % 3) * 0.3;
    orc_dsr(rw, 20, 2, disc, 0.01, A0, B0, out);
    orc_ddr(rw, 20, 2, disc, 0.01, A0, B0, out);
    orc_ppc(rw, ports, 20, 1, 3, tgt, 0.05, disc, out);
    for (int sh = ORC_SHAPER_SHARPE; sh <= ORC_SHAPER_SORTINO_B; ++sh) orc_naive(sh, rw, 20, 2, disc, 3.0, out);
    fprintf(stderr, "ok ring + shapers\n");
  }
  if (!bad) printf("sanitize_oracle: all cases clean\n");
  return bad;
}
