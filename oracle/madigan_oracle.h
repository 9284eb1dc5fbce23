/*
 * madigan_oracle.h -- CPU restatement of madigan's market-simulation step.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP
 * product path (madigan_amd/csrc) and the CPU baseline timed by bench.py's
 * cpu_baseline leg.  Nothing under madigan_amd/ may link, import or call it.
 *
 * Every function in madigan_oracle.c cites the reference statement it
 * restates (paths relative to the reference checkout, e.g.
 * madigan/environments/cpp/Portfolio.cpp:284-323).
 *
 * Layout: one orc_env object per environment (AoS, as the reference keeps one
 * Env -> Broker -> Account -> Portfolio chain per env).  All arrays handed in
 * or out are dense row-major (N, A) / (N, A+1) / (K, N, ...).
 *
 * Parity basis: strict IEEE binary64, -ffp-contract=off.  Reductions over
 * assets use the canonical pairwise tree (assets 0..A-1 padded with +0.0 to
 * the next power of two).  The reference's Eigen dot/sum order under
 * -ffast-math is not reproducible bit-for-bit; parity with the
 * reference itself is pinned by its own known-answer tests (envTest.py).
 */
#ifndef MADIGAN_ORACLE_H_
#define MADIGAN_ORACLE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MAX_ASSETS 64
#define ORC_MAX_NSTEP 256

/* RiskInfo enum order: madigan/environments/cpp/DataTypes.h:70-75 */
enum { ORC_GREEN = 0, ORC_INSUFF_MARGIN = 1, ORC_MARGIN_CALL = 2, ORC_BLOWN_OUT = 3 };

/* per-asset generator kinds */
enum { ORC_SRC_EXTERNAL = 0, ORC_SRC_SINE = 1, ORC_SRC_OU = 2, ORC_SRC_TRENDOU = 3,
       ORC_SRC_REPLAY = 4 /* HDFSourceSingle over in-memory arrays (all assets) */,
       ORC_SRC_SIMPLETREND = 5, ORC_SRC_TRENDYOU = 6, ORC_SRC_GAUSSIAN = 7,
       ORC_SRC_SAWTOOTH = 8, ORC_SRC_TRIANGLE = 9, ORC_SRC_OUPAIR = 10,
       ORC_SRC_SINEADDER = 11, ORC_SRC_SINEDYNAMIC = 12, ORC_SRC_SINEDYNTREND = 13 };
#define ORC_SRC_PARAMS 64   /* doubles of parameters per asset */
#define ORC_AUX_WIDTH 24    /* doubles of extra source state per asset (multi-component kinds) */

/* reward shapers (nstep_buffer.py:378-408) */
enum { ORC_SHAPER_NONE = 0, ORC_SHAPER_DSR = 1, ORC_SHAPER_DDR = 2, ORC_SHAPER_PPC = 3,
       ORC_SHAPER_SHARPE = 4, ORC_SHAPER_SORTINO_A = 5, ORC_SHAPER_SORTINO_B = 6 };

/* which raw reward feeds the shaper */
enum { ORC_REWARD_ENV_LOG = 0, ORC_REWARD_AGENT_SUM = 1, ORC_REWARD_AGENT_PER_ASSET = 2 };

/* StackerDiscrete normalisers (preprocessor.py:53-107) */
enum { ORC_NORM_NONE = 0, ORC_NORM_LOG = 1, ORC_NORM_LOOKBACK = 2,
       ORC_NORM_STANDARD_NORMAL = 3, ORC_NORM_LOOKBACK_LOG = 4,
       ORC_NORM_LOG_STANDARD_NORMAL = 5 };

/* step variants: Env.h:189-204 (none), :206-230 (units), :232-256 (single) */
enum { ORC_STEP_NONE = 0, ORC_STEP_UNITS = 1, ORC_STEP_SINGLE = 2 };

/*
 * Per-asset generator parameters.
 *  SINE    p = {freq, mu, amp, phase, dX, noise}
 *  OU      p = {mean, theta, phi}
 *  TRENDOU p = {trendProb, minPeriod, maxPeriod, dYMin, dYMax, start,
 *               theta, phi, noiseTrend, emaAlpha}
 *  SIMPLETREND p = {trendProb, minPeriod, maxPeriod, noise, start, dYMin, dYMax}
 *  TRENDYOU    p = as TRENDOU
 *  GAUSSIAN    p = {mean, var (the normal's stddev argument)}
 *  SAWTOOTH / TRIANGLE p = as SINE
 *  OUPAIR      p = {theta, phi, noise, role}: role 0 / 1 = first / second
 *              asset of the pair, adjacent in asset order
 *  SINEADDER   p = {C, dX, noise, freq[C], mu[C], amp[C], phase[C]}, C <= 8
 *  SINEDYNAMIC p = {C, sampleRate, noise, tableLen[C], then per component
 *              freqRange[3], muRange[3], ampRange[3]}, C <= 4
 *  SINEDYNTREND p = SINEDYNAMIC's, then {T, per trend: minLen, maxLen, incr,
 *              prob}, T <= 2
 *  aux state (ORC_AUX_WIDTH per asset): SINEADDER x[C]; SINEDYNAMIC per
 *  component {phasor, freq, mu, amp}; SINEDYNTREND also [16] trendComponent,
 *  per trend [17+3t] trending, [18+3t] direction, [19+3t] remaining length
 */
typedef struct {
  int32_t kind;
  int32_t pad_;
  double p[ORC_SRC_PARAMS];
} orc_asset_src;

typedef struct {
  int32_t n_envs;
  int32_t n_assets;
  int64_t env_offset;          /* global index of env 0 (sharding) */
  uint64_t seed;
  double init_cash;
  double required_margin;
  double maintenance_margin;
  double slippage_rel, slippage_abs;
  double tc_rel, tc_abs;
  int32_t shaper;
  int32_t reward_mode;
  double adaptation_rate;
  double cosine_temp;
  double desired_portfolio[ORC_MAX_ASSETS + 1];
  int32_t window;
  int32_t norm_type;
  int32_t auto_reset;
  int32_t action_atoms;
  double unit_size;
  int32_t nstep;               /* n-step return length (nstep_return), <= ORC_MAX_NSTEP */
  int32_t pad2_;
  double discount;             /* gamma of the n-step aggregation */
  int32_t n_feats;             /* State.price width (replay features); 0 = n_assets */
  int32_t pad3_;
  double sortino_exp;          /* sortino_shaperA/B exponent (shaper config "sortino_exp") */
} orc_config;

/* Outputs of one step for all envs.  Any pointer may be NULL. */
typedef struct {
  double *reward;        /* (N)     env log reward */
  double *agent_reward;  /* (N) or (N,A) per reward_mode */
  double *shaped;        /* (N[,n],D) shaper outputs emitted this step, in pop order
                            (n-step: (N,n,D); n == 1: (N,D)) */
  uint8_t *done;         /* (N) */
  double *obs_price;     /* (N,F)   State.price (F = A for the generators) */
  double *obs_port;      /* (N,A+1) State.portfolio = ledgerNormedFull */
  uint64_t *timestamp;   /* (N) */
  double *tprice;        /* (N,A) BrokerResponse.transactionPrice */
  double *tunits;        /* (N,A) */
  double *tcost;         /* (N,A) */
  uint8_t *risk;         /* (N,A) */
  uint8_t *margin_call;  /* (N) */
  uint8_t *n_shaped;     /* (N) shaped rewards emitted this step (n-step) */
  uint8_t *data_end;     /* (N) EnvInfo.dataEnd */
} orc_out;

/* StackerDiscrete deques of N envs: ring (N,W,F+P), ring_ts (N,W), head/len (N) */
typedef struct {
  int32_t n_envs, n_price, n_port, window, norm_type, pad_;
  double *ring;
  uint64_t *ring_ts;
  int32_t *head, *len;
} orc_ring;
void orc_ring_push(const orc_ring *r, const double *price, const double *port, const uint64_t *ts);
void orc_ring_clear(const orc_ring *r, const uint8_t *mask);
void orc_ring_gather(const orc_ring *r, double *price, double *port, uint64_t *ts);

typedef struct orc_batch orc_batch;

orc_batch *orc_create(const orc_config *cfg, const orc_asset_src *srcs);
void orc_destroy(orc_batch *b);
/* Env::reset for envs with mask[e] != 0 (mask NULL: all). */
void orc_reset(orc_batch *b, const uint8_t *mask);
/* One Env::step* for every env. units: (N,A) for STEP_UNITS; for
 * STEP_SINGLE asset_idx (N) and units (N). */
void orc_step(orc_batch *b, int kind, const double *units, const int32_t *asset_idx,
              const orc_out *out);
/* K fused steps driven by discrete actions (K,N,A) int8 through
 * action_to_transaction (dqn.py:160-179); out arrays are (K, ...). */
void orc_rollout(orc_batch *b, const int8_t *actions, int k_steps, const orc_out *out);
void orc_rollout_mt(orc_batch *b, const int8_t *actions, int k_steps, const orc_out *out,
                    int threads);
/* dqn.py:160-179 on the current state: actions (N,A) -> units (N,A) */
void orc_action_to_units(orc_batch *b, const int8_t *actions, double *units);
/* external prices for the next getData (N,A), ORC_SRC_EXTERNAL assets */
void orc_set_prices(orc_batch *b, const double *prices);
void orc_set_sources(orc_batch *b, const orc_asset_src *srcs, const double *prices);
/* HDFSourceSingle for every env of an ORC_SRC_REPLAY batch, over the file's
 * arrays held in memory: price (T,A), feats (T,F), ts (T), time bounds
 * [first, second) as findBounds left them, cacheSize.  Env g's source is first
 * advanced (g * stride) mod period getData calls, then the Env constructor's
 * getData runs (Env.h:150-165).  Returns the period (rows per cycle). */
int64_t orc_set_replay(orc_batch *b, const double *price, const double *feats, const uint64_t *ts,
                       int64_t T, int64_t first, int64_t second, int64_t cache_size,
                       int64_t stride);

/* state access: field ids */
enum { ORC_F_LEDGER = 0, ORC_F_MEP = 1, ORC_F_BORROWED = 2, ORC_F_PRICE = 3,
       ORC_F_SINE_X = 4, ORC_F_OU_MEAN = 5, ORC_F_DY = 6, ORC_F_TLEN = 7,
       ORC_F_TRENDING = 8, ORC_F_DIR = 9, ORC_F_SHAPER_A = 10, ORC_F_SHAPER_B = 11 };
void orc_get_field(const orc_batch *b, int field, double *out); /* (N,A) as double */
void orc_set_field(orc_batch *b, int field, const double *in);
enum { ORC_S_CASH = 0, ORC_S_EQUITY = 1, ORC_S_PNL = 2, ORC_S_BALANCE = 3,
       ORC_S_AVAILABLE_MARGIN = 4, ORC_S_USED_MARGIN = 5, ORC_S_BORROWED_MARGIN = 6,
       ORC_S_BORROWED_ASSET_VALUE = 7, ORC_S_ASSET_VALUE = 8, ORC_S_TIMESTAMP = 9,
       ORC_S_CHECK_RISK = 10, ORC_S_SHAPER_A = 11, ORC_S_SHAPER_B = 12,
       ORC_S_EP_RET = 13, ORC_S_EP_LEN = 14, ORC_S_LAST_RET = 15, ORC_S_LAST_LEN = 16,
       ORC_S_LAST_EQUITY = 17, ORC_S_N_DONE = 18, ORC_S_DSKIP = 19 };
void orc_get_scalar(const orc_batch *b, int which, double *out); /* (N) */
void orc_set_cash(orc_batch *b, const double *cash);

/* Portfolio-level known-answer hooks (Portfolio.cpp) on env e */
void orc_port_handle_transaction(orc_batch *b, int e, int asset, double tprice,
                                 double units, double cost);
int orc_port_check_risk(const orc_batch *b, int e);
int orc_port_check_risk_order(const orc_batch *b, int e, int asset, double units);
void orc_port_ledger_normed_full(const orc_batch *b, int e, double *out); /* (A+1) */
/* Broker::handleTransaction(port, i, u) on env e: fills resp[4] = {tp,u,cost,risk} */
void orc_broker_handle_transaction(orc_batch *b, int e, int asset, double units,
                                   double *resp);
/* Broker::close(assetIdx) on env e: resp[4] = {tp, units, cost, risk (green)} */
void orc_broker_close(orc_batch *b, int e, int asset, double *resp);
/* Portfolio::close(assetIdx, transactionPrice, transactionCost) on env e */
void orc_port_close(orc_batch *b, int e, int asset, double tprice, double cost);

/* Sliding window (StackerDiscrete.current_data) for all envs:
 * price (N,W,A) normalised, port (N,W,A+1), ts (N,W). */
void orc_window(const orc_batch *b, double *price, double *port, uint64_t *ts);
/* stream the current State of every env into its window (stream_state) */
void orc_window_stream(orc_batch *b);

/* Standalone shaper restatements (nstep_buffer.py:30-204) for n=1..L:
 * rewards (L, D) oldest first, A/B (D) updated in place, out (D). */
void orc_dsr(const double *rewards, int L, int D, const double *discounts,
             double eta, double *A, double *B, double *out);
void orc_ddr(const double *rewards, int L, int D, const double *discounts,
             double eta, double *A, double *B, double *out);

void orc_ppc(const double *rewards, const double *ports, int L, int D, int P, const double *target,
             double temp, const double *discounts, double *out);

/* sharpe_shaper / sortino_shaperA / sortino_shaperB (nstep_buffer.py:207-312),
 * benchmark 0.: rewards (L, D) oldest first, out (D).  Stateless. */
void orc_naive(int shaper, const double *rewards, int L, int D, const double *discounts,
               double exp_, double *out);

/* RNG + deterministic math shared (by specification) with the device path */
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
double orc_log(double x);
double orc_sin(double x);
double orc_asin(double x);
/* the variates (specification v3, mgn_math.h): d = draw index */
double orc_vlog(double x);
void orc_vsincos2pi(double u, double *sn, double *cs);
double orc_normal(uint64_t seed, uint64_t env, uint32_t asset, uint64_t d);
void orc_draw0(uint64_t seed, uint64_t env, uint32_t asset, uint64_t d, double *z, double *ut,
               uint32_t *dbit);
void orc_uniform2(uint64_t seed, uint64_t env, uint32_t asset, uint32_t slot, uint64_t tick,
                  double *u0, double *u1);
double orc_canon_sum(const double *v, int n);

#ifdef __cplusplus
}
#endif
#endif
