/*
 * madigan_amd.h -- C ABI of the MI355X-native batched market-simulation step.
 *
 * One handle = N independent madigan Envs on one GPU, advanced together by
 * hand-written HIP kernels (libmadigan_hip.so).  Plain pointers and sizes only:
 * every pointer marked _dev is device memory; nothing here depends on torch.
 *
 * Which reference interface each entry point replaces (paths relative to the
 * reference checkout, madigan/environments/cpp/ unless stated):
 *   mgn_create        Env(type, initCash, config) + setRequiredMargin/
 *                     setMaintenanceMargin/setSlippage/setTransactionCost
 *                     (env.cpp:843-869, Env.h:21-29, :94-111;
 *                      madigan/environments/__init__.py:9-22 make_env)
 *   mgn_reset         Env::reset (Env.h:181-187) [+ preprocessor reset_state /
 *                     initialize_history, madigan/utils/preprocessor.py:191-199]
 *   mgn_step          Env::step() / step(units) / step(assetIdx, units)
 *                     (Env.h:189-256, env.cpp:991-1005) plus the n=1 reward
 *                     shaper (madigan/utils/buffers/nstep_buffer.py:30-204)
 *   mgn_rollout       K x { DQN.action_to_transaction (modelling/algorithm/
 *                     dqn.py:160-179); Env::step(units) } fused in one launch
 *   mgn_set_prices    DataSourceTick plug-in fed from the host
 *                     (DataSource.h:48-64, PyDataSource.h:9-24, Env.h:174-179)
 *   mgn_set_sources   Env::setDataSource (Env.h:174-179): swap the source,
 *                     keep the Broker / Portfolio
 *   mgn_stats_allgather the episode-statistics all-gather of the sharded path
 *                     (run/trainer.py:277-281 consumes the stats)
 *   mgn_save_state /  checkpoint / resume of the env state (the reference
 *   mgn_load_state    resumes through agent checkpoints only,
 *                     modelling/algorithm/base.py:153-186; Env.h:31)
 *   mgn_attach_replay HDFSourceSingle as the env's DataSource (DataSource.h:89-149,
 *                     DataSource.cpp:194-408): the device-resident replay tape
 *                     staged by libmadigan_hdf.so (include/madigan_hdf.h)
 *   mgn_window*       StackerDiscrete.stream_state / current_data
 *                     (madigan/utils/preprocessor.py:143-199)
 *   mgn_rollout_hist  K x { env.step; preprocessor.stream_state; current_data }
 *   mgn_window_hist   of the agent loop (madigan/modelling/algorithm/
 *   mgn_rollout_window offpolicy_q.py:143, 193-194): K steps in one launch,
 *                     then every step's window
 *   mgn_get_views     zero-copy property views (env.cpp:897-913)
 *   mgn_last_error    pybind11 exception translation (DataTypes.h:36-46)
 *
 * Threading: a handle is not thread-safe; all work is ordered on the handle's
 * stream and no call synchronises the host unless documented.
 */
#ifndef MADIGAN_AMD_H_
#define MADIGAN_AMD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MGN_ABI_VERSION 10
#define MGN_MAX_ASSETS 64
#define MGN_MAX_NSTEP 256

/* status codes; the Python layer maps them to the reference's exceptions */
enum {
  MGN_OK = 0,
  MGN_ERR_CONFIG = 1,   /* ConfigError / NotImplemented -> RuntimeError */
  MGN_ERR_INDEX = 2,    /* std::out_of_range            -> IndexError   */
  MGN_ERR_LENGTH = 3,   /* std::length_error            -> ValueError   */
  MGN_ERR_DEVICE = 4,   /* HIP runtime failure                          */
  MGN_ERR_ARG = 5       /* bad pointer / handle                         */
};

/* RiskInfo (DataTypes.h:70-75) */
enum { MGN_GREEN = 0, MGN_INSUFF_MARGIN = 1, MGN_MARGIN_CALL = 2, MGN_BLOWN_OUT = 3 };

/* per-asset generator kind (DataSource.cpp:56-108 factory names) */
enum { MGN_SRC_EXTERNAL = 0, MGN_SRC_SINE = 1, MGN_SRC_OU = 2, MGN_SRC_TRENDOU = 3,
       MGN_SRC_REPLAY = 4 /* every asset of the env, from the attached replay tape */,
       MGN_SRC_SIMPLETREND = 5, MGN_SRC_TRENDYOU = 6, MGN_SRC_GAUSSIAN = 7,
       MGN_SRC_SAWTOOTH = 8, MGN_SRC_TRIANGLE = 9, MGN_SRC_OUPAIR = 10,
       MGN_SRC_SINEADDER = 11, MGN_SRC_SINEDYNAMIC = 12, MGN_SRC_SINEDYNTREND = 13 };
#define MGN_SRC_PARAMS 64   /* doubles of parameters per asset */
#define MGN_AUX_WIDTH 24    /* doubles of extra source state per asset (views.aux) */

/* n-step pops (mgn_config.nstep_pop).  EXACT: every pop re-evaluates the
 * buffer's summands with the current shaper state and sums them in entry order
 * (nstep_buffer.py:62-91, 128-162 as written; ledger / State bit-exact, pops
 * within rtol 1e-10 of the reference).  RUNNING: DSR / DDR / PPC / none pops
 * formed from per-env discounted running sums of the buffer's entries, O(1)
 * per pop, within north_star's 1e-6 relative of the exact pop (re-formed from
 * the buffer every n pops); the shaper state A / B stays exact.  A permission,
 * not a requirement: kernels or shapers without the running form (the naive
 * shapers, per-asset rewards, the two-role and single-role schedules, or
 * gamma^n < 1e-3) pop exactly. */
enum { MGN_NSTEP_POP_EXACT = 0, MGN_NSTEP_POP_RUNNING = 1 };

/* reward shapers (nstep_buffer.py:378-408): DSR :30-98, DDR :101-169, PPC = cosine_port_shaper
 * :182-204, SHARPE = sharpe_shaper :207-239, SORTINO_A/B = sortino_shaperA/B :242-312 */
enum { MGN_SHAPER_NONE = 0, MGN_SHAPER_DSR = 1, MGN_SHAPER_DDR = 2, MGN_SHAPER_PPC = 3,
       MGN_SHAPER_SHARPE = 4, MGN_SHAPER_SORTINO_A = 5, MGN_SHAPER_SORTINO_B = 6 };
enum { MGN_REWARD_ENV_LOG = 0, MGN_REWARD_AGENT_SUM = 1, MGN_REWARD_AGENT_PER_ASSET = 2 };
enum { MGN_NORM_NONE = 0, MGN_NORM_LOG = 1, MGN_NORM_LOOKBACK = 2,
       MGN_NORM_STANDARD_NORMAL = 3, MGN_NORM_LOOKBACK_LOG = 4,
       MGN_NORM_LOG_STANDARD_NORMAL = 5 /* log_standard_norm, preprocessor.py:95-107 */ };
/* ring push transforms: StackerDiscretePairs' price[:, 0] / price[:, 1]
 * (preprocessor.py:303-316) is row-wise, so it is applied once at push */
enum { MGN_RING_PLAIN = 0, MGN_RING_PAIR_RATIO = 1 };
/* step kinds: Env::step() / step(units) / step(assetIdx, units) */
enum { MGN_STEP_NONE = 0, MGN_STEP_UNITS = 1, MGN_STEP_SINGLE = 2 };

/* Per-asset generator parameters (Composite = concatenation in config order).
 *  SINE    p = {freq, mu, amp, phase, dX, noise}            DataSource.cpp:455-473
 *  OU      p = {mean, theta, phi}                           DataSource.cpp:1118-1137
 *  TRENDOU p = {trendProb, minPeriod, maxPeriod, dYMin, dYMax, start,
 *               theta, phi, noiseTrend, emaAlpha}           DataSource.cpp:1364-1408
 *  REPLAY  p = {}  (all assets or none; see mgn_attach_replay)
 *  SIMPLETREND p = {trendProb, minPeriod, maxPeriod, noise, start, dYMin, dYMax}
 *                                                           DataSource.cpp:1252-1356
 *  TRENDYOU    p = as TRENDOU                               DataSource.cpp:1506-1653
 *  GAUSSIAN    p = {mean, var (the normal's stddev)}        DataSource.cpp:1057-1114
 *  SAWTOOTH / TRIANGLE p = as SINE                          DataSource.cpp:557-577
 *  OUPAIR      p = {theta, phi, noise, role}: role 0 / 1 = the pair's first /
 *              second asset, adjacent in asset order        DataSource.cpp:1183-1250
 *  SINEADDER   p = {C, dX, noise, freq[C], mu[C], amp[C], phase[C]}, C <= 8: one
 *              asset, the sum of C noisy sines              DataSource.cpp:582-673
 *  SINEDYNAMIC p = {C, sampleRate, noise, tableLen[C], then per component
 *              freqRange[3], muRange[3], ampRange[3] ({lo, hi, step})}, C <= 4:
 *              one asset, C WaveTableOsc sines with random-walk parameters
 *                                                           DataSource.cpp:678-845,
 *                                                           WaveTableOsc.h
 *  SINEDYNTREND p = SINEDYNAMIC's, then {T, per trend {minLen, maxLen, incr,
 *              prob}}, T <= 2                               DataSource.cpp:850-1051
 *  The multi-component kinds keep their extra state in views.aux
 *  (N, A, MGN_AUX_WIDTH): SINEADDER x[C]; SINEDYNAMIC {phasor, freq, mu, amp}
 *  per component; SINEDYNTREND also [16] trendComponent and per trend
 *  [17+3t] trending, [18+3t] direction, [19+3t] remaining length. */
typedef struct {
  int32_t kind;
  int32_t pad_;
  double p[MGN_SRC_PARAMS];
} mgn_asset_source;

typedef struct {
  int32_t n_envs;
  int32_t n_assets;
  int64_t env_offset;          /* global index of env 0 when sharded over GPUs */
  uint64_t seed;               /* Philox key */
  double init_cash;
  double required_margin;
  double maintenance_margin;
  double slippage_rel, slippage_abs;
  double tc_rel, tc_abs;
  int32_t shaper;              /* MGN_SHAPER_* */
  int32_t reward_mode;         /* MGN_REWARD_* : raw reward fed to the shaper */
  double adaptation_rate;      /* DSR/DDR eta */
  double cosine_temp;          /* PPC alpha */
  double desired_portfolio[MGN_MAX_ASSETS + 1];
  int32_t window;              /* StackerDiscrete window_length, 0 = none */
  int32_t norm_type;           /* MGN_NORM_* applied by mgn_window */
  int32_t auto_reset;          /* reset done envs inside the step kernel */
  int32_t action_atoms;        /* discrete actions for mgn_rollout */
  double unit_size;            /* unit_size_proportion_avM */
  int32_t nstep;               /* n-step return length (nstep_return), 1..MGN_MAX_NSTEP;
                                  NStepBuffer semantics, nstep_buffer.py:315-356 */
  int32_t nstep_pop;           /* MGN_NSTEP_POP_*: how an n-step pop is evaluated (ABI 9;
                                  ABI 10: MGN_MAX_NSTEP 64 -> 256) */
  double discount;             /* gamma of the n-step aggregation */
  int32_t n_feats;             /* F = State.price width: n_assets for the generators
                                  (0 = n_assets); the feature columns of a replay source */
  int32_t pad3_;
  double sortino_exp;          /* sortino_shaperA/B exponent (shaper config "sortino_exp") */
  int32_t aux;                 /* 1: some asset is a multi-component kind (SINEADDER,
                                  SINEDYNAMIC, SINEDYNTREND) -> views.aux is allocated */
  int32_t pad4_;
} mgn_config;

/* Per-step outputs.  For mgn_step they are the handle's buffers (see views);
 * for mgn_rollout the caller passes (K, ...) device arrays, any may be NULL. */
typedef struct {
  double *reward;        /* (N)            env log reward                 */
  double *agent_reward;  /* (N) or (N,A)   offpolicy_q.py:152-164         */
  double *shaped;        /* (N[,n][,A])    shaped rewards popped this step, in
                            pop order (n-step: (N,n) or (N,n,A); n == 1: (N) or (N,A)) */
  uint8_t *done;         /* (N)                                           */
  double *obs_price;     /* (N,F)          State.price (features; F = A for generators) */
  double *obs_port;      /* (N,A+1)        State.portfolio                */
  uint64_t *timestamp;   /* (N)            State.timestamp                */
  double *tprice;        /* (N,A)          BrokerResponse.transactionPrice */
  double *tunits;        /* (N,A)                                         */
  double *tcost;         /* (N,A)                                         */
  uint8_t *risk;         /* (N,A)          RiskInfo                       */
  uint8_t *margin_call;  /* (N)                                           */
  uint8_t *n_shaped;     /* (N)            number of shaped rewards popped (n-step) */
  uint8_t *data_end;     /* (N)            EnvInfo.dataEnd (Env.h:226; DataSource.h:126) */
} mgn_traj;

/* Device pointers into the handle's arena (row-major, env-major). */
typedef struct {
  double *ledger, *mean_entry, *borrowed, *prices;   /* (N,A) */
  double *sine_x, *ou_mean, *trend_dy;               /* (N,A) generator state */
  int32_t *trend_len;                                /* (N,A) */
  uint8_t *trend_flags;                              /* (N,A) bit0 trending, bit1 dir<0 */
  double *cash;                                      /* (N) */
  uint64_t *timestamp;                               /* (N) */
  double *shaper_a, *shaper_b;                       /* (N,D) */
  double *ep_stats;                                  /* (N,2) running {return, length} */
  double *episode_stats;                             /* (N,4) {last return, last length,
                                                               last final equity, done count} */
  double *ext_prices;                                /* (N,A) external source input */
  double *units;                                     /* (N,A) staging for mgn_step input */
  int32_t *asset_idx;                                /* (N)   staging for STEP_SINGLE */
  double *ring;                                      /* (N,W,F+A+1) window ring */
  uint64_t *ring_ts;                                 /* (N,W) */
  int32_t *ring_head, *ring_len;                     /* (N) */
  double *win_price, *win_port;                      /* (N,W,F), (N,W,A+1) gathered window */
  uint64_t *win_ts;                                  /* (N,W) */
  uint8_t *reset_mask;                               /* (N) staging for mgn_reset */
  double *nstep_ring;                                /* (N,n,D) NStepBuffer rewards */
  int32_t *nstep_len, *nstep_head;                   /* (N) fill count, oldest index */
  int64_t *replay_cursor;                            /* (N) next tape row of a replay env */
  double *aux;                                       /* (N,A,MGN_AUX_WIDTH) multi-component
                                                        source state (NULL if unused) */
  uint64_t *draw_skip;                               /* (N) resets so far: the variates'
                                                        draw index is timestamp + draw_skip
                                                        (ABI 8; DESIGN.md, variates v3) */
  mgn_traj out;                                      /* mgn_step outputs */
  int32_t n_envs, n_assets, window, reward_dim, nstep, n_feats;
} mgn_views;

/* Replay tape (caller-owned device memory, borrowed until mgn_destroy): one
 * period of the rows HDFSourceSingle::getData visits, in visiting order
 * (mgn_hdf_stage fills it).  Env e (global index g = env_offset + e) starts
 * at tape row (g * stride) mod rows; stride 0 replays the reference's single
 * path in every env. */
typedef struct {
  const double *price;       /* (rows, A)  currentPrices */
  const double *feats;       /* (rows, F)  currentData = State.price */
  const uint64_t *ts;        /* (rows)     timestamps = State.timestamp */
  const uint8_t *data_end;   /* (rows)     dataEnd() after that row */
  int64_t rows;
  int64_t stride;
} mgn_replay_tape;

/* Stand-alone StackerDiscrete ring (preprocessor.py:143-199), caller-owned
 * device memory: ring (N, W, n_price + n_port), ring_ts (N, W), head/len (N).
 * transform: MGN_RING_* applied to the pushed price row (PAIR_RATIO: the
 * pushed row has 2 columns, the ring stores n_price = 1).  out_stride /
 * out_offset: row stride (0 = n_price) and first column of the gathered price
 * in the caller's buffer, so the rings of a MultiStackerDiscrete
 * (preprocessor.py:202-288) gather side by side into one (N, W, sum) array. */
typedef struct {
  int32_t n_envs, n_price, n_port, window, norm_type, transform;
  double *ring;
  uint64_t *ring_ts;
  int32_t *head, *len;
  int32_t out_stride, out_offset;
} mgn_ring;

typedef struct mgn_env mgn_env;

int mgn_abi_version(void);
/* bytes of device memory a handle needs (caller-provided arena) */
size_t mgn_arena_bytes(const mgn_config *cfg);
/* arena: device memory of mgn_arena_bytes() bytes, or NULL to allocate;
 * stream: hipStream_t or NULL for the null stream.  Runs the Env constructor
 * (source init + initAccountants' first getData, Env.h:139-165). */
int mgn_create(const mgn_config *cfg, const mgn_asset_source *sources, void *stream, void *arena,
               size_t arena_bytes, mgn_env **out);
int mgn_destroy(mgn_env *env);
int mgn_set_stream(mgn_env *env, void *stream);
int mgn_get_views(const mgn_env *env, mgn_views *views);
/* Env::reset for envs with mask_dev[e] != 0 (NULL: all envs). */
int mgn_reset(mgn_env *env, const uint8_t *mask_dev);
/* one Env::step for every env; kind MGN_STEP_*; units_dev (N,A) for UNITS,
 * (N) for SINGLE with asset_idx_dev (N).  Outputs land in views.out. */
int mgn_step(mgn_env *env, int32_t kind, const double *units_dev, const int32_t *asset_idx_dev);
/* k_steps fused steps; actions_dev (K,N,A) int8 discrete atoms */
int mgn_rollout(mgn_env *env, const int8_t *actions_dev, int32_t k_steps, const mgn_traj *out);
/* k_steps fused Env::step(units); units_dev (K,N,A) fp64 */
int mgn_rollout_units(mgn_env *env, const double *units_dev, int32_t k_steps, const mgn_traj *out);
/* prices (N,A) consumed by the next getData of MGN_SRC_EXTERNAL assets */
int mgn_set_prices(mgn_env *env, const double *prices_dev);
/* Env::setDataSource (Env.h:174-179; PyDataSource.h:9-15): swap the price
 * source of every env in place.  Ledger, cash, mean entry, borrowed margin,
 * shaper, window and statistics are kept, as the reference keeps its Broker /
 * Portfolio.  sources (host, n_assets entries): MGN_SRC_EXTERNAL (a host
 * DataSourceTick that feeds mgn_set_prices before each tick) or the asset's
 * current kind with new parameters; replay handles cannot switch.
 * prices_dev (N,A): the new source's currentPrices(), at which the Broker
 * values the portfolio from now on (Env.h:177-178); NULL keeps the prices.
 * Synchronises the handle's stream (the source table is uploaded). */
int mgn_set_sources(mgn_env *env, const mgn_asset_source *sources, const double *prices_dev);
/* attach the replay tape of a MGN_SRC_REPLAY handle and run the Env
 * constructor's first getData (Env.h:150-165) from it; stepping a replay
 * handle before this fails with MGN_ERR_CONFIG */
int mgn_attach_replay(mgn_env *env, const mgn_replay_tape *tape);
/* StackerDiscrete.stream_state with explicit rows (any may be NULL = current State) */
int mgn_window_push(mgn_env *env, const double *price_dev, const double *port_dev,
                    const uint64_t *ts_dev);
/* StackerDiscrete.reset_state for masked envs (NULL: all) */
int mgn_window_clear(mgn_env *env, const uint8_t *mask_dev);
/* StackerDiscrete.current_data into caller buffers (NULL: views.win_*) */
int mgn_window(mgn_env *env, double *price_dev, double *port_dev, uint64_t *ts_dev);
/* the agent loop of a windowed env with K steps in one launch: every step k
 * of mgn_rollout (offpolicy_q.py:143 env.step) followed by
 * preprocessor.stream_state / current_data (offpolicy_q.py:193-194,
 * preprocessor.py:172-189).  mgn_rollout_hist runs the K steps and keeps
 * every ring push of the launch in a handle-owned history (W + K*(W+1) rows
 * per env, allocated on first use); mgn_window_hist then writes all K windows
 * to (K,N,W,F) / (K,N,W,A+1) / (K,N,W) caller buffers (any may be NULL;
 * element-wise normalisers only).  mgn_rollout_window: per_step 1 = both;
 * per_step 0 = mgn_rollout + mgn_window (the last window only). */
int mgn_rollout_hist(mgn_env *env, const int8_t *actions_dev, int32_t k_steps, const mgn_traj *out);
int mgn_window_hist(mgn_env *env, double *price_dev, double *port_dev, uint64_t *ts_dev);
int mgn_rollout_window(mgn_env *env, const int8_t *actions_dev, int32_t k_steps, const mgn_traj *out,
                       double *price_dev, double *port_dev, uint64_t *ts_dev, int32_t per_step);
/* run mgn_window_hist on `stream` (NULL: the handle's stream): the history
 * is then double-buffered, so the gather of launch L overlaps the step launch
 * L+1 (ordered by events; the caller's window buffers of launch L are
 * complete once `stream` has passed the gather) */
int mgn_set_window_stream(mgn_env *env, void *stream);
/* kernel timing with HIP events on each kernel's own stream: on = 1 starts
 * (and clears) recording marker events around the step kernel of mgn_rollout /
 * mgn_rollout_hist and the gather of mgn_window_hist; on = 2 has mgn_rollout's
 * step launch record its own start / stop events (hipExtLaunchKernel: the
 * kernel's begin and end, without the marker packets' dispatch gaps); events
 * come from a per-handle pool, created once; 0 stops.  mgn_get_timing waits
 * for them and returns {step ms total, step launches, gather ms total,
 * gather launches} */
int mgn_set_timing(mgn_env *env, int32_t on);
int mgn_get_timing(mgn_env *env, double *out4);
/* uniform discrete actions U{0..atoms-1} (K,N,A) from Philox (benchmark input) */
int mgn_generate_actions(mgn_env *env, int8_t *actions_dev, int32_t k_steps, uint64_t seed);
/* Portfolio accessors for every env into out_dev (N,10): {cash, equity, pnl,
 * balance, availableMargin, usedMargin, borrowedMargin, borrowedAssetValue,
 * assetValue, checkRisk} (Portfolio.cpp:170-252, env.cpp:930-960) */
int mgn_valuation(mgn_env *env, double *out_dev);
/* Env::setRequiredMargin / setMaintenanceMargin / setSlippage /
 * setTransactionCost (Env.h:94-111): take effect at the next launch */
int mgn_set_broker(mgn_env *env, double required_margin, double maintenance_margin,
                   double slippage_rel, double slippage_abs, double tc_rel, double tc_abs);
/* stream_state: rows price (N,n_price), port (N,n_port), ts (N) */
int mgn_ring_push(const mgn_ring *ring, const double *price_dev, const double *port_dev,
                  const uint64_t *ts_dev, void *stream);
/* reset_state for masked envs (NULL: all) */
int mgn_ring_clear(const mgn_ring *ring, const uint8_t *mask_dev, void *stream);
/* current_data: price (N,W,n_price) normalised, port (N,W,n_port), ts (N,W) */
int mgn_ring_gather(const mgn_ring *ring, double *price_dev, double *port_dev, uint64_t *ts_dev,
                    void *stream);
/* StackerDiscreteReturns.current_data's np.diff (preprocessor.py:319-327; numpy's
 * default axis -1, i.e. across the price columns): out (rows, cols - 1) =
 * in[:, 1:] - in[:, :-1] for a (rows, cols) device array */
int mgn_feat_diff(const double *in_dev, double *out_dev, int64_t rows, int32_t cols, void *stream);
/* Lane layout of the step kernels: assets held per lane (1, 2, 4, 8; 0 =
 * automatic, the default).  Results are bit-identical for every layout (the
 * canonical reduction tree does not depend on it); only speed changes. */
int mgn_set_layout(mgn_env *env, int32_t assets_per_lane);
int mgn_get_layout(const mgn_env *env);
/* Step schedule: MGN_SCHED_SINGLE = k_step (every lane runs the whole Env
 * step for its assets); MGN_SCHED_DUO = k_step_duo (each asset also has a lane
 * in a generator wave that shares the SIMD; 2..16 assets, generator sources
 * or a replay tape, n-step rings that fit LDS); MGN_SCHED_TRIO = k_step_trio
 * (generator, ledger and finish waves pipelined one step apart, `done`
 * speculated; 2..16 assets, generator sources with n = 1 with or without a
 * window, or a scalar n-step reward without a window whose rings fit the
 * workgroup's LDS, and replay tapes at 16 assets for N >= 4096; 9..16
 * assets at N >= 4096 with discrete actions and n = 1 run two asset slots per
 * lane); MGN_SCHED_AUTO (default) = TRIO where eligible and measured faster
 * (up to 8 assets; 9..16 assets with n = 1 -- windows only at N >= 4096 --
 * or replay), else DUO where eligible and the layout is one asset per lane,
 * else SINGLE.  Results are bit-identical; only speed changes. */
enum { MGN_SCHED_AUTO = 0, MGN_SCHED_SINGLE = 1, MGN_SCHED_DUO = 2, MGN_SCHED_TRIO = 3 };
int mgn_set_schedule(mgn_env *env, int32_t schedule);
int mgn_get_schedule(const mgn_env *env);
/* Zero-copy per-step windows (element-wise normalisers: none, log).  After
 * mgn_rollout_hist, the launch history holds every ring push of the launch,
 * oldest first, per env: window k of env e (StackerDiscrete.current_data after
 * step k, preprocessor.py:177-189) is history rows [hend - hlen, hend) of env
 * e, hend / hlen at [k * n_envs + e], and its rows hlen..W-1 are the zero
 * padding mgn_window_hist writes.  The price columns are log-normalised at push
 * for norm "log", so each window is a contiguous row range read in place --
 * no (K, N, W, .) copy.  The pointers are the handle's and stay valid until
 * its next mgn_rollout_hist (with a window stream: until the one after). */
typedef struct {
  const double *hist;       /* (n_envs, rows, cols): price features, then ledgerNormedFull */
  const uint64_t *hist_ts;  /* (n_envs, rows) */
  const int32_t *hend;      /* (k_steps, n_envs) one past window k's last row */
  const int32_t *hlen;      /* (k_steps, n_envs) window k's fill (<= window) */
  int32_t rows, cols, k_steps, window, n_feats, pad_;
} mgn_hist_view;
int mgn_window_hist_view(mgn_env *env, mgn_hist_view *out);
/* Broker / Portfolio operations outside a step (no tick, no reward): the
 * drop-in's env.broker / env.portfolio objects, per env on device.
 *   MGN_OP_BROKER_UNITS  Broker::handleTransaction(units) / handleAction /
 *                        handleEvent (Broker.cpp:144-158, Broker.h:96-101):
 *                        units_dev (N, A); responses (N, A)
 *   MGN_OP_BROKER_SINGLE Broker::handleTransaction(assetIdx, units)
 *                        (Broker.cpp:124-142): asset_idx_dev, units_dev (N);
 *                        responses (N)
 *   MGN_OP_BROKER_CLOSE  Broker::close(assetIdx) (Broker.cpp:160-169): the
 *                        position closed at slippage and cost, always green;
 *                        responses (N)
 *   MGN_OP_PORT_TXN      Portfolio::handleTransaction(assetIdx, transactionPrice,
 *                        units, transactionCost) (Portfolio.cpp:284-323), no
 *                        risk check: asset_idx_dev, units_dev, tprice_dev,
 *                        tcost_dev (N; null = 0)
 *   MGN_OP_PORT_CLOSE    Portfolio::close(assetIdx, transactionPrice,
 *                        transactionCost) (Portfolio.cpp:327-333)
 *   MGN_OP_CHECK_ORDER   Portfolio::checkRisk(assetIdx, units)
 *                        (Portfolio.cpp:254-279) into out->risk (N); no change
 * out: tprice / tunits / tcost / risk / margin_call device pointers (null =
 * not written); margin_call = Portfolio::checkRisk() after the operation.
 * An asset index outside [0, n_assets) leaves that env untouched (response
 * zero, risk code 0xFF, margin_call 0); the Python layer raises IndexError
 * before calling, as the reference's std::out_of_range. */
enum { MGN_OP_BROKER_UNITS = 0, MGN_OP_BROKER_SINGLE = 1, MGN_OP_BROKER_CLOSE = 2,
       MGN_OP_PORT_TXN = 3, MGN_OP_PORT_CLOSE = 4, MGN_OP_CHECK_ORDER = 5 };
int mgn_ledger_op(mgn_env *env, int32_t op, const int32_t *asset_idx_dev, const double *units_dev,
                  const double *tprice_dev, const double *tcost_dev, const mgn_traj *out);
/* The one collective of the sharded path: all-gather the (N,4)
 * episode statistics of every rank over a caller-provided RCCL communicator
 * (an ncclComm_t, e.g. torch's ProcessGroupNCCL._comm_ptr()), ordered on the
 * handle's stream.  Each rank contributes rows_per_rank rows (>= N; 0 = N):
 * its N rows of statistics, then zero rows, so ragged shards gather with one
 * ncclAllGather; out_dev receives nranks * rows_per_rank * 4 doubles in rank
 * order.  ncclAllGather is resolved from the RCCL the process has already
 * loaded (else librccl.so.1), so the communicator and the call share one
 * library instance. */
int mgn_stats_allgather(mgn_env *env, void *nccl_comm, int32_t rows_per_rank, double *out_dev);
/* Checkpoint / resume: the handle's whole device state (ledger,
 * cash, generator and shaper state, window ring, n-step buffer, statistics,
 * replay cursors, source table) plus its configuration, as one host blob of
 * mgn_state_bytes() bytes.  mgn_save_state synchronises the stream;
 * mgn_load_state restores the blob into a handle of the same dimensions
 * (configuration, broker settings and RNG key included), so the restored
 * handle continues every episode bit-exactly.  A replay tape is not part of
 * the state: attach the same tape before loading. */
size_t mgn_state_bytes(const mgn_env *env);
int mgn_save_state(mgn_env *env, void *host_dst, size_t bytes);
int mgn_load_state(mgn_env *env, const void *host_src, size_t bytes);
/* Measurement only: the attainable HBM bandwidth of a plain
 * device copy of bytes (a multiple of 16) from src_dev to dst_dev on stream,
 * 16 B per lane: the best of six copy shapes (one 16- or 32-KiB chunk per
 * workgroup or a grid-stride loop; plain or nontemporal stores), each timed over reps
 * launches with HIP events; *gbps_out = (read + write bytes) / time in GB/s.
 * Synchronises. */
int mgn_bandwidth_probe(void *dst_dev, const void *src_dev, size_t bytes, int32_t reps, void *stream,
                        double *gbps_out);
/* synchronise the handle's stream */
int mgn_synchronize(mgn_env *env);
/* synchronise the handle's stream by polling it (hipStreamQuery until the
 * stream is idle: the calling thread busy-waits; for short waits, e.g. an
 * agent loop's per-step wait) */
int mgn_synchronize_spin(mgn_env *env);
const char *mgn_last_error(const mgn_env *env);
const char *mgn_global_error(void);

#ifdef __cplusplus
}
#endif
#endif
