// mgn_api.hip -- C ABI (include/madigan_amd.h) over the gfx950 kernels.
//
// One handle owns every device buffer of N envs in one arena (caller-provided
// or hipMalloc'd), launches on one stream and never synchronises the host
// except in mgn_create's parameter upload and mgn_synchronize.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <new>
#include <string>
#include <vector>

#include "../../include/madigan_amd.h"
#include "mgn_aux_kernels.h"
#include "mgn_launch.h"

namespace {

// window gather: LDS staging per workgroup (bytes)
constexpr size_t kGatherLdsTarget = 40 * 1024;
constexpr size_t kGatherLdsBudget = 64 * 1024;
// launch-history gather: windows (steps) per workgroup
constexpr int kHistStepsPerGroup = 16;
constexpr size_t kHistGroupBytes = 80 * 1024;  // k_hist_gather: output bytes per workgroup to reach

thread_local std::string g_error;

// bump allocator over the arena: every buffer 256-B aligned
struct Layout {
  size_t total = 0;
  size_t add(size_t bytes) {
    const size_t o = total;
    total += (bytes + 255) & ~size_t(255);
    return o;
  }
};

int next_pow2(int a) {
  int p = 1;
  while (p < a) p <<= 1;
  return p;
}

}  // namespace

struct mgn_env {
  mgn_config cfg;
  int N, A, W, D, F, apad;
  bool replay = false;        // MGN_SRC_REPLAY handle
  bool attached = false;      // replay tape attached (mgn_attach_replay)
  mgn_replay_tape tape{};
  hipStream_t stream;
  void* arena;
  bool own_arena;
  size_t arena_bytes;
  mgn_views v;
  mgn_asset_source* src_dev;
  double* target_dev;
  double* disc_dev;  // (n) gamma^i
  std::string err;
  int ablate = 0;
  int m = 1;  // assets per lane
  int sched = MGN_SCHED_AUTO;  // requested step schedule
  bool layout_auto = true;     // assets per lane chosen by auto_layout
  bool duo = false;            // the two-role kernel runs the steps
  bool trio = false;           // the three-role pipelined kernel runs the steps
  // launch history (mgn_rollout_hist): grown on demand, owned by the handle;
  // two buffers when the gathers run on a window stream (one is written by
  // the next step launch while the other is gathered)
  struct HistBuf {
    double* hist = nullptr;
    uint64_t* ts = nullptr;
    int32_t* hend = nullptr;
    int32_t* hlen = nullptr;
    size_t rows_cap = 0, k_cap = 0;
    int rows = 0;  // rows per env of its last mgn_rollout_hist
    int k = 0;     // its step count (0: none yet)
    hipEvent_t ready = nullptr;  // written (main stream)
    hipEvent_t read = nullptr;   // gathered (window stream)
  } hb[2];
  int hcur = 0;
  hipStream_t wstream = nullptr;  // window stream (mgn_set_window_stream), null: the handle's
  // kernel timing (mgn_set_timing): start/stop event pairs on each kernel's stream
  int timing = 0;  // 1: marker events around each launch; 2: events recorded by the step launch
  std::vector<hipEvent_t> t_step, t_gather;  // event pools, reused across mgn_set_timing calls
  size_t t_step_n = 0, t_gather_n = 0;        // events recorded since mgn_set_timing
  bool hist_on = false;  // kparams() hands the history to the step kernel
  std::vector<int32_t> kinds;  // the source kind of every asset (host copy of src_dev's)
  // mgn_stats_allgather: the rank's padded send rows (rows_per_rank x 4)
  double* ag_send = nullptr;
  size_t ag_rows = 0;
};

namespace {

struct Offsets {
  size_t L, mep, Bm, P, sx, oum, dy, tlen, tfl, cash, ts, dskip, sA, sB, ep, epstats, ext, units, aidx,
      ring, ring_ts, rhead, rlen, wprice, wport, wts, mask, reward, areward, shaped, done, obsp,
      obsport, obsts, tprice, tunits, tcost, risk, mcall, nshaped, dend, nring, nlen, nhead, disc,
      src, target, rcur, aux;
  size_t total;
};

Offsets plan(const mgn_config* c) {
  const size_t N = (size_t)c->n_envs, A = (size_t)c->n_assets;
  const size_t W = (size_t)(c->window > 0 ? c->window : 0);
  const size_t D = (c->reward_mode == MGN_REWARD_AGENT_PER_ASSET) ? A : 1;
  const size_t n = (size_t)(c->nstep > 0 ? c->nstep : 1);
  const size_t F = (size_t)(c->n_feats > 0 ? c->n_feats : c->n_assets);
  Layout l;
  Offsets o;
  o.L = l.add(N * A * 8);
  o.mep = l.add(N * A * 8);
  o.Bm = l.add(N * A * 8);
  o.P = l.add(N * A * 8);
  o.sx = l.add(N * A * 8);
  o.oum = l.add(N * A * 8);
  o.dy = l.add(N * A * 8);
  o.tlen = l.add(N * A * 4);
  o.tfl = l.add(N * A);
  o.cash = l.add(N * 8);
  o.ts = l.add(N * 8);
  o.dskip = l.add(N * 8);
  o.sA = l.add(N * D * 8);
  o.sB = l.add(N * D * 8);
  o.ep = l.add(N * 2 * 8);
  o.epstats = l.add(N * 4 * 8);
  o.ext = l.add(N * A * 8);
  o.units = l.add(N * A * 8);
  o.aidx = l.add(N * 4);
  o.ring = l.add(N * W * (F + A + 1) * 8);
  o.ring_ts = l.add(N * W * 8);
  o.rhead = l.add(N * 4);
  o.rlen = l.add(N * 4);
  o.wprice = l.add(N * W * F * 8);
  o.wport = l.add(N * W * (A + 1) * 8);
  o.wts = l.add(N * W * 8);
  o.mask = l.add(N);
  o.reward = l.add(N * 8);
  o.areward = l.add(N * D * 8);
  o.shaped = l.add(N * n * D * 8);
  o.done = l.add(N);
  o.obsp = l.add(N * F * 8);
  o.obsport = l.add(N * (A + 1) * 8);
  o.obsts = l.add(N * 8);
  o.tprice = l.add(N * A * 8);
  o.tunits = l.add(N * A * 8);
  o.tcost = l.add(N * A * 8);
  o.risk = l.add(N * A);
  o.mcall = l.add(N);
  o.nshaped = l.add(N);
  o.dend = l.add(N);
  o.nring = l.add(n > 1 ? N * n * D * 8 : 0);
  o.nlen = l.add(N * 4);
  o.nhead = l.add(N * 4);
  o.disc = l.add(2 * n * 8);  // gamma^i, then (sortino_shaperB's running pop) (gamma^i)^(1/exp)
  o.src = l.add(A * sizeof(mgn_asset_source));
  o.target = l.add((A + 1) * 8);
  o.rcur = l.add(N * 8);
  o.aux = l.add(c->aux ? N * A * MGN_AUX_WIDTH * 8 : 0);
  o.total = l.total;
  return o;
}

int fail(mgn_env* e, int code, const std::string& msg) {
  if (e) e->err = msg;
  g_error = msg;
  return code;
}

int check_hip(mgn_env* e, hipError_t st, const char* what) {
  if (st == hipSuccess) return MGN_OK;
  return fail(e, MGN_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(st));
}

int validate(const mgn_config* c, const mgn_asset_source* s, std::string& msg) {
  if (!c || !s) { msg = "null config"; return MGN_ERR_ARG; }
  if (c->n_envs < 1) { msg = "n_envs must be >= 1"; return MGN_ERR_LENGTH; }
  if (c->n_assets < 1) { msg = "n_assets must be >= 1"; return MGN_ERR_LENGTH; }
  if (c->n_assets > MGN_MAX_ASSETS) {  // this build's cap: an unsupported config
    msg = "n_assets must be in [1, 64] (MGN_MAX_ASSETS)";
    return MGN_ERR_CONFIG;
  }
  if (c->window < 0) { msg = "window must be >= 0"; return MGN_ERR_CONFIG; }
  if (c->shaper < 0 || c->shaper > MGN_SHAPER_SORTINO_B) { msg = "unknown reward shaper"; return MGN_ERR_CONFIG; }
  if (c->reward_mode < 0 || c->reward_mode > MGN_REWARD_AGENT_PER_ASSET) {
    msg = "unknown reward_mode";
    return MGN_ERR_CONFIG;
  }
  if (c->norm_type < 0 || c->norm_type > MGN_NORM_LOG_STANDARD_NORMAL) {
    msg = "unknown norm_type";
    return MGN_ERR_CONFIG;
  }
  if (c->shaper >= MGN_SHAPER_SORTINO_A && !(c->sortino_exp > 0.)) {
    msg = "sortino_exp must be > 0";
    return MGN_ERR_CONFIG;
  }
  if (c->nstep < 1 || c->nstep > MGN_MAX_NSTEP) {
    msg = "nstep_return must be in [1, 256]";
    return MGN_ERR_CONFIG;
  }
  if (c->nstep_pop != MGN_NSTEP_POP_EXACT && c->nstep_pop != MGN_NSTEP_POP_RUNNING) {
    msg = "unknown nstep_pop";
    return MGN_ERR_CONFIG;
  }
  int n_replay = 0;
  for (int i = 0; i < c->n_assets; ++i) n_replay += s[i].kind == MGN_SRC_REPLAY;
  if (n_replay != 0 && n_replay != c->n_assets) {
    msg = "a replay source supplies every asset of the env (HDFSourceSingle is not a Composite child)";
    return MGN_ERR_CONFIG;
  }
  if (c->n_feats < 0 || c->n_feats > MGN_MAX_ASSETS) { msg = "n_feats must be in [0, 64]"; return MGN_ERR_LENGTH; }
  if (n_replay == 0 && c->n_feats != 0 && c->n_feats != c->n_assets) {
    msg = "generator sources have n_feats == n_assets";
    return MGN_ERR_LENGTH;
  }
  for (int i = 0; i < c->n_assets; ++i) {
    const int k = s[i].kind;
    if (k < MGN_SRC_EXTERNAL || k > MGN_SRC_SINEDYNTREND) {
      msg = "unknown data source kind for asset " + std::to_string(i);
      return MGN_ERR_CONFIG;
    }
    if (k >= MGN_SRC_SINEADDER) {
      const int C = (int)s[i].p[0];
      const int cmax = (k == MGN_SRC_SINEADDER) ? 8 : 4;
      if (!c->aux) {
        msg = "multi-component source kinds need mgn_config.aux = 1 (asset " + std::to_string(i) + ")";
        return MGN_ERR_CONFIG;
      }
      if (C < 1 || C > cmax) {
        msg = "component count out of range for asset " + std::to_string(i);
        return MGN_ERR_LENGTH;
      }
      if (k != MGN_SRC_SINEADDER) {
        for (int j = 0; j < C; ++j)
          if (s[i].p[3 + j] < 2.0 || !(s[i].p[1] >= 1.0)) {
            msg = "wave table length / sample rate invalid for asset " + std::to_string(i);
            return MGN_ERR_CONFIG;
          }
        if (k == MGN_SRC_SINEDYNTREND) {
          const int T = (int)s[i].p[3 + 10 * C];
          if (T < 0 || T > 2) {
            msg = "SineDynamicTrend supports at most 2 trends (asset " + std::to_string(i) + ")";
            return MGN_ERR_LENGTH;
          }
        }
      }
    }
    if (k == MGN_SRC_OUPAIR) {
      const bool first = s[i].p[3] == 0.0;
      const int j = first ? i + 1 : i - 1;
      if (j < 0 || j >= c->n_assets || s[j].kind != MGN_SRC_OUPAIR || (s[j].p[3] == 0.0) == first) {
        msg = "OUPair assets come in adjacent (role 0, role 1) pairs; asset " + std::to_string(i);
        return MGN_ERR_CONFIG;
      }
    }
    if ((k == MGN_SRC_TRENDOU || k == MGN_SRC_TRENDYOU || k == MGN_SRC_SIMPLETREND) &&
        s[i].p[2] < s[i].p[1]) {
      msg = "TrendOU maxPeriod < minPeriod for asset " + std::to_string(i);
      return MGN_ERR_CONFIG;
    }
  }
  return MGN_OK;
}

// MGN_NSTEP_POP_RUNNING granted: the shapers with a running-sum pop, scalar
// rewards, and a discount whose slides stay well conditioned (the sums'
// rounding grows by 1/gamma per pop between the re-sums every n pops)
static bool nst_run_granted(const mgn_env* e) {
  const mgn_config& c = e->cfg;
  if (!(c.nstep_pop == MGN_NSTEP_POP_RUNNING && c.nstep > 1 && e->D == 1 && c.discount > 0. &&
        std::pow(c.discount, (double)c.nstep) >= 1e-3))
    return false;
  if (c.shaper == MGN_SHAPER_SORTINO_B)  // (its second sum slides by gamma^(-1/exp))
    return c.sortino_exp > 0. && std::pow(c.discount, (double)c.nstep / c.sortino_exp) >= 1e-3;
  return c.shaper == MGN_SHAPER_DSR || c.shaper == MGN_SHAPER_DDR || c.shaper == MGN_SHAPER_PPC ||
         c.shaper == MGN_SHAPER_NONE;
}

mgn::KParams kparams(const mgn_env* e) {
  mgn::KParams p;
  const mgn_config& c = e->cfg;
  p.N = e->N; p.A = e->A; p.W = e->W; p.D = e->D; p.F = e->F;
  p.replay = e->replay ? 1 : 0;
  p.ring_log = (e->W > 0 && c.norm_type == MGN_NORM_LOG) ? 1 : 0;
  p.rp_price = e->tape.price; p.rp_feat = e->tape.feats; p.rp_ts = e->tape.ts;
  p.rp_end = e->tape.data_end; p.rp_rows = e->tape.rows; p.rp_stride = e->tape.stride;
  p.env_offset = c.env_offset; p.seed = c.seed;
  p.init_cash = c.init_cash; p.reqM = c.required_margin; p.mainM = c.maintenance_margin;
  p.slip_rel = c.slippage_rel; p.slip_abs = c.slippage_abs; p.tc_rel = c.tc_rel; p.tc_abs = c.tc_abs;
  p.shaper = c.shaper; p.reward_mode = c.reward_mode; p.auto_reset = c.auto_reset;
  p.atoms = c.action_atoms; p.eta = c.adaptation_rate; p.cos_temp = c.cosine_temp;
  p.unit_size = c.unit_size;
  p.sexp = c.sortino_exp;
  p.ablate = e->ablate;
  p.reqm_one = (c.required_margin == 1.0) ? 1 : 0;
  const mgn_views& v = e->v;
  p.L = v.ledger; p.mep = v.mean_entry; p.Bm = v.borrowed; p.P = v.prices;
  p.sx = v.sine_x; p.oum = v.ou_mean; p.dy = v.trend_dy; p.tlen = v.trend_len; p.tfl = v.trend_flags;
  p.cash = v.cash; p.ts = v.timestamp; p.dskip = v.draw_skip; p.sA = v.shaper_a; p.sB = v.shaper_b;
  p.ep = v.ep_stats; p.epstats = v.episode_stats; p.ext = v.ext_prices;
  p.ring = v.ring; p.ring_ts = v.ring_ts; p.rhead = v.ring_head; p.rlen = v.ring_len;
  p.src = e->src_dev; p.src_g = e->src_dev; p.target = e->target_dev;
  p.nstep = c.nstep; p.nring = v.nstep_ring; p.nlen = v.nstep_len; p.nhead = v.nstep_head;
  p.disc = e->disc_dev;
  // MGN_NSTEP_POP_RUNNING: the shapers with a running-sum pop, scalar
  // rewards, and a discount whose slides stay well conditioned (the sums'
  // rounding grows by 1/gamma per pop between the re-sums every n pops)
  p.nst_run = nst_run_granted(e) ? 1 : 0;
  p.nst_rg = p.nst_run ? 1.0 / c.discount : 0.;
  p.nst_rg2 = (p.nst_run && c.shaper == MGN_SHAPER_SORTINO_B) ? 1.0 / std::pow(c.discount, 1.0 / c.sortino_exp) : 0.;
  p.disc2 = e->disc_dev + c.nstep;
  p.rcur = e->v.replay_cursor;
  p.aux = e->v.aux;
  const auto& hb = e->hb[e->hcur];
  p.hist = e->hist_on ? hb.hist : nullptr;
  p.hist_ts = hb.ts;
  p.hend = hb.hend;
  p.hlen = hb.hlen;
  p.hrows = hb.rows;
  return p;
}

template <typename Arg>
void launch(void (*const* fns)(int, const Arg&), int apad, int m, const Arg& a) {
  const int idx = apad <= 1 ? 0 : apad <= 2 ? 1 : apad <= 4 ? 2 : apad <= 8 ? 3 : apad <= 16 ? 4 : apad <= 32 ? 5 : 6;
  fns[idx](m, a);
}
void (*const kStep[7])(int, const mgn::StepArgs&) = {mgn::launch_step_a1, mgn::launch_step_a2, mgn::launch_step_a4, mgn::launch_step_a8, mgn::launch_step_a16, mgn::launch_step_a32, mgn::launch_step_a64};
void (*const kDuo[7])(const mgn::StepArgs&) = {mgn::launch_duo_a1, mgn::launch_duo_a2, mgn::launch_duo_a4, mgn::launch_duo_a8, mgn::launch_duo_a16, mgn::launch_duo_a32, mgn::launch_duo_a64};
void (*const kTrio[7])(const mgn::StepArgs&) = {mgn::launch_trio_a1, mgn::launch_trio_a2, mgn::launch_trio_a4, mgn::launch_trio_a8, mgn::launch_trio_a16, mgn::launch_trio_a32, mgn::launch_trio_a64};
void (*const kInit[7])(int, const mgn::InitArgs&) = {mgn::launch_init_a1, mgn::launch_init_a2, mgn::launch_init_a4, mgn::launch_init_a8, mgn::launch_init_a16, mgn::launch_init_a32, mgn::launch_init_a64};
void (*const kVal[7])(int, const mgn::ValArgs&) = {mgn::launch_val_a1, mgn::launch_val_a2, mgn::launch_val_a4, mgn::launch_val_a8, mgn::launch_val_a16, mgn::launch_val_a32, mgn::launch_val_a64};

void launch_step(const mgn_env* e, const mgn_traj& out, int in_kind, const double* units,
                 const int32_t* aidx, const int8_t* act, int K, hipEvent_t ev0 = nullptr,
                 hipEvent_t ev1 = nullptr);
void launch_init(const mgn_env* e, int mode, const uint8_t* mask);
void launch_val(const mgn_env* e, double* out);

// Lane layout: as few lanes per env as keeps >= 2 waves per SIMD resident
// (256 CUs x 4 SIMDs x 2), so large batches run thread-per-env-like (less
// cross-lane work per env) and small batches spread each env over more lanes.
// the two-role kernel: one lane per asset per role, padded width 2..16,
// generator sources or a replay tape; n-step buffers (generator sources)
// while the envs' rings fit the LDS budget (k_step handles the rest and the
// multi-component sources)
constexpr size_t kDuoNstLds = 64 * 1024;
bool duo_eligible(const mgn_env* e) {
  if (e->apad < 2 || e->apad > 16 || e->cfg.aux) return false;
  if (e->cfg.nstep > 1) {
    const size_t epb = (size_t)(256 / e->apad);  // DUO_BLOCK / 2 lanes per role (mgn_duo.h)
    if (e->replay || epb * e->cfg.nstep * (e->D + 1) * sizeof(double) > kDuoNstLds) return false;
  }
  return true;
}
// the three-role kernel: 1..16 assets (one asset on two lanes per role, the
// second a pad), generator sources (replay tapes at 16 assets on the 256-lane
// layout); one-step rewards or n-step aggregation of a scalar reward (the
// finish role's rings in dynamic LDS), with or without a window (the
// confirmed steps' rows are pushed by its finish role).  Some launches of an
// eligible handle have no instantiation (trio_launchable) and run another
// kernel -- every kernel reads and writes the same state, bit-identically
bool trio_eligible(const mgn_env* e) {
  // (its output indices are k x a 32-bit stride: N (A + 1), N F and N n fit 32 bits)
  const uint64_t row = (uint64_t)(e->A + 1 > e->F ? e->A + 1 : e->F);
  const bool nst_ok = e->cfg.nstep == 1 || e->D == 1;
  // replay tapes: 16 assets at the 256-lane layout (N * 16 >= 256 * 256), n = 1
  const bool rp_ok = !e->replay || (e->apad == 16 && e->cfg.nstep == 1 && (uint64_t)e->N * 16 >= 65536);
  if (!(e->apad >= 1 && e->apad <= 16 && !e->cfg.aux && rp_ok && nst_ok &&
        (uint64_t)e->N * row < (1ull << 32) && (uint64_t)e->N * (uint64_t)e->cfg.nstep < (1ull << 32)))
    return false;
  // n-step: the static arrays plus the envs' rings in dynamic LDS within a
  // workgroup's 160 KiB (2 assets at n = 64 would need more: the two-role /
  // single-role kernels run those)
  if (e->cfg.nstep > 1) {
    // (one asset: the two-lane layout's, APAD 2)
    static size_t (*const lds_of[5])(long long, int, bool) = {nullptr, mgn::trio_nst_lds_a2, mgn::trio_nst_lds_a4,
                                                              mgn::trio_nst_lds_a8, mgn::trio_nst_lds_a16};
    const int idx = e->apad <= 2 ? 1 : e->apad <= 4 ? 2 : e->apad <= 8 ? 3 : 4;
    if (lds_of[idx](e->N, e->cfg.nstep, e->W > 0) > mgn::kTrioLdsMax) return false;
  }
  return true;
}
// the launches of a three-role handle with an instantiation: discrete steps
// (the agent loop) always; units / single orders unless the env has one asset
// or keeps a window with n-step rings
bool trio_launchable(const mgn_env* e, int in_kind) {
  if (in_kind == mgn::IN_DISCRETE) return true;
  return e->apad > 1 && !(e->W > 0 && e->cfg.nstep > 1);
}
// automatic: where the single-role kernel would run one lane per asset (small
// batches: one wave per SIMD), give every asset a second (and a third) lane
// in partner waves
void choose_sched(mgn_env* e) {
  e->trio = false;
  if (e->sched == MGN_SCHED_SINGLE) {
    e->duo = false;
  } else if (e->sched == MGN_SCHED_DUO) {
    e->duo = duo_eligible(e);
  } else if (e->sched == MGN_SCHED_TRIO) {
    e->trio = trio_eligible(e);
    e->duo = !e->trio && duo_eligible(e);
  } else {
    // 16 assets: the three-role kernel where measured faster -- generator
    // sources with one-step rewards and no window (5.2 vs 6.3 us/step at
    // 8192 x 16 TrendOU) and replay tapes (C5: 405 vs 485 us per 64-step launch),
    // and, where its two-slots-per-lane layout runs the agent loop's discrete
    // steps (trio_m2_ok), windowed generator handles too
    // one asset with a window: the two-lane layout's one-wave-per-role grid
    // holds 16384 envs in one round (two workgroups per CU); beyond it the
    // single-role kernel's one lane per env measured faster (R1 at 65536:
    // 1098 vs 1507 us per 64-step launch, profiles/r05c_bench_R1_64k{_single,}.json;
    // at 8192 envs the three-role kernel 337 vs 809, r05c_bench_R1_8k{,_single}.json)
    // -- with the exact n-step pop.  With the running-sum pop (which only the
    // three-role kernel has) it stays faster at every batch: R1 at 65536 695
    // vs 1141 us, at 32768 398 vs 896 (profiles/r06p_*.json)
    const bool one_win_big = e->apad == 1 && e->W > 0 && e->N > 16384 && !nst_run_granted(e);
    e->trio = trio_eligible(e) && e->m == 1 && !one_win_big &&
              (e->apad <= 8 ||
               (e->apad <= 16 && ((e->W == 0 && e->cfg.nstep == 1) || e->replay ||
                                  mgn::trio_m2_ok(e->N, e->A, e->cfg.nstep, e->D, mgn::IN_DISCRETE))));
    e->duo = !e->trio && duo_eligible(e) && e->m == 1;
  }
}
int choose_m(int n_envs, int apad);
// automatic layout: the two-role kernel wherever it is eligible (at C3 it runs
// 2.8e9 env-steps/s at 8192 envs and 3.0e9 at 65536, where the single-role
// layout rule below would pick 4 assets per lane and run 1.7e9); else as few
// lanes per env as keep >= 2 waves per SIMD
void auto_layout(mgn_env* e) {
  if (e->layout_auto)
    e->m = (e->sched != MGN_SCHED_SINGLE && (duo_eligible(e) || trio_eligible(e))) ? 1 : choose_m(e->N, e->apad);
  choose_sched(e);
}

int choose_m(int n_envs, int apad) {
  int m = mgn::min_m(apad);
  while (m < 8 && m < apad) {
    const long long waves = (long long)n_envs * (apad / (2 * m)) / 64;
    if (waves < 2048) break;
    m *= 2;
  }
  return m;
}

void launch_step(const mgn_env* e, const mgn_traj& out, int in_kind, const double* units,
                 const int32_t* aidx, const int8_t* act, int K, hipEvent_t ev0, hipEvent_t ev1) {
  mgn::StepArgs a{kparams(e), out, in_kind, units, aidx, act, K, e->stream, ev0, ev1};
#if !(defined(MGN_DIAG) && defined(MGN_NO_GK))  // diagnostic A/B builds: the generic generator role everywhere
  a.gkind = e->kinds[0];
  for (int i = 1; i < e->A; ++i)
    if (e->kinds[i] != a.gkind) a.gkind = -1;
#endif
  // a 9..16-asset window handle takes the three-role kernel (automatic
  // schedule) for the launches its two-slot layout runs -- discrete steps,
  // trio_m2_ok; its one-slot layout measured slower than the two-role kernel
  // there, so the handle's other launches (units, single orders) run that
  bool trio = e->trio;
  if (trio && e->sched == MGN_SCHED_AUTO && e->apad > 8 && e->W > 0 && !e->replay &&
      !mgn::trio_m2_ok(e->N, e->A, e->cfg.nstep, e->D, in_kind) && duo_eligible(e)) {
    kDuo[4](a);
    return;
  }
  if (trio && !trio_launchable(e, in_kind)) {
    // no three-role instantiation for this launch: the two-role kernel where
    // eligible, else the single-role one (same state, same bits)
    if (duo_eligible(e)) {
      kDuo[e->apad <= 2 ? 1 : e->apad <= 4 ? 2 : e->apad <= 8 ? 3 : 4](a);
      return;
    }
    launch(kStep, e->apad, e->m, a);
    return;
  }
  if (trio) {
    const int idx = e->apad <= 2 ? 1 : e->apad <= 4 ? 2 : e->apad <= 8 ? 3 : 4;
    kTrio[idx](a);
    return;
  }
  if (e->duo) {
    const int idx = e->apad <= 2 ? 1 : e->apad <= 4 ? 2 : e->apad <= 8 ? 3 : 4;
    kDuo[idx](a);
    return;
  }
  launch(kStep, e->apad, e->m, a);
}
void launch_init(const mgn_env* e, int mode, const uint8_t* mask) {
  mgn::InitArgs a{kparams(e), mode, mask, e->stream};
  launch(kInit, e->apad, e->m, a);
}
void launch_val(const mgn_env* e, double* out) {
  mgn::ValArgs a{kparams(e), out, e->stream};
  launch(kVal, e->apad, e->m, a);
}

mgn::RingDesc ring_desc(const mgn_env* e) {
  mgn::RingDesc r;
  r.N = e->N; r.F = e->F; r.Pn = e->A + 1; r.W = e->W; r.norm = e->cfg.norm_type;
  r.prelog = e->cfg.norm_type == MGN_NORM_LOG;  // the step kernel logs at push
  r.transform = MGN_RING_PLAIN; r.ostride = e->F; r.ooff = 0;
  r.ring = e->v.ring; r.ring_ts = e->v.ring_ts; r.head = e->v.ring_head; r.len = e->v.ring_len;
  return r;
}

// StackerDiscrete.current_data: element-parallel for the element-wise
// normalisers; column-parallel (two passes over the window per column) for
// standard_normal
void launch_gather(const mgn::RingDesc& r, double* price, double* port, uint64_t* ts,
                   hipStream_t stream) {
  const int C = r.F + r.Pn;
  if (r.norm == MGN_NORM_STANDARD_NORMAL || r.norm == MGN_NORM_LOG_STANDARD_NORMAL ||
      r.ostride != r.F || r.ooff != 0) {
    const int64_t threads = (int64_t)r.N * C;
    hipLaunchKernelGGL(mgn::k_ring_gather, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                       stream, r, price, port, ts);
  } else if (r.W % 2 == 0 && (size_t)r.W * (C + 1) * 8 <= kGatherLdsBudget) {
    // LDS-staged: envs per workgroup so the staged rows fill ~40 KB (4 per CU)
    const size_t per_env = (size_t)r.W * (C + 1) * 8;
    mgn::GatherLds g;
    g.epb = (int)std::min<size_t>(64, std::max<size_t>(1, kGatherLdsTarget / per_env));
    // small batches (the agent loop's one window per step at a few thousand
    // envs): no fewer than four workgroups per CU, so the chip fills
    g.epb = std::max(1, std::min(g.epb, r.N / (4 * 256)));
    g.inv_f = 1.0f / (float)r.F;
    g.inv_p = 1.0f / (float)r.Pn;
    g.inv_w = 1.0f / (float)r.W;
    const unsigned blocks = (unsigned)((r.N + g.epb - 1) / g.epb);
    hipLaunchKernelGGL(mgn::k_ring_gather_lds, dim3(blocks), dim3(256), per_env * g.epb, stream,
                       r, price, port, ts, g);
  } else if ((int64_t)r.N * r.W * C < ((int64_t)1 << 31) && r.W % 2 == 0) {
    const uint32_t pairs = (uint32_t)((int64_t)r.N * r.W * C / 2);
    const uint32_t per_block = 256 * mgn::GATHER_U;
    hipLaunchKernelGGL(mgn::k_ring_gather_elem, dim3((pairs + per_block - 1) / per_block), dim3(256),
                       0, stream, r, price, port, ts, pairs, 1.0 / (double)(r.W * C), 1.0 / (double)C);
  } else {  // odd window or > 2^31 ring elements: the column-parallel kernel
    const int64_t threads = (int64_t)r.N * C;
    hipLaunchKernelGGL(mgn::k_ring_gather, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                       stream, r, price, port, ts);
  }
}

}  // namespace

extern "C" {

int mgn_abi_version(void) { return MGN_ABI_VERSION; }

size_t mgn_arena_bytes(const mgn_config* cfg) {
  if (!cfg || cfg->n_envs < 1 || cfg->n_assets < 1 || cfg->n_assets > MGN_MAX_ASSETS) return 0;
  return plan(cfg).total;
}

int mgn_create(const mgn_config* cfg, const mgn_asset_source* sources, void* stream, void* arena,
               size_t arena_bytes, mgn_env** out) {
  if (!out) return fail(nullptr, MGN_ERR_ARG, "out handle pointer is null");
  *out = nullptr;
  std::string msg;
  int st = validate(cfg, sources, msg);
  if (st != MGN_OK) return fail(nullptr, st, msg);
  mgn_env* e = new (std::nothrow) mgn_env();
  if (!e) return fail(nullptr, MGN_ERR_DEVICE, "host allocation failed");
  e->cfg = *cfg;
  e->N = cfg->n_envs;
  e->A = cfg->n_assets;
  e->W = cfg->window > 0 ? cfg->window : 0;
  e->D = (cfg->reward_mode == MGN_REWARD_AGENT_PER_ASSET) ? e->A : 1;
  e->F = cfg->n_feats > 0 ? cfg->n_feats : e->A;
  e->cfg.n_feats = e->F;
  e->replay = sources[0].kind == MGN_SRC_REPLAY;
  e->kinds.resize(e->A);
  for (int i = 0; i < e->A; ++i) e->kinds[i] = sources[i].kind;
  e->apad = next_pow2(e->A);
  auto_layout(e);
  e->stream = (hipStream_t)stream;
  const Offsets o = plan(cfg);
  e->arena_bytes = o.total;
  if (arena) {
    if (arena_bytes < o.total) {
      delete e;
      return fail(nullptr, MGN_ERR_LENGTH, "arena smaller than mgn_arena_bytes()");
    }
    e->arena = arena;
    e->own_arena = false;
  } else {
    hipError_t h = hipMalloc(&e->arena, o.total);
    if (h != hipSuccess) {
      delete e;
      return fail(nullptr, MGN_ERR_DEVICE, std::string("hipMalloc: ") + hipGetErrorString(h));
    }
    e->own_arena = true;
  }
  char* b = (char*)e->arena;
  mgn_views& v = e->v;
  v.ledger = (double*)(b + o.L); v.mean_entry = (double*)(b + o.mep); v.borrowed = (double*)(b + o.Bm);
  v.prices = (double*)(b + o.P); v.sine_x = (double*)(b + o.sx); v.ou_mean = (double*)(b + o.oum);
  v.trend_dy = (double*)(b + o.dy); v.trend_len = (int32_t*)(b + o.tlen); v.trend_flags = (uint8_t*)(b + o.tfl);
  v.cash = (double*)(b + o.cash); v.timestamp = (uint64_t*)(b + o.ts);
  v.draw_skip = (uint64_t*)(b + o.dskip);
  v.shaper_a = (double*)(b + o.sA); v.shaper_b = (double*)(b + o.sB);
  v.ep_stats = (double*)(b + o.ep); v.episode_stats = (double*)(b + o.epstats);
  v.ext_prices = (double*)(b + o.ext); v.units = (double*)(b + o.units); v.asset_idx = (int32_t*)(b + o.aidx);
  v.ring = e->W ? (double*)(b + o.ring) : nullptr; v.ring_ts = e->W ? (uint64_t*)(b + o.ring_ts) : nullptr;
  v.ring_head = (int32_t*)(b + o.rhead); v.ring_len = (int32_t*)(b + o.rlen);
  v.win_price = e->W ? (double*)(b + o.wprice) : nullptr; v.win_port = e->W ? (double*)(b + o.wport) : nullptr;
  v.win_ts = e->W ? (uint64_t*)(b + o.wts) : nullptr; v.reset_mask = (uint8_t*)(b + o.mask);
  v.out.reward = (double*)(b + o.reward); v.out.agent_reward = (double*)(b + o.areward);
  v.out.shaped = (double*)(b + o.shaped); v.out.done = (uint8_t*)(b + o.done);
  v.out.obs_price = (double*)(b + o.obsp); v.out.obs_port = (double*)(b + o.obsport);
  v.out.timestamp = (uint64_t*)(b + o.obsts); v.out.tprice = (double*)(b + o.tprice);
  v.out.tunits = (double*)(b + o.tunits); v.out.tcost = (double*)(b + o.tcost);
  v.out.risk = (uint8_t*)(b + o.risk); v.out.margin_call = (uint8_t*)(b + o.mcall);
  v.out.n_shaped = (uint8_t*)(b + o.nshaped);
  v.out.data_end = (uint8_t*)(b + o.dend);
  v.replay_cursor = (int64_t*)(b + o.rcur);
  v.aux = cfg->aux ? (double*)(b + o.aux) : nullptr;
  v.nstep_ring = cfg->nstep > 1 ? (double*)(b + o.nring) : nullptr;
  v.nstep_len = (int32_t*)(b + o.nlen); v.nstep_head = (int32_t*)(b + o.nhead);
  v.n_envs = e->N; v.n_assets = e->A; v.window = e->W; v.reward_dim = e->D;
  v.nstep = cfg->nstep; v.n_feats = e->F;
  e->src_dev = (mgn_asset_source*)(b + o.src);
  e->target_dev = (double*)(b + o.target);
  e->disc_dev = (double*)(b + o.disc);
  // discounts gamma^i = math.pow(gamma, i) (nstep_buffer.py:328), host libm pow
  double disc[2 * MGN_MAX_NSTEP];
  for (int i = 0; i < cfg->nstep; ++i) disc[i] = std::pow(cfg->discount, (double)i);
  // sortino_shaperB's running pop: the discounts' 1/exp-th roots ((x d)^(1/e)
  // of a negative discounted entry = d^(1/e) x^(1/e))
  for (int i = 0; i < cfg->nstep; ++i)
    disc[cfg->nstep + i] = cfg->sortino_exp > 0. ? std::pow(disc[i], 1.0 / cfg->sortino_exp) : 0.;

  int rc = check_hip(e, hipMemsetAsync(e->arena, 0, o.total, e->stream), "hipMemsetAsync");
  if (rc == MGN_OK)
    rc = check_hip(e, hipMemcpyAsync(e->src_dev, sources, sizeof(mgn_asset_source) * e->A,
                                     hipMemcpyHostToDevice, e->stream), "hipMemcpyAsync(src)");
  if (rc == MGN_OK)
    rc = check_hip(e, hipMemcpyAsync(e->target_dev, cfg->desired_portfolio, 8 * (e->A + 1),
                                     hipMemcpyHostToDevice, e->stream), "hipMemcpyAsync(target)");
  if (rc == MGN_OK)
    rc = check_hip(e, hipMemcpyAsync(e->disc_dev, disc, 2 * 8 * cfg->nstep, hipMemcpyHostToDevice,
                                     e->stream), "hipMemcpyAsync(discounts)");
  // the constructor's first getData; a replay handle runs it at mgn_attach_replay
  if (rc == MGN_OK && !e->replay) {
    launch_init(e, 0, nullptr);
    rc = check_hip(e, hipGetLastError(), "k_init_reset");
  }
  if (rc == MGN_OK) rc = check_hip(e, hipStreamSynchronize(e->stream), "hipStreamSynchronize");
  if (rc != MGN_OK) {
    const std::string m = e->err;
    if (e->own_arena) (void)hipFree(e->arena);
    delete e;
    return fail(nullptr, rc, m);
  }
  *out = e;
  return MGN_OK;
}

int mgn_destroy(mgn_env* e) {
  if (!e) return MGN_ERR_ARG;
  (void)hipStreamSynchronize(e->stream);
  if (e->own_arena) (void)hipFree(e->arena);
  if (e->wstream) (void)hipStreamSynchronize(e->wstream);
  for (auto& b : e->hb) {
    if (b.hist) (void)hipFree(b.hist);
    if (b.ts) (void)hipFree(b.ts);
    if (b.hend) (void)hipFree(b.hend);
    if (b.hlen) (void)hipFree(b.hlen);
    if (b.ready) (void)hipEventDestroy(b.ready);
    if (b.read) (void)hipEventDestroy(b.read);
  }
  for (hipEvent_t ev : e->t_step) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : e->t_gather) (void)hipEventDestroy(ev);
  if (e->ag_send) (void)hipFree(e->ag_send);
  delete e;
  return MGN_OK;
}

int mgn_set_stream(mgn_env* e, void* stream) {
  if (!e) return MGN_ERR_ARG;
  e->stream = (hipStream_t)stream;
  return MGN_OK;
}

int mgn_get_views(const mgn_env* e, mgn_views* views) {
  if (!e || !views) return MGN_ERR_ARG;
  *views = e->v;
  return MGN_OK;
}

static int need_tape(mgn_env* e) {
  if (e->replay && !e->attached)
    return fail(e, MGN_ERR_CONFIG, "replay source: attach the replay tape (mgn_attach_replay) first");
  return MGN_OK;
}

int mgn_attach_replay(mgn_env* e, const mgn_replay_tape* t) {
  if (!e) return fail(nullptr, MGN_ERR_ARG, "null handle");
  if (!e->replay) return fail(e, MGN_ERR_CONFIG, "handle was not created with MGN_SRC_REPLAY sources");
  if (!t || !t->price || !t->feats || !t->ts || !t->data_end)
    return fail(e, MGN_ERR_ARG, "null replay tape pointer");
  if (t->rows < 1) return fail(e, MGN_ERR_LENGTH, "replay tape needs >= 1 row");
  if (t->stride < 0) return fail(e, MGN_ERR_CONFIG, "replay stride must be >= 0");
  e->tape = *t;
  e->attached = true;
  launch_init(e, 0, nullptr);
  return check_hip(e, hipGetLastError(), "mgn_attach_replay");
}

int mgn_reset(mgn_env* e, const uint8_t* mask_dev) {
  if (!e) return fail(nullptr, MGN_ERR_ARG, "null handle");
  if (need_tape(e) != MGN_OK) return MGN_ERR_CONFIG;
  launch_init(e, 1, mask_dev);
  return check_hip(e, hipGetLastError(), "mgn_reset");
}

int mgn_step(mgn_env* e, int32_t kind, const double* units_dev, const int32_t* aidx_dev) {
  if (!e) return fail(nullptr, MGN_ERR_ARG, "null handle");
  int in_kind;
  if (kind == MGN_STEP_NONE) in_kind = mgn::IN_NONE;
  else if (kind == MGN_STEP_UNITS) in_kind = mgn::IN_UNITS;
  else if (kind == MGN_STEP_SINGLE) in_kind = mgn::IN_SINGLE;
  else return fail(e, MGN_ERR_CONFIG, "unknown step kind");
  if (in_kind != mgn::IN_NONE && !units_dev) return fail(e, MGN_ERR_ARG, "units pointer is null");
  if (in_kind == mgn::IN_SINGLE && !aidx_dev) return fail(e, MGN_ERR_ARG, "asset index pointer is null");
  if (need_tape(e) != MGN_OK) return MGN_ERR_CONFIG;
  launch_step(e, e->v.out, in_kind, units_dev, aidx_dev, nullptr, 1);
  return check_hip(e, hipGetLastError(), "mgn_step");
}

static void time_mark(mgn_env* e, std::vector<hipEvent_t>& v, size_t& n, hipStream_t st);
static bool time_pair(mgn_env* e, hipEvent_t& a, hipEvent_t& b);

int mgn_rollout(mgn_env* e, const int8_t* actions_dev, int32_t k_steps, const mgn_traj* out) {
  if (!e) return fail(nullptr, MGN_ERR_ARG, "null handle");
  if (!actions_dev || !out) return fail(e, MGN_ERR_ARG, "null actions/out");
  if (k_steps < 1) return fail(e, MGN_ERR_LENGTH, "k_steps must be >= 1");
  if (need_tape(e) != MGN_OK) return MGN_ERR_CONFIG;
  hipEvent_t a = nullptr, b = nullptr;
  if (e->timing == 2) (void)time_pair(e, a, b);
  else time_mark(e, e->t_step, e->t_step_n, e->stream);
  launch_step(e, *out, mgn::IN_DISCRETE, nullptr, nullptr, actions_dev, (int)k_steps, a, b);
  if (e->timing != 2) time_mark(e, e->t_step, e->t_step_n, e->stream);
  return check_hip(e, hipGetLastError(), "mgn_rollout");
}

int mgn_rollout_units(mgn_env* e, const double* units_dev, int32_t k_steps, const mgn_traj* out) {
  if (!e) return fail(nullptr, MGN_ERR_ARG, "null handle");
  if (!units_dev || !out) return fail(e, MGN_ERR_ARG, "null units/out");
  if (k_steps < 1) return fail(e, MGN_ERR_LENGTH, "k_steps must be >= 1");
  if (need_tape(e) != MGN_OK) return MGN_ERR_CONFIG;
  launch_step(e, *out, mgn::IN_UNITS, units_dev, nullptr, nullptr, (int)k_steps);
  return check_hip(e, hipGetLastError(), "mgn_rollout_units");
}

int mgn_set_prices(mgn_env* e, const double* prices_dev) {
  if (!e || !prices_dev) return fail(e, MGN_ERR_ARG, "null handle/prices");
  return check_hip(e, hipMemcpyAsync(e->v.ext_prices, prices_dev, sizeof(double) * e->N * e->A,
                                     hipMemcpyDeviceToDevice, e->stream), "mgn_set_prices");
}

int mgn_set_sources(mgn_env* e, const mgn_asset_source* sources, const double* prices_dev) {
  if (!e) return fail(nullptr, MGN_ERR_ARG, "null handle");
  if (!sources) return fail(e, MGN_ERR_ARG, "null source table");
  if (e->replay) return fail(e, MGN_ERR_CONFIG, "a replay handle cannot switch its data source");
  std::vector<mgn_asset_source> cur(e->A);
  int rc = check_hip(e, hipMemcpyAsync(cur.data(), e->src_dev, sizeof(mgn_asset_source) * e->A,
                                       hipMemcpyDeviceToHost, e->stream), "mgn_set_sources (read)");
  if (rc == MGN_OK) rc = check_hip(e, hipStreamSynchronize(e->stream), "mgn_set_sources (sync)");
  if (rc != MGN_OK) return rc;
  for (int i = 0; i < e->A; ++i) {
    const int k = sources[i].kind;
    if (k != MGN_SRC_EXTERNAL && k != cur[i].kind)
      return fail(e, MGN_ERR_CONFIG, "asset " + std::to_string(i) +
                                         ": a new source is MGN_SRC_EXTERNAL or the asset's current kind");
  }
  std::string msg;
  const int st = validate(&e->cfg, sources, msg);
  if (st != MGN_OK) return fail(e, st, msg);
  std::memcpy(cur.data(), sources, sizeof(mgn_asset_source) * e->A);
  for (int i = 0; i < e->A; ++i) e->kinds[i] = sources[i].kind;
  rc = check_hip(e, hipMemcpyAsync(e->src_dev, cur.data(), sizeof(mgn_asset_source) * e->A,
                                   hipMemcpyHostToDevice, e->stream), "mgn_set_sources (write)");
  if (rc == MGN_OK && prices_dev)
    rc = check_hip(e, hipMemcpyAsync(e->v.prices, prices_dev, sizeof(double) * e->N * e->A,
                                     hipMemcpyDeviceToDevice, e->stream), "mgn_set_sources (prices)");
  if (rc == MGN_OK) rc = check_hip(e, hipStreamSynchronize(e->stream), "mgn_set_sources (sync)");
  return rc;
}

int mgn_window_push(mgn_env* e, const double* price_dev, const double* port_dev, const uint64_t* ts_dev) {
  if (!e) return fail(nullptr, MGN_ERR_ARG, "null handle");
  if (e->W == 0) return fail(e, MGN_ERR_CONFIG, "handle has no window (window_length = 0)");
  const mgn::RingDesc r = ring_desc(e);
  const double* pr = price_dev ? price_dev : e->v.out.obs_price;
  const double* po = port_dev ? port_dev : e->v.out.obs_port;
  const uint64_t* t = ts_dev ? ts_dev : e->v.out.timestamp;
  hipLaunchKernelGGL(mgn::k_ring_push, dim3((e->N + 255) / 256), dim3(256), 0, e->stream, r, pr, po, t);
  return check_hip(e, hipGetLastError(), "mgn_window_push");
}

int mgn_window_clear(mgn_env* e, const uint8_t* mask_dev) {
  if (!e) return fail(nullptr, MGN_ERR_ARG, "null handle");
  if (e->W == 0) return fail(e, MGN_ERR_CONFIG, "handle has no window (window_length = 0)");
  hipLaunchKernelGGL(mgn::k_ring_clear, dim3((e->N + 255) / 256), dim3(256), 0, e->stream,
                     ring_desc(e), mask_dev);
  return check_hip(e, hipGetLastError(), "mgn_window_clear");
}

static void time_mark(mgn_env* e, std::vector<hipEvent_t>& v, size_t& n, hipStream_t st);

int mgn_window(mgn_env* e, double* price_dev, double* port_dev, uint64_t* ts_dev) {
  if (!e) return fail(nullptr, MGN_ERR_ARG, "null handle");
  if (e->W == 0) return fail(e, MGN_ERR_CONFIG, "handle has no window (window_length = 0)");
  time_mark(e, e->t_gather, e->t_gather_n, e->stream);
  launch_gather(ring_desc(e), price_dev ? price_dev : e->v.win_price,
                port_dev ? port_dev : e->v.win_port, ts_dev ? ts_dev : e->v.win_ts, e->stream);
  time_mark(e, e->t_gather, e->t_gather_n, e->stream);
  return check_hip(e, hipGetLastError(), "mgn_window");
}

static void time_mark(mgn_env* e, std::vector<hipEvent_t>& v, size_t& n, hipStream_t st) {
  if (!e->timing) return;
  if (n == v.size()) {
    hipEvent_t ev;
    if (hipEventCreate(&ev) != hipSuccess) return;
    v.push_back(ev);
  }
  (void)hipEventRecord(v[n++], st);
}

// mode 2: the next start / stop pair of the step pool, recorded by the launch
static bool time_pair(mgn_env* e, hipEvent_t& a, hipEvent_t& b) {
  while (e->t_step.size() < e->t_step_n + 2) {
    hipEvent_t ev;
    if (hipEventCreate(&ev) != hipSuccess) return false;
    e->t_step.push_back(ev);
  }
  a = e->t_step[e->t_step_n];
  b = e->t_step[e->t_step_n + 1];
  e->t_step_n += 2;
  return true;
}

static int grow(mgn_env* e, void** p, size_t bytes) {
  (void)hipDeviceSynchronize();  // first use / larger K only
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  return check_hip(e, hipMalloc(p, bytes), "history alloc");
}

int mgn_set_window_stream(mgn_env* e, void* stream) {
  if (!e) return fail(nullptr, MGN_ERR_ARG, "null handle");
  (void)hipStreamSynchronize(e->stream);
  if (e->wstream) (void)hipStreamSynchronize(e->wstream);
  e->wstream = (hipStream_t)stream;
  for (auto& b : e->hb) {
    if (!b.ready && hipEventCreateWithFlags(&b.ready, hipEventDisableTiming) != hipSuccess)
      return fail(e, MGN_ERR_DEVICE, "event create");
    if (!b.read && hipEventCreateWithFlags(&b.read, hipEventDisableTiming) != hipSuccess)
      return fail(e, MGN_ERR_DEVICE, "event create");
  }
  return MGN_OK;
}

int mgn_set_timing(mgn_env* e, int32_t on) {
  if (!e) return fail(nullptr, MGN_ERR_ARG, "null handle");
  (void)hipDeviceSynchronize();
  e->t_step_n = 0;
  e->t_gather_n = 0;
  if (on < 0 || on > 2) return fail(e, MGN_ERR_CONFIG, "mgn_set_timing: 0 off, 1 marker events, 2 launch events");
  e->timing = on;
  return MGN_OK;
}

int mgn_get_timing(mgn_env* e, double* out4) {
  if (!e || !out4) return fail(e, MGN_ERR_ARG, "null handle/out");
  const std::vector<hipEvent_t>* v[2] = {&e->t_step, &e->t_gather};
  const size_t cnt[2] = {e->t_step_n, e->t_gather_n};
  for (int i = 0; i < 2; ++i) {
    double ms = 0.;
    const size_t n = cnt[i] / 2;
    for (size_t j = 0; j < n; ++j) {
      float t = 0.f;
      (void)hipEventSynchronize((*v[i])[2 * j + 1]);
      if (hipEventElapsedTime(&t, (*v[i])[2 * j], (*v[i])[2 * j + 1]) == hipSuccess) ms += t;
    }
    out4[2 * i] = ms;
    out4[2 * i + 1] = (double)n;
  }
  return MGN_OK;
}

int mgn_rollout_hist(mgn_env* e, const int8_t* actions_dev, int32_t k_steps, const mgn_traj* out) {
  if (!e) return fail(nullptr, MGN_ERR_ARG, "null handle");
  if (!actions_dev || !out) return fail(e, MGN_ERR_ARG, "null actions/out");
  if (k_steps < 1) return fail(e, MGN_ERR_LENGTH, "k_steps must be >= 1");
  if (e->W == 0) return fail(e, MGN_ERR_CONFIG, "handle has no window (window_length = 0)");
  if (e->W % 2) return fail(e, MGN_ERR_CONFIG, "the launch history needs an even window length");
  if (k_steps > mgn::HIST_KMAX) return fail(e, MGN_ERR_LENGTH, "the launch history holds at most 64 steps");
  if (need_tape(e) != MGN_OK) return MGN_ERR_CONFIG;
  const int C = e->F + e->A + 1;
  const size_t rows = (size_t)e->W + (size_t)k_steps * (e->W + 1);
  if ((size_t)e->N * rows * C >= ((size_t)1 << 31))
    return fail(e, MGN_ERR_LENGTH, "launch history exceeds 2^31 elements: fewer steps per call");
  // with a window stream, alternate buffers; the step launch waits until the
  // gather that last read its buffer has finished
  const int b = e->wstream ? (e->hcur ^ 1) : 0;
  auto& hb = e->hb[b];
  int st = MGN_OK;
  if (rows > hb.rows_cap) {
    hb.rows_cap = 0;
    st = grow(e, (void**)&hb.hist, (size_t)e->N * rows * C * 8);
    if (st == MGN_OK) st = grow(e, (void**)&hb.ts, (size_t)e->N * rows * 8);
    if (st != MGN_OK) return st;
    hb.rows_cap = rows;
  }
  if ((size_t)k_steps > hb.k_cap) {
    hb.k_cap = 0;
    st = grow(e, (void**)&hb.hend, (size_t)k_steps * e->N * 4);
    if (st == MGN_OK) st = grow(e, (void**)&hb.hlen, (size_t)k_steps * e->N * 4);
    if (st != MGN_OK) return st;
    hb.k_cap = (size_t)k_steps;
  }
  if (e->wstream && hb.k > 0) (void)hipStreamWaitEvent(e->stream, hb.read, 0);
  e->hcur = b;
  hb.rows = (int)rows;
  const mgn::RingDesc r = ring_desc(e);
  hipLaunchKernelGGL(mgn::k_hist_prefix, dim3((unsigned)e->N), dim3(256), 0, e->stream, r, hb.hist,
                     hb.ts, (int)rows);
  time_mark(e, e->t_step, e->t_step_n, e->stream);
  e->hist_on = true;
  launch_step(e, *out, mgn::IN_DISCRETE, nullptr, nullptr, actions_dev, (int)k_steps);
  e->hist_on = false;
  time_mark(e, e->t_step, e->t_step_n, e->stream);
  hb.k = k_steps;
  if (e->wstream) (void)hipEventRecord(hb.ready, e->stream);
  return check_hip(e, hipGetLastError(), "mgn_rollout_hist");
}

int mgn_window_hist(mgn_env* e, double* price_dev, double* port_dev, uint64_t* ts_dev) {
  if (!e) return fail(nullptr, MGN_ERR_ARG, "null handle");
  auto& hb = e->hb[e->hcur];
  if (hb.k == 0) return fail(e, MGN_ERR_CONFIG, "no mgn_rollout_hist to gather from");
  if (!price_dev && !port_dev && !ts_dev) return MGN_OK;
  const int C = e->F + e->A + 1;
  mgn::HistDesc h;
  h.N = e->N; h.F = e->F; h.Pn = e->A + 1; h.W = e->W; h.K = hb.k; h.hrows = hb.rows;
  h.norm = e->cfg.norm_type;
  h.prelog = e->cfg.norm_type == MGN_NORM_LOG;
  h.hist = hb.hist; h.hist_ts = hb.ts; h.hend = hb.hend; h.hlen = hb.hlen;
  if (h.norm == MGN_NORM_STANDARD_NORMAL || h.norm == MGN_NORM_LOG_STANDARD_NORMAL)
    return fail(e, MGN_ERR_CONFIG, "mgn_window_hist: element-wise normalisers only (none, log, lookback, lookback_log)");
  // LDS rows: the window before the launch, one row per step and one reset's
  // refill; a longer span reads the history directly
  // steps per workgroup: 16, doubled (up to the launch's K) until a
  // workgroup writes >= 80 KB -- its two dependent memory round trips (the
  // history marks, then the staged rows) are paid once per workgroup, so
  // narrow rows need more windows per workgroup (R1, 2 KB per window: 0.47 of
  // 8 TB/s at 16 steps, 0.66 at 64; C2 / C4 / C5, 5-17 KB per window: best at
  // 16; profiles/r06n_gather_ks_ab.txt)
  int ks = std::min(h.K, kHistStepsPerGroup);
  while (ks < std::min(h.K, mgn::HIST_KMAX) && (size_t)ks * e->W * (C + 1) * 8 < kHistGroupBytes)
    ks = std::min(2 * ks, std::min(h.K, mgn::HIST_KMAX));
  const int kb = (h.K + ks - 1) / ks;
  const int lds_rows = std::min(e->W + ks + (e->W + 1), (int)(kGatherLdsBudget / ((size_t)(C + 1) * 8)));
  const size_t lds = (size_t)lds_rows * (C + 1) * 8;
  const float wf = (float)(e->W * e->F), wp = (float)(e->W * (e->A + 1));
  hipStream_t st = e->wstream ? e->wstream : e->stream;
  if (e->wstream) (void)hipStreamWaitEvent(st, hb.ready, 0);
  time_mark(e, e->t_gather, e->t_gather_n, st);
  hipLaunchKernelGGL(mgn::k_hist_gather, dim3((unsigned)(e->N * kb)), dim3(256), lds, st, h,
                     price_dev, port_dev, ts_dev, ks, lds_rows, 1.0f / (float)e->F, 1.0f / (float)(e->A + 1),
                     1.0f / (float)e->W, 1.0f / wf, 1.0f / wp);
  time_mark(e, e->t_gather, e->t_gather_n, st);
  if (e->wstream) (void)hipEventRecord(hb.read, st);
  return check_hip(e, hipGetLastError(), "mgn_window_hist");
}

int mgn_window_hist_view(mgn_env* e, mgn_hist_view* out) {
  if (!e || !out) return fail(e, MGN_ERR_ARG, "null handle/out");
  const auto& hb = e->hb[e->hcur];
  if (hb.k == 0) return fail(e, MGN_ERR_CONFIG, "no mgn_rollout_hist to view");
  const int nt = e->cfg.norm_type;
  if (nt != MGN_NORM_NONE && nt != MGN_NORM_LOG)
    return fail(e, MGN_ERR_CONFIG, "mgn_window_hist_view: windows are history rows only for norm none / log");
  out->hist = hb.hist;
  out->hist_ts = hb.ts;
  out->hend = hb.hend;
  out->hlen = hb.hlen;
  out->rows = hb.rows;
  out->cols = e->F + e->A + 1;
  out->k_steps = hb.k;
  out->window = e->W;
  out->n_feats = e->F;
  out->pad_ = 0;
  // the history is written on the handle's stream: order a window-stream
  // consumer after it as mgn_window_hist would
  if (e->wstream) (void)hipStreamWaitEvent(e->wstream, hb.ready, 0);
  return MGN_OK;
}

int mgn_rollout_window(mgn_env* e, const int8_t* actions_dev, int32_t k_steps, const mgn_traj* out,
                       double* price_dev, double* port_dev, uint64_t* ts_dev, int32_t per_step) {
  if (!e) return fail(nullptr, MGN_ERR_ARG, "null handle");
  if (per_step) {
    if (!price_dev || !port_dev) return fail(e, MGN_ERR_ARG, "per_step windows need caller price/port buffers");
    const int st = mgn_rollout_hist(e, actions_dev, k_steps, out);
    return st != MGN_OK ? st : mgn_window_hist(e, price_dev, port_dev, ts_dev);
  }
  const int st = mgn_rollout(e, actions_dev, k_steps, out);
  return st != MGN_OK ? st : mgn_window(e, price_dev, port_dev, ts_dev);
}

int mgn_generate_actions(mgn_env* e, int8_t* actions_dev, int32_t k_steps, uint64_t seed) {
  if (!e || !actions_dev) return fail(e, MGN_ERR_ARG, "null handle/actions");
  if (k_steps < 1) return fail(e, MGN_ERR_LENGTH, "k_steps must be >= 1");
  const int64_t total = (int64_t)k_steps * e->N * e->A;
  if ((total + 255) / 256 > (int64_t)0x7fffffff) return fail(e, MGN_ERR_LENGTH, "too many actions for one launch");
  hipLaunchKernelGGL(mgn::k_gen_actions, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     e->stream, actions_dev, (int)k_steps, e->N, e->A, e->cfg.action_atoms, seed,
                     e->cfg.env_offset);
  return check_hip(e, hipGetLastError(), "mgn_generate_actions");
}

int mgn_ledger_op(mgn_env* e, int32_t op, const int32_t* aidx_dev, const double* units_dev,
                  const double* tprice_dev, const double* tcost_dev, const mgn_traj* out) {
  if (!e) return fail(nullptr, MGN_ERR_ARG, "null handle");
  if (op < MGN_OP_BROKER_UNITS || op > MGN_OP_CHECK_ORDER) return fail(e, MGN_ERR_CONFIG, "unknown ledger op");
  if (!units_dev && op != MGN_OP_BROKER_CLOSE && op != MGN_OP_PORT_CLOSE)
    return fail(e, MGN_ERR_ARG, "units pointer is null");
  if (!aidx_dev && op != MGN_OP_BROKER_UNITS) return fail(e, MGN_ERR_ARG, "asset index pointer is null");
  if (!tprice_dev && (op == MGN_OP_PORT_TXN || op == MGN_OP_PORT_CLOSE))
    return fail(e, MGN_ERR_ARG, "transaction price pointer is null");
  if (need_tape(e) != MGN_OK) return MGN_ERR_CONFIG;
  mgn::LedgerOp o{};
  o.op = op;
  o.aidx = aidx_dev;
  o.units = units_dev;
  o.tprice = tprice_dev;
  o.tcost = tcost_dev;
  if (out) {
    o.o_tp = out->tprice;
    o.o_tu = out->tunits;
    o.o_tc = out->tcost;
    o.o_risk = out->risk;
    o.o_mc = out->margin_call;
  }
  hipLaunchKernelGGL(mgn::k_ledger_op, dim3((unsigned)((e->N + mgn::BLOCK - 1) / mgn::BLOCK)), dim3(mgn::BLOCK), 0,
                     e->stream, kparams(e), o);
  return check_hip(e, hipGetLastError(), "mgn_ledger_op");
}

int mgn_valuation(mgn_env* e, double* out_dev) {
  if (!e || !out_dev) return fail(e, MGN_ERR_ARG, "null handle/out");
  launch_val(e, out_dev);
  return check_hip(e, hipGetLastError(), "mgn_valuation");
}

int mgn_set_broker(mgn_env* e, double required_margin, double maintenance_margin,
                   double slippage_rel, double slippage_abs, double tc_rel, double tc_abs) {
  if (!e) return fail(nullptr, MGN_ERR_ARG, "null handle");
  e->cfg.required_margin = required_margin;
  e->cfg.maintenance_margin = maintenance_margin;
  e->cfg.slippage_rel = slippage_rel;
  e->cfg.slippage_abs = slippage_abs;
  e->cfg.tc_rel = tc_rel;
  e->cfg.tc_abs = tc_abs;
  return MGN_OK;
}

static mgn::RingDesc ring_from(const mgn_ring* r) {
  mgn::RingDesc d;
  d.N = r->n_envs; d.F = r->n_price; d.Pn = r->n_port; d.W = r->window; d.norm = r->norm_type;
  d.prelog = 0;
  d.transform = r->transform;
  d.ostride = r->out_stride > 0 ? r->out_stride : r->n_price;
  d.ooff = r->out_offset;
  d.ring = r->ring; d.ring_ts = r->ring_ts; d.head = r->head; d.len = r->len;
  return d;
}

static int ring_ok(const mgn_ring* r) {
  if (!r || !r->ring || !r->ring_ts || !r->head || !r->len) return fail(nullptr, MGN_ERR_ARG, "null ring buffers");
  if (r->n_envs < 1 || r->window < 1 || r->n_price < 0 || r->n_port < 0)
    return fail(nullptr, MGN_ERR_LENGTH, "bad ring dimensions");
  if (r->norm_type < 0 || r->norm_type > MGN_NORM_LOG_STANDARD_NORMAL)
    return fail(nullptr, MGN_ERR_CONFIG, "unknown norm_type");
  if (r->transform != MGN_RING_PLAIN && !(r->transform == MGN_RING_PAIR_RATIO && r->n_price == 1))
    return fail(nullptr, MGN_ERR_CONFIG, "ring transform PAIR_RATIO stores one price column");
  if (r->out_offset < 0 || (r->out_stride > 0 && r->out_offset + r->n_price > r->out_stride))
    return fail(nullptr, MGN_ERR_LENGTH, "gathered price columns exceed out_stride");
  return MGN_OK;
}

int mgn_ring_push(const mgn_ring* r, const double* price_dev, const double* port_dev,
                  const uint64_t* ts_dev, void* stream) {
  int rc = ring_ok(r);
  if (rc != MGN_OK) return rc;
  hipLaunchKernelGGL(mgn::k_ring_push, dim3((r->n_envs + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     ring_from(r), price_dev, port_dev, ts_dev);
  return check_hip(nullptr, hipGetLastError(), "mgn_ring_push");
}

int mgn_ring_clear(const mgn_ring* r, const uint8_t* mask_dev, void* stream) {
  int rc = ring_ok(r);
  if (rc != MGN_OK) return rc;
  hipLaunchKernelGGL(mgn::k_ring_clear, dim3((r->n_envs + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     ring_from(r), mask_dev);
  return check_hip(nullptr, hipGetLastError(), "mgn_ring_clear");
}

int mgn_ring_gather(const mgn_ring* r, double* price_dev, double* port_dev, uint64_t* ts_dev, void* stream) {
  int rc = ring_ok(r);
  if (rc != MGN_OK) return rc;
  launch_gather(ring_from(r), price_dev, port_dev, ts_dev, (hipStream_t)stream);
  return check_hip(nullptr, hipGetLastError(), "mgn_ring_gather");
}

int mgn_feat_diff(const double* in_dev, double* out_dev, int64_t rows, int32_t cols, void* stream) {
  if (!in_dev || !out_dev) return fail(nullptr, MGN_ERR_ARG, "null buffers");
  if (rows < 0 || cols < 1) return fail(nullptr, MGN_ERR_LENGTH, "bad diff dimensions");
  const int64_t n = rows * (int64_t)(cols - 1);
  if (n == 0) return MGN_OK;
  hipLaunchKernelGGL(mgn::k_feat_diff, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, in_dev, out_dev, rows, (int)cols);
  return check_hip(nullptr, hipGetLastError(), "mgn_feat_diff");
}

int mgn_set_layout(mgn_env* e, int32_t assets_per_lane) {
  if (!e) return fail(nullptr, MGN_ERR_ARG, "null handle");
  if (assets_per_lane == 0) {
    e->layout_auto = true;
    auto_layout(e);
    return MGN_OK;
  }
  if (assets_per_lane != 1 && assets_per_lane != 2 && assets_per_lane != 4 && assets_per_lane != 8)
    return fail(e, MGN_ERR_CONFIG, "assets_per_lane must be 0 (auto), 1, 2, 4 or 8");
  int m = assets_per_lane < e->apad ? assets_per_lane : e->apad;
  if (m < mgn::min_m(e->apad)) m = mgn::min_m(e->apad);
  e->m = m;
  e->layout_auto = false;
  choose_sched(e);
  return MGN_OK;
}

int mgn_set_schedule(mgn_env* e, int32_t schedule) {
  if (!e) return fail(nullptr, MGN_ERR_ARG, "null handle");
  if (schedule < MGN_SCHED_AUTO || schedule > MGN_SCHED_TRIO)
    return fail(e, MGN_ERR_CONFIG, "schedule must be MGN_SCHED_AUTO, _SINGLE, _DUO or _TRIO");
  if (schedule == MGN_SCHED_DUO && !duo_eligible(e))
    return fail(e, MGN_ERR_CONFIG,
                "the two-role kernel needs 2..16 assets, no multi-component source, n-step rings within LDS");
  if (schedule == MGN_SCHED_TRIO && !trio_eligible(e))
    return fail(e, MGN_ERR_CONFIG,
                "the three-role kernel needs 2..16 assets, generator sources (or a replay tape at 16 assets), nstep 1 or a scalar n-step reward without a window whose rings fit LDS");
  e->sched = schedule;
  auto_layout(e);
  return MGN_OK;
}

int mgn_get_schedule(const mgn_env* e) {
  return e ? (e->trio ? MGN_SCHED_TRIO : e->duo ? MGN_SCHED_DUO : MGN_SCHED_SINGLE) : 0;
}

int mgn_get_layout(const mgn_env* e) { return e ? e->m : 0; }

#ifdef MGN_DIAG
// diagnostic builds only (tools/build_variant.py), not part of the product
// ABI: timing ablations whose outputs are wrong -- bit 0 skips the Broker
// rounds, bit 1 the generators, bit 2 the output stores, bit 3 the agent
// reward's logarithms (k_step / k_step_duo)
int mgn_set_ablation(mgn_env* e, int32_t flags) {
  if (!e) return MGN_ERR_ARG;
  e->ablate = flags;
  return MGN_OK;
}
#endif

// RCCL entry points from the library instance the process already has loaded
// (torch's, when the communicator is torch's); librccl.so.1 otherwise
static void* rccl_sym(const char* name) {
  void* f = dlsym(RTLD_DEFAULT, name);
  if (f) return f;
  static void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  return h ? dlsym(h, name) : nullptr;
}

int mgn_stats_allgather(mgn_env* e, void* comm, int32_t rows_per_rank, double* out_dev) {
  if (!e) return fail(nullptr, MGN_ERR_ARG, "null handle");
  if (!comm || !out_dev) return fail(e, MGN_ERR_ARG, "null communicator/output");
  const size_t rows = rows_per_rank == 0 ? (size_t)e->N : (size_t)rows_per_rank;
  if (rows_per_rank < 0 || rows < (size_t)e->N)
    return fail(e, MGN_ERR_LENGTH, "rows_per_rank must be >= n_envs (0: n_envs)");
  using AllGather = ncclResult_t (*)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
  using ErrStr = const char* (*)(ncclResult_t);
  const auto ag = reinterpret_cast<AllGather>(rccl_sym("ncclAllGather"));
  const auto es = reinterpret_cast<ErrStr>(rccl_sym("ncclGetErrorString"));
  if (!ag) return fail(e, MGN_ERR_DEVICE, "ncclAllGather not found (no RCCL in the process, no librccl.so.1)");
  const double* send = e->v.episode_stats;
  if (rows > (size_t)e->N) {
    if (rows > e->ag_rows) {
      if (e->ag_send) (void)hipFree(e->ag_send);
      e->ag_send = nullptr;
      e->ag_rows = 0;
      const int rc = check_hip(e, hipMalloc(&e->ag_send, rows * 4 * sizeof(double)), "allgather staging");
      if (rc != MGN_OK) return rc;
      e->ag_rows = rows;
    }
    int rc = check_hip(e, hipMemcpyAsync(e->ag_send, e->v.episode_stats, (size_t)e->N * 4 * sizeof(double),
                                         hipMemcpyDeviceToDevice, e->stream), "allgather staging copy");
    if (rc == MGN_OK)
      rc = check_hip(e, hipMemsetAsync(e->ag_send + (size_t)e->N * 4, 0, (rows - e->N) * 4 * sizeof(double),
                                       e->stream), "allgather staging pad");
    if (rc != MGN_OK) return rc;
    send = e->ag_send;
  }
  const ncclResult_t r = ag(send, out_dev, rows * 4, ncclFloat64, (ncclComm_t)comm, e->stream);
  if (r != ncclSuccess)
    return fail(e, MGN_ERR_DEVICE, std::string("ncclAllGather: ") + (es ? es(r) : std::to_string((int)r)));
  return MGN_OK;
}

namespace {
struct StateHeader {
  char magic[8];
  int32_t abi;
  int32_t replay;  // the handle's sources are a replay tape (MGN_SRC_REPLAY)
  uint64_t arena_bytes;
  mgn_config cfg;
};
constexpr char kStateMagic[8] = {'M', 'G', 'N', 'S', 'T', 'A', 'T', 'E'};
}  // namespace

size_t mgn_state_bytes(const mgn_env* e) { return e ? sizeof(StateHeader) + e->arena_bytes : 0; }

int mgn_save_state(mgn_env* e, void* dst, size_t bytes) {
  if (!e || !dst) return fail(e, MGN_ERR_ARG, "null handle/destination");
  if (bytes < mgn_state_bytes(e)) return fail(e, MGN_ERR_LENGTH, "destination smaller than mgn_state_bytes()");
  StateHeader h{};
  std::memcpy(h.magic, kStateMagic, 8);
  h.abi = MGN_ABI_VERSION;
  h.replay = e->replay ? 1 : 0;
  h.arena_bytes = e->arena_bytes;
  h.cfg = e->cfg;
  std::memcpy(dst, &h, sizeof h);
  int rc = check_hip(e, hipMemcpyAsync((char*)dst + sizeof h, e->arena, e->arena_bytes, hipMemcpyDeviceToHost,
                                       e->stream), "mgn_save_state");
  if (rc == MGN_OK) rc = check_hip(e, hipStreamSynchronize(e->stream), "mgn_save_state (sync)");
  return rc;
}

int mgn_load_state(mgn_env* e, const void* src, size_t bytes) {
  if (!e || !src) return fail(e, MGN_ERR_ARG, "null handle/source");
  StateHeader h;
  if (bytes < sizeof h) return fail(e, MGN_ERR_LENGTH, "state blob too small");
  std::memcpy(&h, src, sizeof h);
  if (std::memcmp(h.magic, kStateMagic, 8) != 0) return fail(e, MGN_ERR_CONFIG, "not a madigan_amd state blob");
  if (h.abi != MGN_ABI_VERSION) return fail(e, MGN_ERR_CONFIG, "state blob of another ABI version");
  const mgn_config& c = h.cfg;
  const mgn_config& m = e->cfg;
  if (h.arena_bytes != e->arena_bytes || bytes < sizeof h + h.arena_bytes || c.n_envs != m.n_envs ||
      c.n_assets != m.n_assets || c.window != m.window || c.reward_mode != m.reward_mode ||
      c.nstep != m.nstep || c.n_feats != m.n_feats || c.aux != m.aux)
    return fail(e, MGN_ERR_LENGTH, "state blob of a handle with other dimensions");
  // the blob carries its own source table: it must describe the same kinds
  // of source as the handle's (a replay blob into a generator handle, or the
  // reverse, would leave e->replay and the restored table disagreeing)
  if ((h.replay != 0) != e->replay)
    return fail(e, MGN_ERR_CONFIG, "state blob of a replay handle loaded into a generator handle, or the reverse");
  {
    const mgn_asset_source* bs = reinterpret_cast<const mgn_asset_source*>(
        static_cast<const char*>(src) + sizeof h + plan(&c).src);
    for (int i = 0; i < e->A; ++i) {
      int32_t k;
      std::memcpy(&k, &bs[i].kind, sizeof k);
      if (k != e->kinds[i] && k != MGN_SRC_EXTERNAL && e->kinds[i] != MGN_SRC_EXTERNAL)
        return fail(e, MGN_ERR_CONFIG, "state blob's source kind differs from the handle's for asset " +
                                           std::to_string(i));
    }
  }
  int rc = check_hip(e, hipMemcpyAsync(e->arena, (const char*)src + sizeof h, e->arena_bytes,
                                       hipMemcpyHostToDevice, e->stream), "mgn_load_state");
  if (rc == MGN_OK) rc = check_hip(e, hipStreamSynchronize(e->stream), "mgn_load_state (sync)");
  if (rc != MGN_OK) return rc;
  e->cfg = c;
  {
    const mgn_asset_source* bs = reinterpret_cast<const mgn_asset_source*>(
        static_cast<const char*>(src) + sizeof h + plan(&c).src);
    for (int i = 0; i < e->A; ++i) std::memcpy(&e->kinds[i], &bs[i].kind, sizeof(int32_t));
  }
  auto_layout(e);
  return MGN_OK;
}

int mgn_bandwidth_probe(void* dst_dev, const void* src_dev, size_t bytes, int32_t reps, void* stream,
                        double* gbps_out) {
  if (!dst_dev || !src_dev || !gbps_out) return fail(nullptr, MGN_ERR_ARG, "null probe buffers");
  if (bytes < 16 || bytes % 16 || reps < 1) return fail(nullptr, MGN_ERR_LENGTH, "bytes: multiple of 16; reps >= 1");
  hipStream_t st = (hipStream_t)stream;
  const int64_t n = (int64_t)(bytes / 16);
  const mgn::probe_v2* s = (const mgn::probe_v2*)src_dev;
  mgn::probe_v2* d = (mgn::probe_v2*)dst_dev;
  hipEvent_t a, b;
  if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess)
    return fail(nullptr, MGN_ERR_DEVICE, "event create");
  // the attainable rate: the best of six standard copy shapes (one 16- or
  // 32-KiB chunk per workgroup, or a grid-stride loop at 16 waves per CU;
  // plain or nontemporal stores), each warmed once and timed over `reps`
  // launches
  const unsigned g_one = (unsigned)((n + 4 * mgn::BLOCK - 1) / (4 * mgn::BLOCK));
  const unsigned g_one8 = (unsigned)((n + 8 * mgn::BLOCK - 1) / (8 * mgn::BLOCK));
  const unsigned g_loop = 256 * 16;
  double best = 0.;
  int rc = MGN_OK;
  for (int v = 0; v < 6 && rc == MGN_OK; ++v) {
    auto go = [&]() {
      switch (v) {
        case 0: hipLaunchKernelGGL((mgn::k_copy_probe<false, true, 4>), dim3(g_one), dim3(mgn::BLOCK), 0, st, s, d, n); break;
        case 1: hipLaunchKernelGGL((mgn::k_copy_probe<true, true, 4>), dim3(g_one), dim3(mgn::BLOCK), 0, st, s, d, n); break;
        case 2: hipLaunchKernelGGL((mgn::k_copy_probe<false, true, 8>), dim3(g_one8), dim3(mgn::BLOCK), 0, st, s, d, n); break;
        case 3: hipLaunchKernelGGL((mgn::k_copy_probe<true, true, 8>), dim3(g_one8), dim3(mgn::BLOCK), 0, st, s, d, n); break;
        case 4: hipLaunchKernelGGL((mgn::k_copy_probe<false, false>), dim3(g_loop), dim3(mgn::BLOCK), 0, st, s, d, n); break;
        default: hipLaunchKernelGGL((mgn::k_copy_probe<true, false>), dim3(g_loop), dim3(mgn::BLOCK), 0, st, s, d, n); break;
      }
    };
    go();  // warm
    (void)hipEventRecord(a, st);
    for (int r = 0; r < reps; ++r) go();
    (void)hipEventRecord(b, st);
    rc = check_hip(nullptr, hipEventSynchronize(b), "mgn_bandwidth_probe");
    float ms = 0.f;
    if (rc == MGN_OK) rc = check_hip(nullptr, hipEventElapsedTime(&ms, a, b), "mgn_bandwidth_probe");
    if (rc == MGN_OK && ms > 0.f) {
      const double gbps = 2.0 * (double)bytes * reps / (ms * 1e-3) / 1e9;
      if (gbps > best) best = gbps;
    }
  }
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  if (rc != MGN_OK) return rc;
  *gbps_out = best;
  return MGN_OK;
}

int mgn_synchronize(mgn_env* e) {
  if (!e) return MGN_ERR_ARG;
  return check_hip(e, hipStreamSynchronize(e->stream), "hipStreamSynchronize");
}

int mgn_synchronize_spin(mgn_env* e) {
  if (!e) return MGN_ERR_ARG;
  hipError_t st;
  while ((st = hipStreamQuery(e->stream)) == hipErrorNotReady) {
  }
  return check_hip(e, st, "hipStreamQuery");
}

const char* mgn_last_error(const mgn_env* e) { return e ? e->err.c_str() : g_error.c_str(); }
const char* mgn_global_error(void) { return g_error.c_str(); }

}  // extern "C"
