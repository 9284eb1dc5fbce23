"""Reference config dict -> per-asset generator table and env knobs.

Mirrors the reference's config handling for the data sources on the hot path:
  makeConfigFromPyDict               madigan/environments/cpp/Config.cpp:5-164
  Synth keys  (freq mu amp phase dX noise)             Config.cpp:166-214
  OU keys     (mean theta phi)                         Config.cpp:353-386
  TrendOU keys(trend_prob min_period max_period dYMin dYMax start theta phi
               noise_trend ema_alpha)                   Config.cpp:479-549
  Composite   {name: {data_source_type, data_source_config}} Config.cpp:107-126,
              children concatenated, one per type, duplicate asset codes
              renamed code+"_1"                         DataSource.cpp:411-437
  default constructors Synth()/OU()/TrendOU()          DataSource.cpp:475-482, :1142,
                                                       :1418-1423
  SimpleTrend keys (trend_prob min_period max_period noise dYMin dYMax start)
                                                       Config.cpp:422-476
  TrendyOU    keys as TrendOU                          Config.cpp:127-139, :479-549
  OUPair      keys (theta phi noise)                   Config.cpp:387-419
  SawTooth / Triangle keys as Synth                    Config.cpp:15-28
  Gaussian    from config always raises: its key check asks for "" (Config.cpp:324),
              reproduced; the default constructor works
  HDFSourceSingle keys (filepath group_key price_key feature_key timestamp_key
              cache_size [start_time end_time])        Config.cpp:551-576,
                                                       DataSource.cpp:227-262
  SineAdder   keys as Synth (one asset: the sum)        Config.cpp:15-28, DataSource.cpp:582-661
  SineDynamic keys (freqRange muRange ampRange dX noise) Config.cpp:216-259,
                                                       DataSource.cpp:678-792
  SineDynamicTrend + (trendRange trendIncr trendProb)  Config.cpp:261-318,
                                                       DataSource.cpp:850-992
Errors follow the reference: missing keys -> RuntimeError (ConfigError),
mismatched vector lengths -> ValueError (std::length_error), unknown source
type -> RuntimeError (NotImplemented).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, List, Optional, Tuple

from . import _lib as L

SUPPORTED = ("Synth", "OU", "TrendOU", "Composite", "HDFSourceSingle", "SimpleTrend", "TrendyOU",
             "Gaussian", "SawTooth", "Triangle", "OUPair", "SineAdder", "SineDynamic",
             "SineDynamicTrend")
NOT_YET = ()
AUX_KINDS = (L.SRC_SINEADDER, L.SRC_SINEDYNAMIC, L.SRC_SINEDYNTREND)
HDF_KEYS = ("filepath", "group_key", "feature_key", "timestamp_key", "price_key", "cache_size")


class ConfigError(RuntimeError):
    """madigan::ConfigError (DataTypes.h:36-40) surfaces as RuntimeError."""


@dataclass
class SourceSpec:
    kinds: List[int] = field(default_factory=list)
    params: List[List[float]] = field(default_factory=list)
    assets: List[str] = field(default_factory=list)
    n_feats: int = 0                 # State.price width; 0 = n_assets (generators)
    hdf: Optional[dict] = None       # HDFSourceSingle data_source_config (replay)

    @property
    def n_assets(self) -> int:
        return len(self.kinds)

    @property
    def replay(self) -> bool:
        return bool(self.kinds) and self.kinds[0] == L.SRC_REPLAY

    def extend(self, other: "SourceSpec") -> None:
        if other.replay or self.replay:
            raise RuntimeError("HDFSourceSingle cannot be a Composite child (Config.cpp:107-126)")
        for k, p, a in zip(other.kinds, other.params, other.assets):
            self.kinds.append(k)
            self.params.append(p)
            # Composite renames duplicate codes (DataSource.cpp:428-431)
            self.assets.append(a + "_1" if a in self.assets else a)


def _get(cfg: Any, key: str, default=None):
    if isinstance(cfg, dict):
        return cfg.get(key, default)
    return getattr(cfg, key, default)


def _require(params: dict, keys: Tuple[str, ...]) -> None:
    for k in keys:
        if k not in params:
            raise ConfigError(f"{k} key not found in data_source_config in config")


def _same_len(name: str, *vecs) -> int:
    n = len(vecs[0])
    if any(len(v) != n for v in vecs):
        raise ValueError(f"parameters passed to DataSource<PriceVector> of type {name} need to be "
                         "vectors of same length")
    return n


def synth_spec(freq, mu, amp, phase, dX, noise=0.0, kind: int = L.SRC_SINE,
               name: str = "Synth") -> SourceSpec:
    """Synth (and its SawTooth / Triangle subclasses, DataSource.h:413-423)."""
    n = _same_len(name, freq, mu, amp, phase)
    s = SourceSpec()
    for i in range(n):
        s.kinds.append(kind)
        s.params.append([float(freq[i]), float(mu[i]), float(amp[i]), float(phase[i]), float(dX),
                         float(noise)])
        s.assets.append(f"sine_{i}")
    return s


def ou_spec(mean, theta, phi) -> SourceSpec:
    n = _same_len("OU", mean, theta, phi)
    s = SourceSpec()
    for i in range(n):
        s.kinds.append(L.SRC_OU)
        s.params.append([float(mean[i]), float(theta[i]), float(phi[i])])
        s.assets.append(f"OU_{i}")
    return s


def trendou_spec(trendProb, minPeriod, maxPeriod, dYMin, dYMax, start, theta, phi, noiseTrend,
                 emaAlpha) -> SourceSpec:
    n = _same_len("TrendOU", trendProb, minPeriod, maxPeriod, dYMin, dYMax, start, theta, phi,
                  noiseTrend, emaAlpha)
    s = SourceSpec()
    for i in range(n):
        s.kinds.append(L.SRC_TRENDOU)
        s.params.append([float(trendProb[i]), float(int(minPeriod[i])), float(int(maxPeriod[i])),
                         float(dYMin[i]), float(dYMax[i]), float(start[i]), float(theta[i]),
                         float(phi[i]), float(noiseTrend[i]), float(emaAlpha[i])])
        s.assets.append(f"TrendOU_{i}")
    return s


def simpletrend_spec(trendProb, minPeriod, maxPeriod, noise, start, dYMin, dYMax) -> SourceSpec:
    """SimpleTrend::initParams (DataSource.cpp:1252-1283)."""
    n = _same_len("SimpleTrend", trendProb, minPeriod, maxPeriod, noise, start, dYMin, dYMax)
    s = SourceSpec()
    for i in range(n):
        s.kinds.append(L.SRC_SIMPLETREND)
        s.params.append([float(trendProb[i]), float(int(minPeriod[i])), float(int(maxPeriod[i])),
                         float(noise[i]), float(start[i]), float(dYMin[i]), float(dYMax[i])])
        s.assets.append(f"SimpleTrend_{i}")
    return s


def trendyou_spec(trendProb, minPeriod, maxPeriod, dYMin, dYMax, start, theta, phi, noiseTrend,
                  emaAlpha) -> SourceSpec:
    """TrendyOU::initParams (DataSource.cpp:1506-1552): TrendOU's parameters."""
    s = trendou_spec(trendProb, minPeriod, maxPeriod, dYMin, dYMax, start, theta, phi, noiseTrend,
                     emaAlpha)
    s.kinds = [L.SRC_TRENDYOU] * s.n_assets
    s.assets = [f"TrendyOU_{i}" for i in range(s.n_assets)]
    return s


def gaussian_spec(mean, var) -> SourceSpec:
    """Gaussian::initParams (DataSource.cpp:1057-1075): normal(mean, var)."""
    n = _same_len("Gaussian", mean, var)
    return SourceSpec(kinds=[L.SRC_GAUSSIAN] * n, params=[[float(m), float(v)] for m, v in zip(mean, var)],
                      assets=[f"Gaussian_{i}" for i in range(n)])


def oupair_spec(theta, phi, noise) -> SourceSpec:
    """OUPair::initParams (DataSource.cpp:1183-1196): two assets, one shared mean."""
    p = [float(theta), float(phi), float(noise)]
    return SourceSpec(kinds=[L.SRC_OUPAIR] * 2, params=[p + [0.0], p + [1.0]],
                      assets=["OUPair_0", "OUPair_1"])


def sineadder_spec(freq, mu, amp, phase, dX, noise=0.0) -> SourceSpec:
    """SineAdder::initParams (DataSource.cpp:591-661): one asset, "multi_sine",
    the sum of the components; x starts at phase."""
    n = _same_len("SineAdder", freq, mu, amp, phase)
    if not 1 <= n <= 8:
        raise ValueError(f"SineAdder supports 1..8 components on the MI355X path, got {n}")
    p = [float(n), float(dX), float(noise)]
    for v in (freq, mu, amp, phase):
        p += [float(x) for x in v]
    return SourceSpec(kinds=[L.SRC_SINEADDER], params=[p], assets=["multi_sine"])


def _wave_table_len(sample_rate: int, base_freq: float) -> int:
    """setSineOsc's table length (WaveTableOsc.h:129-146): the harmonic count
    sampleRate / (3 baseFreq) + 0.5 (int), rounded up to a power of two by the
    bit trick (unsigned 32-bit), times 2 * overSample (= 2)."""
    max_harms = int(sample_rate / (3.0 * base_freq) + 0.5)
    v = (max_harms - 1) & 0xFFFFFFFF
    for sh in (1, 2, 4, 8, 16):
        v |= v >> sh
    v = (v + 1) & 0xFFFFFFFF
    return v * 2 * 2


def _sine_dynamic_params(name, freqRange, muRange, ampRange, dX, noise):
    """SineDynamic(Trend)::initParams (DataSource.cpp:742-792, :925-983)."""
    if not (len(freqRange) == len(muRange) == len(ampRange)):
        raise ValueError(f"parameters passed to DataSource<PriceVector> of type {name} need to be "
                         "vectors of same length")
    C = len(freqRange)
    if not 1 <= C <= 4:
        raise ValueError(f"{name} supports 1..4 components on the MI355X path, got {C}")
    with_dx = float(dX)
    sample_rate = int(1.0 / with_dx) if with_dx != 0 else None
    rows = [[float(x) for x in r] for r in (list(freqRange) + list(muRange) + list(ampRange))]
    if any(len(r) != 3 for r in rows):
        raise ValueError("freqRange / muRange / ampRange entries are [low, high, step]")
    for i in range(C):
        # sampleRate = (int)(1 / dX) must be at least the Nyquist rate (:763-776);
        # a dX of 0 (the default constructors pass the unset member) fails the same test
        if sample_rate is None or float(freqRange[i][1]) * 2 > sample_rate:
            raise RuntimeError("Sampling Rate as determined by 1 / dX must be at least the nyquist "
                               f"sampling rate relative to the largest frequency. freqRange entry #{i}")
    p = [float(C), float(sample_rate), float(noise)]
    p += [float(_wave_table_len(sample_rate, float(freqRange[i][0]))) for i in range(C)]
    for i in range(C):
        p += [float(x) for x in freqRange[i]] + [float(x) for x in muRange[i]] + \
             [float(x) for x in ampRange[i]]
    return p


def sinedynamic_spec(freqRange, muRange, ampRange, dX, noise=0.0) -> SourceSpec:
    p = _sine_dynamic_params("SineDynamic", freqRange, muRange, ampRange, dX, noise)
    return SourceSpec(kinds=[L.SRC_SINEDYNAMIC], params=[p], assets=["sine_dynamic"])


def sinedynamictrend_spec(freqRange, muRange, ampRange, trendRange, trendIncr, trendProb, dX,
                          noise=0.0) -> SourceSpec:
    if not (len(trendRange) == len(trendIncr) == len(trendProb)):
        raise ValueError("the following parameters passed to DataSource<PriceVector>of type "
                         "SineDynamicTrend need to be vectors of same length:trendRange\n "
                         "trendIncr\n trendProb\n")
    p = _sine_dynamic_params("SineDynamicTrend", freqRange, muRange, ampRange, dX, noise)
    T = len(trendRange)
    if T > 2:
        raise ValueError(f"SineDynamicTrend supports at most 2 trends on the MI355X path, got {T}")
    p.append(float(T))
    for t in range(T):
        p += [float(int(trendRange[t][0])), float(int(trendRange[t][1])), float(trendIncr[t]),
              float(trendProb[t])]
    return SourceSpec(kinds=[L.SRC_SINEDYNTREND], params=[p], assets=["sine_dynamic_trend"])


def replay_spec(n_assets: int, n_feats: int = 0, assets=None, hdf: Optional[dict] = None) -> SourceSpec:
    """Every asset from a replay tape (HDFSourceSingle, or a tape given directly)."""
    codes = list(assets) if assets is not None else [f"asset_{i}" for i in range(n_assets)]
    return SourceSpec(kinds=[L.SRC_REPLAY] * n_assets, params=[[] for _ in range(n_assets)],
                      assets=codes, n_feats=int(n_feats) or n_assets, hdf=hdf)


def hdf_spec(params: dict) -> SourceSpec:
    """HDFSourceSingle(Config) (DataSource.cpp:227-262): required keys, then
    init() on the file (checkKeys, assets, dims, time bounds)."""
    missing = [k for k in HDF_KEYS if k not in params]
    if missing:
        raise ConfigError("Missing keys in call to HDFSourceSingle: \n" + ", ".join(missing) + ", \n")
    from .hdf import HDFFile
    start, end = 0, 0
    if "start_time" in params and "end_time" in params:
        start, end = int(params["start_time"]), int(params["end_time"])
    f = HDFFile(params["filepath"], params["group_key"], params["price_key"],
                params["feature_key"], params["timestamp_key"], start, end)
    cfg = dict(params)
    cfg["start_time"], cfg["end_time"] = int(f.info.start_time), int(f.info.end_time)
    return replay_spec(f.n_assets, f.n_feats, f.asset_codes, hdf=cfg)


def default_spec(source_type: str) -> SourceSpec:
    """Default constructors (Env(type, initCash) without config)."""
    if source_type == "Synth":
        return synth_spec([1., 0.3, 2., 0.5], [2., 2.1, 2.2, 2.3], [1., 1.2, 1.3, 1.],
                          [0., 1., 2., 1.], 0.01, 0.)
    if source_type == "OU":
        return ou_spec([2., 4.3, 3., 0.5], [1., 0.3, 2., 0.5], [2., 2.1, 2.2, 2.3])
    if source_type in ("TrendOU", "TrendyOU"):
        f = trendou_spec if source_type == "TrendOU" else trendyou_spec
        return f([0.001, 0.001], [100, 500], [200, 1500], [0.001, 0.01], [0.003, 0.03],
                 [10., 15.], [1., 0.5], [2., 2.1], [1., 1.2], [0.1, 0.2])
    if source_type in ("SawTooth", "Triangle"):  # Synth() (DataSource.cpp:475-482)
        kind = L.SRC_SAWTOOTH if source_type == "SawTooth" else L.SRC_TRIANGLE
        return synth_spec([1., 0.3, 2., 0.5], [2., 2.1, 2.2, 2.3], [1., 1.2, 1.3, 1.],
                          [0., 1., 2., 1.], 0.01, 0., kind=kind, name=source_type)
    if source_type == "SimpleTrend":  # DataSource.cpp:1291-1293
        return simpletrend_spec([0.001, 0.001], [100, 500], [200, 1500], [1., 0.1], [10., 15.],
                                [0.001, 0.01], [0.003, 0.03])
    if source_type == "Gaussian":     # DataSource.cpp:1079
        return gaussian_spec([2., 5., 10., 15.], [1., 1., 2., 5.])
    if source_type == "OUPair":       # DataSource.cpp:1201
        return oupair_spec(.015, .01, .03)
    if source_type == "SineAdder":    # DataSource.cpp:582-589 (dX member default .01)
        return sineadder_spec([1., 0.3, 2., 0.5], [2., 2.1, 2.2, 2.3], [1., 1.2, 1.3, 1.],
                              [0., 1., 2., 1.], 0.01, 0.)
    if source_type == "SineDynamic":  # DataSource.cpp:678-687: passes the unset member dX (0)
        return sinedynamic_spec(_SD_FREQ, _SD_MU, _SD_AMP, 0.0, 1.)
    if source_type == "SineDynamicTrend":  # DataSource.cpp:850-862: same
        return sinedynamictrend_spec(_SD_FREQ, _SD_MU, _SD_AMP, [[100, 500], [100, 300]],
                                     [0.1, 0.2], [.001, .01], 0.0, 1.)
    return _not_implemented(source_type)


_SD_FREQ = [[.1, 1., .01], [0.3, 3.0, .01], [5., 15., .1], [10., 50., .1]]
_SD_MU = [[1., 5., .02], [.3, 3., .05], [.2, 5., .02], [.5, 5., .02]]
_SD_AMP = [[1., 5., .01], [.3, 3., .02], [.2, 2., .04], [.5, 5., .05]]


def _not_implemented(source_type: str):
    if source_type in NOT_YET:
        raise RuntimeError(f"Constructor from config for {source_type} as dataSource is not "
                           "implemented on the MI355X path yet (SURVEY 8f)")
    raise RuntimeError(f"Constructor from config for{source_type} as dataSource is not implemented")


def spec_from_config(config: Any) -> SourceSpec:
    """makeConfigFromPyDict + makeDataSource<PriceVector>(type, config)."""
    source_type = _get(config, "data_source_type")
    if source_type is None:
        raise ConfigError("Config needs entry for data_source_type")
    params = _get(config, "data_source_config")
    if source_type == "Composite":
        if params is None:
            raise ConfigError("config passed but doesn't contain generator params")
        children = {}
        for _, sub in dict(params).items():
            ctype = _get(sub, "data_source_type")
            children[ctype] = sub  # keyed by type: one child per type (Config.cpp:121)
        spec = SourceSpec()
        for ctype, sub in children.items():
            spec.extend(spec_from_config(sub))
        return spec
    if params is None:
        raise ConfigError(f"config for DataSource type {source_type} needs generator params")
    params = dict(params)
    if source_type == "Synth":
        _require(params, ("freq", "mu", "amp", "phase", "dX", "noise"))
        return synth_spec(params["freq"], params["mu"], params["amp"], params["phase"],
                          params["dX"], params["noise"])
    if source_type == "OU":
        _require(params, ("mean", "theta", "phi"))
        return ou_spec(params["mean"], params["theta"], params["phi"])
    if source_type == "HDFSourceSingle":
        return hdf_spec(params)
    if source_type in ("SawTooth", "Triangle"):
        _require(params, ("freq", "mu", "amp", "phase", "dX", "noise"))
        kind = L.SRC_SAWTOOTH if source_type == "SawTooth" else L.SRC_TRIANGLE
        return synth_spec(params["freq"], params["mu"], params["amp"], params["phase"],
                          params["dX"], params["noise"], kind=kind, name=source_type)
    if source_type == "SimpleTrend":
        _require(params, ("trend_prob", "min_period", "max_period", "noise", "dYMin", "dYMax",
                          "start"))
        return simpletrend_spec(params["trend_prob"], params["min_period"], params["max_period"],
                                params["noise"], params["start"], params["dYMin"], params["dYMax"])
    if source_type == "Gaussian":
        # makeGaussianConfigFromPyDict checks for the keys {"mean", ""} (Config.cpp:324):
        # the empty key is never present, so the reference always raises here
        _require(params, ("mean", ""))
    if source_type == "OUPair":
        _require(params, ("theta", "phi", "noise"))
        return oupair_spec(params["theta"], params["phi"], params["noise"])
    if source_type == "SineAdder":  # makeSynthConfigFromPyDict (Config.cpp:166-214)
        _require(params, ("freq", "mu", "amp", "phase", "dX", "noise"))
        return sineadder_spec(params["freq"], params["mu"], params["amp"], params["phase"],
                              params["dX"], params["noise"])
    if source_type == "SineDynamic":  # Config.cpp:216-259
        _require(params, ("freqRange", "muRange", "ampRange", "dX", "noise"))
        return sinedynamic_spec(params["freqRange"], params["muRange"], params["ampRange"],
                                params["dX"], params["noise"])
    if source_type == "SineDynamicTrend":  # Config.cpp:261-318
        _require(params, ("freqRange", "muRange", "ampRange", "trendRange", "trendProb",
                          "trendIncr", "dX", "noise"))
        return sinedynamictrend_spec(params["freqRange"], params["muRange"], params["ampRange"],
                                     params["trendRange"], params["trendIncr"],
                                     params["trendProb"], params["dX"], params["noise"])
    if source_type in ("TrendOU", "TrendyOU"):
        _require(params, ("trend_prob", "min_period", "max_period", "dYMin", "dYMax", "start",
                          "theta", "phi", "noise_trend", "ema_alpha"))
        f = trendou_spec if source_type == "TrendOU" else trendyou_spec
        return f(params["trend_prob"], params["min_period"], params["max_period"],
                            params["dYMin"], params["dYMax"], params["start"], params["theta"],
                            params["phi"], params["noise_trend"], params["ema_alpha"])
    return _not_implemented(source_type)


# NStepBuffer.make_reward_shaper (nstep_buffer.py:378-408): cosine aliases, the
# sortino pair, DSR / DDR, any module-level shaper function by name
# (sum_default, sharpe_shaper), and None
SHAPER_CODES = {None: L.SHAPER_NONE, "None": L.SHAPER_NONE, "none": L.SHAPER_NONE,
                "sum_default": L.SHAPER_NONE,
                "DSR": L.SHAPER_DSR, "DDR": L.SHAPER_DDR, "PPC": L.SHAPER_PPC, "cosine": L.SHAPER_PPC,
                "cosine_similarity": L.SHAPER_PPC, "cosine_port_shaper": L.SHAPER_PPC,
                "sharpe_shaper": L.SHAPER_SHARPE, "sortino_shaperA": L.SHAPER_SORTINO_A,
                "sortino_shaperB": L.SHAPER_SORTINO_B}
REWARD_MODES = {"env_log": L.REWARD_ENV_LOG, "agent_sum": L.REWARD_AGENT_SUM,
                "agent_per_asset": L.REWARD_AGENT_PER_ASSET}
NORM_CODES = {None: L.NORM_NONE, "none": L.NORM_NONE, "log": L.NORM_LOG,
              "lookback": L.NORM_LOOKBACK, "standard_normal": L.NORM_STANDARD_NORMAL,
              "lookback_log": L.NORM_LOOKBACK_LOG, "log_standard_normal": L.NORM_LOG_STANDARD_NORMAL}


def shaper_code(name) -> int:
    if name not in SHAPER_CODES:
        raise NotImplementedError(f"Reward Shaper type {name} not implemented")
    return SHAPER_CODES[name]


def norm_code(name) -> int:
    if name not in NORM_CODES:
        raise NotImplementedError(
            f"norm_type {name} is not implemented. choose from : 'lookback', 'lookback_log', "
            "'standard_normal', 'log'")
    return NORM_CODES[name]


NSTEP_POPS = {"exact": L.NSTEP_POP_EXACT, "running": L.NSTEP_POP_RUNNING}


def build_config(spec: SourceSpec, *, n_envs: int, init_cash: float = 1_000_000.0,
                 required_margin: float = 0.0, maintenance_margin: float = 0.0,
                 slippage_rel: float = 0.0, slippage_abs: float = 0.0,
                 transaction_cost_rel: float = 0.0, transaction_cost_abs: float = 0.0,
                 reward_shaper=None, reward_mode: str = "env_log", adaptation_rate: float = 0.001,
                 cosine_temp: float = 0.0, desired_portfolio=None, window: int = 0,
                 norm_type=None, auto_reset: bool = False, action_atoms: int = 3,
                 unit_size: float = 0.05, seed: int = 0, env_offset: int = 0,
                 nstep_return: int = 1, discount: float = 0.99, sortino_exp=None,
                 nstep_pop: str = "exact"):
    A = spec.n_assets
    if A < 1:
        raise ValueError(f"n_assets must be >= 1, got {A}")
    if A > L.MAX_ASSETS:
        # a limit of this build (the reference's Eigen vectors are dynamic):
        # raised as the reference raises an unsupported config (ConfigError ->
        # RuntimeError, DataTypes.h:36-46)
        raise ConfigError(f"n_assets must be in [1, {L.MAX_ASSETS}] (MGN_MAX_ASSETS), got {A}")
    c = L.Config()
    c.n_envs = int(n_envs)
    c.n_assets = A
    c.env_offset = int(env_offset)
    c.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    c.init_cash = float(init_cash)
    c.required_margin = float(required_margin)
    c.maintenance_margin = float(maintenance_margin)
    c.slippage_rel, c.slippage_abs = float(slippage_rel), float(slippage_abs)
    c.tc_rel, c.tc_abs = float(transaction_cost_rel), float(transaction_cost_abs)
    c.shaper = shaper_code(reward_shaper)
    if reward_mode not in REWARD_MODES:
        raise ConfigError(f"unknown reward_mode {reward_mode}")
    c.reward_mode = REWARD_MODES[reward_mode]
    c.adaptation_rate = float(adaptation_rate)
    c.cosine_temp = float(cosine_temp)
    dp = list(desired_portfolio) if desired_portfolio is not None else [1.0] + [0.0] * A
    if len(dp) != A + 1:
        raise ValueError(f"desired_portfolio needs {A + 1} entries (cash + assets), got {len(dp)}")
    for i, v in enumerate(dp):
        c.desired_portfolio[i] = float(v)
    c.window = int(window)
    c.norm_type = norm_code(norm_type)
    c.auto_reset = 1 if auto_reset else 0
    c.action_atoms = int(action_atoms)
    c.unit_size = float(unit_size)
    if not 1 <= int(nstep_return) <= L.MAX_NSTEP:
        raise ConfigError(f"nstep_return must be in [1, {L.MAX_NSTEP}] (MGN_MAX_NSTEP), got {nstep_return}")
    c.nstep = int(nstep_return)  # config.py:126 (Agent/Model spec)
    c.discount = float(discount)  # config.py:154
    # how an n-step pop is evaluated (include/madigan_amd.h MGN_NSTEP_POP_*):
    # "exact" re-evaluates the buffer's summands as nstep_buffer.py does;
    # "running" forms DSR / DDR / PPC / none pops from discounted running sums
    # (O(1) per pop, within 1e-6 of the exact pop) where the kernel has them
    if nstep_pop not in NSTEP_POPS:
        raise ConfigError(f"nstep_pop must be one of {sorted(NSTEP_POPS)}, got {nstep_pop!r}")
    c.nstep_pop = NSTEP_POPS[nstep_pop]
    c.n_feats = int(spec.n_feats) if spec.replay else 0
    if c.shaper in (L.SHAPER_SORTINO_A, L.SHAPER_SORTINO_B):
        if sortino_exp is None:  # shaper_config["sortino_exp"] (nstep_buffer.py:392)
            raise KeyError("sortino_exp")
        if not float(sortino_exp) > 0:
            raise ConfigError(f"sortino_exp must be > 0, got {sortino_exp}")
    c.sortino_exp = float(sortino_exp) if sortino_exp is not None else 2.0
    c.aux = 1 if any(k in AUX_KINDS for k in spec.kinds) else 0
    srcs = (L.AssetSource * A)()
    for i, (k, p) in enumerate(zip(spec.kinds, spec.params)):
        srcs[i].kind = k
        for j, v in enumerate(p):
            srcs[i].p[j] = v
    return c, srcs
