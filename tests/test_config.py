"""Config parsing mirrors madigan/environments/cpp/Config.cpp and the
DataSource constructors (keys, defaults, Composite, error types)."""
import pytest

from madigan_amd import _lib as L
from madigan_amd.config import ConfigError, build_config, default_spec, ou_spec, spec_from_config

SYNTH = {"data_source_type": "Synth",
         "data_source_config": {"freq": [1., 0.3], "mu": [2., 2.1], "amp": [1., 1.2],
                                "phase": [0., 1.], "dX": 0.01, "noise": 0.}}
OU = {"data_source_type": "OU", "data_source_config": {"mean": [10.] * 3, "theta": [.15] * 3,
                                                        "phi": [.04] * 3}}
TOU = {"data_source_type": "TrendOU",
       "data_source_config": {"trend_prob": [.001] * 3, "noise_trend": [.001] * 3,
                              "min_period": [100] * 3, "max_period": [500] * 3, "start": [5.] * 3,
                              "theta": [.15] * 3, "phi": [.04] * 3, "dYMin": [.001] * 3,
                              "dYMax": [.005] * 3, "ema_alpha": [.99] * 3}}


def test_synth_ou_trendou_keys():
    s = spec_from_config(SYNTH)
    assert s.kinds == [L.SRC_SINE] * 2 and s.assets == ["sine_0", "sine_1"]
    assert s.params[1] == [0.3, 2.1, 1.2, 1.0, 0.01, 0.0]
    o = spec_from_config(OU)
    assert o.kinds == [L.SRC_OU] * 3 and o.params[0] == [10., .15, .04]
    t = spec_from_config(TOU)
    assert t.kinds == [L.SRC_TRENDOU] * 3
    assert t.params[0] == [.001, 100., 500., .001, .005, 5., .15, .04, .001, .99]


def test_missing_key_is_config_error():
    bad = {"data_source_type": "Synth", "data_source_config": dict(SYNTH["data_source_config"])}
    del bad["data_source_config"]["noise"]  # Config.cpp:166-176 requires all six keys
    with pytest.raises(RuntimeError, match="noise key not found"):
        spec_from_config(bad)
    with pytest.raises(ConfigError):
        spec_from_config({"data_source_config": {}})


def test_length_mismatch_is_value_error():
    bad = {"data_source_type": "OU", "data_source_config": {"mean": [1., 2.], "theta": [.1],
                                                             "phi": [.1, .2]}}
    with pytest.raises(ValueError, match="same length"):
        spec_from_config(bad)


def test_composite_order_one_child_per_type_and_renames():
    comp = {"data_source_type": "Composite",
            "data_source_config": {"a": SYNTH, "b": OU, "c": TOU,
                                   "d": {"data_source_type": "OU", "data_source_config": {
                                       "mean": [1.], "theta": [.1], "phi": [.2]}}}}
    s = spec_from_config(comp)
    # one child per type (Config.cpp:121): the later OU config replaces the first
    assert s.kinds == [L.SRC_SINE] * 2 + [L.SRC_OU] + [L.SRC_TRENDOU] * 3
    assert s.params[2] == [1., .1, .2]
    dup = {"data_source_type": "Composite",
           "data_source_config": {"a": OU, "b": {"data_source_type": "Synth",
                                                 "data_source_config": SYNTH["data_source_config"]}}}
    assert spec_from_config(dup).assets == ["OU_0", "OU_1", "OU_2", "sine_0", "sine_1"]


def test_defaults_match_reference_default_constructors():
    s = default_spec("Synth")  # DataSource.cpp:475-482
    assert [p[0] for p in s.params] == [1., 0.3, 2., 0.5]
    o = default_spec("OU")     # DataSource.cpp:1142
    assert [p[0] for p in o.params] == [2., 4.3, 3., 0.5]
    t = default_spec("TrendOU")  # DataSource.cpp:1418-1423
    assert [p[5] for p in t.params] == [10., 15.]


def test_unsupported_sources_raise_runtime_error():
    with pytest.raises(RuntimeError, match="nyquist"):  # default ctor passes dX = 0 (DataSource.cpp:686)
        default_spec("SineDynamic")
    with pytest.raises(RuntimeError, match="not implemented"):
        spec_from_config({"data_source_type": "Bogus", "data_source_config": {}})


def test_build_config_fields():
    c, srcs = build_config(spec_from_config(OU), n_envs=16, reward_shaper="DDR",
                           reward_mode="agent_per_asset", window=8, norm_type="log", seed=3)
    assert (c.n_envs, c.n_assets, c.shaper, c.reward_mode, c.window, c.norm_type) == \
        (16, 3, L.SHAPER_DDR, L.REWARD_AGENT_PER_ASSET, 8, L.NORM_LOG)
    assert list(c.desired_portfolio)[:4] == [1., 0., 0., 0.]
    assert srcs[2].kind == L.SRC_OU
    with pytest.raises(NotImplementedError):
        build_config(spec_from_config(OU), n_envs=1, reward_shaper="nope")
    with pytest.raises(ValueError):
        build_config(spec_from_config(OU), n_envs=1, desired_portfolio=[1., 0.])


def test_make_preprocessor_dispatch_like_reference():
    """make_preprocessor (preprocessor.py:28-50): StackerDiscreteReturns maps to
    plain StackerDiscrete; Pairs / Multi dispatch by substring test."""
    from madigan_amd import (MultiStackerDiscrete, StackerDiscrete, StackerDiscretePairs,
                             make_preprocessor)
    base = {"window_length": 8, "norm": True, "norm_type": "lookback"}
    mk = lambda t, **kw: make_preprocessor({"preprocessor_type": t,
                                            "preprocessor_config": {**base, **kw}}, 2)
    assert type(mk("StackerDiscreteReturns")) is StackerDiscrete
    assert type(mk("WindowedStacker")) is StackerDiscrete
    assert type(mk("StackerDiscretePairs")) is StackerDiscretePairs
    m = mk("MultiStackerDiscrete", dilations=[1, 4])
    assert type(m) is MultiStackerDiscrete and m.feature_output_shape == (8, 4)
    assert mk("StackerDiscretePairs").feature_output_shape == (8, 1)
    with pytest.raises(NotImplementedError):
        mk("RollerDiscrete")
    with pytest.raises(NotImplementedError):
        mk("StackerDiscrete", norm_type="bogus")
    mk("StackerDiscrete", norm_type="expanding")  # builds; current_data raises TypeError
    mk("StackerDiscrete", norm_type="log_standard_normal")


def test_naive_shaper_config():
    from madigan_amd.config import build_config, shaper_code
    from madigan_amd import _lib as L
    assert shaper_code("sharpe_shaper") == L.SHAPER_SHARPE
    assert shaper_code("sortino_shaperB") == L.SHAPER_SORTINO_B
    assert shaper_code("sum_default") == L.SHAPER_NONE
    spec = ou_spec([1.0], [0.1], [0.1])
    with pytest.raises(KeyError):
        build_config(spec, n_envs=2, reward_shaper="sortino_shaperA")
    c, _ = build_config(spec, n_envs=2, reward_shaper="sortino_shaperA", sortino_exp=3)
    assert c.sortino_exp == 3.0 and c.shaper == L.SHAPER_SORTINO_A


def test_build_caps_raise_runtime_error():
    """This build's fixed caps (include/madigan_amd.h MGN_MAX_ASSETS = 64,
    MGN_MAX_NSTEP = 256; the reference's Eigen vectors and NStepBuffer are
    unbounded, DataTypes.h:28-29, nstep_buffer.py:315-330) are refused as the
    reference refuses an unsupported config: ConfigError, a RuntimeError
    (DataTypes.h:36-46), before any device call."""
    wide = ou_spec([10.] * (L.MAX_ASSETS + 1), [.15] * (L.MAX_ASSETS + 1), [.04] * (L.MAX_ASSETS + 1))
    with pytest.raises(RuntimeError, match="MGN_MAX_ASSETS"):
        build_config(wide, n_envs=4)
    full = ou_spec([10.] * L.MAX_ASSETS, [.15] * L.MAX_ASSETS, [.04] * L.MAX_ASSETS)
    assert build_config(full, n_envs=4)[0].n_assets == L.MAX_ASSETS
    with pytest.raises(RuntimeError, match="MGN_MAX_NSTEP"):
        build_config(spec_from_config(OU), n_envs=4, reward_shaper="DDR", nstep_return=L.MAX_NSTEP + 1)
    assert build_config(spec_from_config(OU), n_envs=4, reward_shaper="DDR",
                        nstep_return=L.MAX_NSTEP)[0].nstep == L.MAX_NSTEP
