"""SURVEY 8f #4 generators in the oracle: SimpleTrend, TrendyOU, Gaussian,
SawTooth, Triangle, OUPair.  Like the other generators their draws cannot be
replayed against the reference (wall-clock seeded std::default_random_engine,
DataSource.cpp:1283, :1552, :1071, :1195): parity with the reference is the
deterministic formulas (noise 0) and the statistics each getData implies;
bitwise parity oracle <-> HIP is in tests/test_gpu_generators.py."""
import math

import numpy as np
import pytest

from oracle import oracle as O
from tests.configs import (gaussian_sources, oupair_sources, simpletrend_sources, trendyou_sources,
                           wave_sources)


def run(sources, N, T, **cfg):
    orc = O.OracleBatch(dict(n_envs=N, seed=cfg.pop("seed", 3), **cfg), sources)
    prices = [orc.field(O.F_PRICE)]
    for _ in range(T):
        prices.append(orc.step()["obs_price"])
    return orc, np.array(prices)


def test_fdlibm_asin_vs_libm():
    L = O.lib()
    rng = np.random.default_rng(2)
    xs = np.concatenate([rng.uniform(-1, 1, 20000), [-1.0, 1.0, 0.0, -0.0, 0.5, -0.5, 0.975, 1e-9]])
    for x in xs:
        assert abs(L.orc_asin(x) - math.asin(x)) <= np.spacing(abs(math.asin(x)))
    assert math.isnan(L.orc_asin(1.5))


def test_sawtooth_triangle_formulas():
    """noise 0: SawTooth mu + amp*modf(x*freq), Triangle mu + 4amp/PI2 *
    asin(sin(PI2*x/freq)), x += dX after each tick (DataSource.cpp:557-577)."""
    freq, mu, amp, ph = [1., 0.3, 2.], [2., -2.1, 2.2], [1., 1.2, 1.3], [0., 1., -2.]
    for kind in (O.SRC_SAWTOOTH, O.SRC_TRIANGLE):
        orc, P = run(wave_sources(kind, freq, mu, amp, ph, 0.013), 2, 400)
        PI2 = 3.141592653589793238463 * 2
        x = np.array(ph, dtype=float)
        for t in range(401):
            for i in range(3):
                if kind == O.SRC_SAWTOOTH:
                    want = 0.0 + mu[i] + amp[i] * math.modf(x[i] * freq[i])[0]
                    assert P[t, 0, i] == want
                else:
                    want = 0.0 + mu[i] + 4 * amp[i] / PI2 * math.asin(math.sin(PI2 * x[i] / freq[i]))
                    assert abs(P[t, 1, i] - want) <= 4e-16 * max(1.0, abs(want))
            x += 0.013


def test_gaussian_moments():
    orc, P = run(gaussian_sources([2., 50.], [1., 5.]), 400, 250)
    v = P[1:].reshape(-1, 2)
    assert abs(v[:, 0].mean() - 2) < 0.02 and abs(v[:, 0].std() - 1) < 0.02
    assert abs(v[:, 1].mean() - 50) < 0.1 and abs(v[:, 1].std() - 5) < 0.1


def test_oupair_shared_mean_and_reversion():
    """mean += mean*N(0, noise); x_i += theta(mean - x_i) + mean*N(0, phi)
    (DataSource.cpp:1236-1244): both assets track one mean; the spread has the
    OU stationary variance 2 (mean phi)^2 / (1 - (1-theta)^2) near mean 10."""
    theta, phi = 0.2, 0.002
    orc, P = run(oupair_sources(theta, phi, 0.0), 200, 400)
    assert np.all(orc.field(O.F_OU_MEAN) == 10.0)          # noise 0: the mean stays put
    spread = (P[100:, :, 0] - P[100:, :, 1]).ravel()
    want = 2 * (10 * phi) ** 2 / (1 - (1 - theta) ** 2)
    assert abs(spread.var() / want - 1) < 0.05
    orc2, P2 = run(oupair_sources(0.015, 0.01, 0.03), 50, 60)
    m = orc2.field(O.F_OU_MEAN)
    assert np.array_equal(m[:, 0], m[:, 1]) and not np.all(m == 10.0)


def test_simpletrend_statistics():
    """No trend (trendProb 0): y *= 1 + N(0, noise), floored at .01; with
    trends: the switch rate matches trendProb and lengths lie in [min, max]."""
    orc, P = run(simpletrend_sources(2, [0.0, 20, 80, 0.01, 10.0, 0.001, 0.01]), 300, 200)
    r = (P[1:] / P[:-1] - 1).ravel()
    assert abs(r.std() - 0.01) < 5e-4 and abs(r.mean()) < 5e-4
    orc, P = run(simpletrend_sources(1, [0.02, 20, 80, 0.0, 10.0, 0.001, 0.01]), 400, 300)
    tl = orc.field(O.F_TLEN)
    assert tl.min() >= 0 and tl.max() <= 80
    # noise 0: a trending step moves y by exactly y*dY*dir
    moves = P[1:, :, 0] / P[:-1, :, 0] - 1
    active = np.abs(moves) > 0
    assert 0.05 < active.mean() < 0.95
    assert np.all(np.abs(moves[active]) <= 0.0100000001) and np.all(np.abs(moves[active]) >= 0.00099999)


def test_trendyou_statistics():
    """ouComponent mean-reverts to 0 with noise scaled by the trend component;
    price = ou + trend; reset restores start (DataSource.cpp:1608-1653)."""
    orc, P = run(trendyou_sources(3, [0.0, 10, 60, 0.001, 0.03, 5.0, 0.1, 0.02, 0.0, 0.1]), 300, 300)
    ou = orc.field(O.F_SINE_X)
    tc = orc.field(O.F_OU_MEAN)
    assert np.all(tc == 5.0)                                 # no trends: component stays at start
    want = (5.0 * 0.02) ** 2 / (1 - 0.9 ** 2)
    assert abs(ou.var() / want - 1) < 0.15 and abs(ou.mean()) < 0.03
    assert np.array_equal(P[-1], ou + tc)
    orc.reset()
    assert np.all(orc.field(O.F_OU_MEAN) == 5.0)
    orc, P = run(trendyou_sources(2), 300, 400)
    assert orc.field(O.F_OU_MEAN).min() >= 0.1               # floored at .1


def test_config_surface():
    from madigan_amd.config import ConfigError, default_spec, spec_from_config
    from madigan_amd import _lib as L
    s = spec_from_config({"data_source_type": "SimpleTrend", "data_source_config": {
        "trend_prob": [.01], "min_period": [5], "max_period": [9], "noise": [.01], "dYMin": [.001],
        "dYMax": [.002], "start": [3.]}})
    assert s.kinds == [L.SRC_SIMPLETREND] and s.params[0][4] == 3.0 and s.assets == ["SimpleTrend_0"]
    s = spec_from_config({"data_source_type": "OUPair", "data_source_config": {
        "theta": .1, "phi": .01, "noise": .02}})
    assert s.kinds == [L.SRC_OUPAIR] * 2 and [p[3] for p in s.params] == [0.0, 1.0]
    with pytest.raises(ConfigError, match=" key not found"):   # Config.cpp:324 quirk
        spec_from_config({"data_source_type": "Gaussian",
                          "data_source_config": {"mean": [1.], "var": [1.]}})
    assert default_spec("Gaussian").n_assets == 4 and default_spec("OUPair").n_assets == 2
    assert default_spec("TrendyOU").kinds == [L.SRC_TRENDYOU] * 2
    assert default_spec("Triangle").kinds == [L.SRC_TRIANGLE] * 4
    comp = spec_from_config({"data_source_type": "Composite", "data_source_config": {
        "a": {"data_source_type": "OUPair", "data_source_config": {"theta": .1, "phi": .01, "noise": 0.}},
        "b": {"data_source_type": "TrendyOU", "data_source_config": {
            "trend_prob": [.01], "min_period": [5], "max_period": [9], "dYMin": [.001],
            "dYMax": [.002], "start": [3.], "theta": [.1], "phi": [.01], "noise_trend": [0.],
            "ema_alpha": [.1]}}}})
    assert comp.kinds == [L.SRC_OUPAIR, L.SRC_OUPAIR, L.SRC_TRENDYOU]
