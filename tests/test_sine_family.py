"""SineAdder, SineDynamic and SineDynamicTrend (DataSource.cpp:582-1051,
WaveTableOsc.h) in the oracle and the config layer.  Their reference draws are
wall-clock / random_device seeded (DataSource.cpp:660, :762, :960;
randomBoolGenerator.h), so parity with the reference is the deterministic
formulas (noise 0, zero-step random walks), the constructors' checks, and the
statistics of the walks; bitwise oracle <-> HIP is in tests/test_gpu_generators.py."""
import math

import numpy as np
import pytest

from madigan_amd import config as CF
from oracle import oracle as O
from tests.configs import sources_from_spec

PI2 = 3.141592653589793238463 * 2


def run(spec, N, T, **cfg):
    orc = O.OracleBatch(dict(n_envs=N, seed=cfg.pop("seed", 5), **cfg), sources_from_spec(spec))
    prices = [orc.field(O.F_PRICE)]
    for _ in range(T):
        prices.append(orc.step()["obs_price"])
    return orc, np.array(prices)


def test_sineadder_formula():
    """noise 0: P = sum_c (0 + mu_c) + amp_c sin((PI2 x_c) f_c), x_c from phase_c, += dX
    (DataSource.cpp:663-673); the Env constructor's getData is tick 0."""
    f, mu, amp, ph = [1., 0.3, 2., 0.5], [2., 2.1, 2.2, 2.3], [1., 1.2, 1.3, 1.], [0., 1., 2., 1.]
    spec = CF.sineadder_spec(f, mu, amp, ph, 0.01, 0.0)
    _, P = run(spec, 2, 300)
    for t in range(301):
        x = np.array(ph) + t * 0.01
        want = 0.0
        for c in range(4):  # sequential sum with x accumulated by repeated += dX
            xc = ph[c]
            for _ in range(t):
                xc += 0.01
            want += (0.0 + mu[c]) + amp[c] * math.sin(PI2 * xc * f[c])
        np.testing.assert_allclose(P[t, :, 0], want, rtol=1e-13, err_msg=f"t={t}")


def test_sineadder_noise_statistics():
    spec = CF.sineadder_spec([1.], [5.], [0.], [0.], 0.01, 0.3)
    _, P = run(spec, 400, 50)
    z = P[1:, :, 0].ravel() - 5.0
    assert abs(z.mean()) < 0.01 and abs(z.std() - 0.3) < 0.01


def _wt(phasor, len_):
    """the interpolated wave-table read (WaveTableOsc.h:84-95) with numpy sin"""
    temp = phasor * len_
    ip = int(temp)
    fr = temp - ip
    s = lambda i: 0.0 if i % len_ == 0 else math.sin(i * 2. * math.pi / len_)
    return s(ip) + (s(ip + 1) - s(ip)) * fr


def test_sinedynamic_oscillator_formula():
    """zero-step walks keep freq/mu/amp at the constructor's draw (lo == hi):
    P_t = sum_c mu_c + amp_c * osc_c, the phasor advancing by freq / sampleRate
    before each read (updatePhase then getOutput, WaveTableOsc.h:31, :98-101)."""
    fr = [[0.7, 0.7, 0.0], [3.3, 3.3, 0.0]]
    mu = [[2.0, 2.0, 0.0], [0.5, 0.5, 0.0]]
    am = [[1.5, 1.5, 0.0], [0.25, 0.25, 0.0]]
    spec = CF.sinedynamic_spec(fr, mu, am, 0.01, 0.0)
    lens = [int(v) for v in spec.params[0][3:5]]
    assert lens == [CF._wave_table_len(100, 0.7), CF._wave_table_len(100, 3.3)]
    _, P = run(spec, 1, 400)
    ph = [0.0, 0.0]
    for t in range(401):
        want = 0.0
        for c in range(2):
            ph[c] += fr[c][0] / 100
            if ph[c] >= 1.0:
                ph[c] -= 1.0
            want += mu[c][0] + am[c][0] * _wt(ph[c], lens[c])
        np.testing.assert_allclose(P[t, 0, 0], want, rtol=1e-12, atol=1e-13, err_msg=f"t={t}")


def test_sinedynamic_random_walk_stays_in_range():
    spec = CF.sinedynamic_spec(*[[r] * 3 for r in ([0.5, 2.0, 0.05], [1.0, 3.0, 0.1], [0.2, 1.0, 0.05])],
                               0.02, 0.0)
    orc, P = run(spec, 50, 600)
    assert np.all(P >= 3 * (1.0 - 1.0)) and np.all(P <= 3 * (3.0 + 1.0))
    # the walk moves: prices are not a fixed-parameter sine sum
    assert np.std(np.diff(P[:, :, 0], axis=0)) > 0.01


def test_sinedynamictrend_trend_component():
    """prob 1, incr .1, lengths in [3, 3]: every tick either continues a trend
    (tc *= 1 + .1*dir, floored at .01) or starts one; tc multiplies the sine
    sum and is added (DataSource.cpp:1017-1047); noise 0."""
    one = [[1.0, 1.0, 0.0]]
    spec = CF.sinedynamictrend_spec(one, [[2.0, 2.0, 0.0]], [[0.0, 0.0, 0.0]], [[3, 3]], [0.1], [1.0],
                                    0.01, 0.0)
    _, P = run(spec, 64, 14)  # (the reconstruction below doubles rounding errors per tick)
    # the sum uses tc before the trend update, the added term after it:
    # P_t = 2 tc_{t-1} + tc_t, tc = 1 before the first tick
    tc = np.empty_like(P[:, :, 0])
    prev = np.ones(P.shape[1])
    for t in range(P.shape[0]):
        tc[t] = P[t, :, 0] - 2 * prev
        prev = tc[t]
    tc = np.vstack([np.ones(P.shape[1]), tc])
    ratios = tc[1:] / tc[:-1]
    ok = np.isclose(ratios, 1.1) | np.isclose(ratios, 0.9) | np.isclose(ratios, 1.0) | (tc[1:] <= 0.0100001)
    assert ok.all()
    assert np.isclose(ratios, 1.1).any() and np.isclose(ratios, 0.9).any()


def test_sine_family_config_like_reference():
    with pytest.raises(RuntimeError):  # the default constructors pass dX = 0: Nyquist check throws
        CF.default_spec("SineDynamic")
    with pytest.raises(RuntimeError):
        CF.default_spec("SineDynamicTrend")
    s = CF.default_spec("SineAdder")
    assert s.assets == ["multi_sine"] and s.params[0][:3] == [4.0, 0.01, 0.0]
    with pytest.raises(RuntimeError):  # missing key -> ConfigError
        CF.spec_from_config({"data_source_type": "SineDynamic",
                             "data_source_config": {"freqRange": [[1, 2, .1]], "muRange": [[1, 2, .1]],
                                                    "ampRange": [[1, 2, .1]], "dX": .01}})
    with pytest.raises(RuntimeError):  # freqRange high * 2 > sampleRate (100)
        CF.sinedynamic_spec([[1., 60., .1]], [[1, 2, .1]], [[1, 2, .1]], 0.01, 0.)
    with pytest.raises(ValueError):
        CF.sinedynamic_spec([[1., 2., .1]], [[1, 2, .1], [1, 2, .1]], [[1, 2, .1]], 0.01, 0.)
    with pytest.raises(ValueError):
        CF.sineadder_spec([1.], [1., 2.], [1.], [0.], 0.01)
    cfg = {"data_source_type": "SineDynamicTrend",
           "data_source_config": {"freqRange": [[.1, 1., .01]], "muRange": [[1., 5., .02]],
                                  "ampRange": [[1., 5., .01]], "trendRange": [[100, 500]],
                                  "trendIncr": [0.1], "trendProb": [.001], "dX": .01, "noise": 1.}}
    s = CF.spec_from_config(cfg)
    assert s.kinds == [O.SRC_SINEDYNTREND] and s.assets == ["sine_dynamic_trend"]
    c, _ = CF.build_config(s, n_envs=2)
    assert c.aux == 1
    assert CF._wave_table_len(100, 0.1) == 2048 and CF._wave_table_len(100, 10.) == 16
