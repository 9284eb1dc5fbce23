"""GPU parity of the SURVEY 8f #4 generators: SimpleTrend, TrendyOU, Gaussian,
SawTooth, Triangle, OUPair (alone and as Composite children), bit-exact
against the oracle on prices and generator state, through resets and every
lane layout (an OUPair's two assets may sit in different lanes)."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.configs import (gaussian_sources, oupair_sources, simpletrend_sources, trendou_sources,
                           trendyou_sources,
                           wave_sources)
from tests.test_gpu_parity import assert_bits, close, gen_state_check, make_pair, out_check, state_check

pytestmark = pytest.mark.gpu

MIX = (simpletrend_sources(2, [0.05, 3, 30, 0.02, 10.0, 0.001, 0.02])
       + oupair_sources(0.05, 0.01, 0.02)
       + trendyou_sources(2, [0.05, 3, 30, 0.01, 0.2, 5.0, 0.1, 0.02, 0.0, 0.1])
       + gaussian_sources([20.0], [1.0])
       + wave_sources(O.SRC_SAWTOOTH, [0.7], [5.0], [1.0], [0.3], 0.011, 0.01)
       + wave_sources(O.SRC_TRIANGLE, [1.3], [6.0], [2.0], [0.1], 0.017, 0.01))


@pytest.mark.parametrize("name,sources", [
    ("SimpleTrend", simpletrend_sources(4, [0.05, 3, 30, 0.02, 10.0, 0.001, 0.02])),
    ("TrendyOU", trendyou_sources(4, [0.05, 3, 30, 0.01, 0.2, 5.0, 0.1, 0.02, 0.0, 0.1])),
    ("Gaussian", gaussian_sources([2., 50., 10.], [1., 5., 0.5])),
    ("SawTooth", wave_sources(O.SRC_SAWTOOTH, [1., 0.3, 2.], [2., 2.1, 2.2], [1., 1.2, 1.3],
                              [0., 1., -2.], 0.013, 0.05)),
    ("Triangle", wave_sources(O.SRC_TRIANGLE, [1., 0.3, 2.], [2., 2.1, 2.2], [1., 1.2, 1.3],
                              [0., 1., -2.], 0.013, 0.05)),
    ("OUPair", oupair_sources(0.05, 0.01, 0.02) * 2),
    ("Mix", MIX),
])
def test_generators_bitwise(gpu, name, sources):
    g, orc = make_pair(sources, 200, required_margin=1.0, maintenance_margin=0.25)
    state_check(g, orc, f"{name} init")
    for t in range(150):
        g.step()
        ref = orc.step()
        o = g.host_outputs()
        assert_bits(o["obs_price"], ref["obs_price"], f"{name} step {t} prices")
    state_check(g, orc, name)
    gen_state_check(g, orc, name)
    assert_bits(g.sine_x.cpu().numpy(), orc.field(O.F_SINE_X), f"{name} x / ouComponent")
    g.reset()
    orc.reset()
    state_check(g, orc, f"{name} reset")
    gen_state_check(g, orc, f"{name} reset")


@pytest.mark.parametrize("layout", [1, 2, 4, 8])
def test_mix_rollout_auto_reset_layouts(gpu, layout):
    """Composite of every new kind under discrete-action rollouts with
    leverage (margin calls -> in-kernel auto-reset) in each lane layout."""
    g, orc = make_pair(MIX, 128, required_margin=0.2, maintenance_margin=0.25,
                       transaction_cost_rel=0.001, reward_shaper="DDR", unit_size=0.5,
                       auto_reset=True, window=6, norm_type="lookback")
    g.lib.mgn_set_layout(g.h, layout)
    acts = g.generate_actions(120, seed=5)
    out = g.rollout(acts)
    ref = orc.rollout(acts.cpu().numpy())
    out_check({k: v.cpu().numpy() for k, v in out.items()}, ref, f"layout {layout}")
    assert ref["done"].any()
    state_check(g, orc, f"layout {layout}")
    gen_state_check(g, orc, f"layout {layout}")
    wp, wq, wt = (t.cpu().numpy() for t in g.window())
    rp, rq, rt = orc.window()
    close(wp, rp, "window price")


def _sine_family():
    from madigan_amd import config as CF
    from tests.configs import sources_from_spec
    add = CF.sineadder_spec([1., 0.3, 2.], [2., 2.1, 2.2], [1., 1.2, 1.3], [0., 1., 2.], 0.01, 0.05)
    dyn = CF.sinedynamic_spec([[.1, 1., .01], [0.3, 3.0, .01], [5., 15., .1]],
                              [[1., 5., .02], [.3, 3., .05], [.2, 5., .02]],
                              [[1., 5., .01], [.3, 3., .02], [.2, 2., .04]], 0.01, 0.5)
    trd = CF.sinedynamictrend_spec([[.1, 1., .01], [5., 15., .1]], [[1., 5., .02], [.2, 5., .02]],
                                   [[1., 5., .01], [.2, 2., .04]], [[3, 9], [2, 5]], [0.1, 0.2],
                                   [.05, .2], 0.01, 0.3)
    return sources_from_spec(add) + sources_from_spec(dyn) + sources_from_spec(trd)


def test_sine_family_bitwise(gpu):
    """SineAdder / SineDynamic / SineDynamicTrend (multi-component state in
    views.aux) bit-exact vs the oracle, through forced margin calls: auto-reset
    resamples the SineDynamic parameters (DataSource.cpp:794-800, :994-1000)."""
    from madigan_amd import _lib as L
    src = _sine_family() + trendou_sources(1, [0.2, 2, 6, 0.05, 0.2, 5.0, 0.15, 0.3, 0.2, 0.99])
    N, K = 160, 64
    kw = dict(required_margin=0.02, maintenance_margin=0.25, transaction_cost_rel=0.02,
              unit_size=0.9, auto_reset=1, init_cash=1e5, reward_shaper="DDR")
    g, orc = make_pair(src, N, **kw)
    assert g.lib.mgn_get_schedule(g.h) == L.SCHED_SINGLE  # multi-component kinds run k_step
    state_check(g, orc, "init")
    acts = g.generate_actions(K, seed=19)
    out = {k: v.cpu().numpy() for k, v in g.rollout(acts).items()}
    ref = orc.rollout(acts.cpu().numpy())
    assert ref["done"].sum() > 0
    out_check(out, ref, "sine family")
    state_check(g, orc, "end")
    for t in range(40):  # no-action ticks
        g.step()
        r = orc.step()
        assert_bits(g.host_outputs()["obs_price"], r["obs_price"], f"tick {t}")
