"""madigan_amd.reward_normalization against the reference's own Cython
normalisers (madigan/environments/reward_normalization.pyx), compiled from the
reference tree by `make -C oracle ref_normalizers` and run by
tests/golden/make_reward_norm_golden.py into tests/golden/reward_norm_vectors.npz
(8 streams x 300 rewards per class and window, resets mid-stream).  The
batched form (all streams in one object, resets by env mask) and the scalar
form (one object per stream, as the reference) match bit for bit."""
import os

import numpy as np
import pytest

from madigan_amd import reward_normalization as RN

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reward_norm_vectors.npz")
CASES = [("SharpeFixedWindow", 5), ("SharpeFixedWindow", 32), ("SortinoFixedWindowA", 7),
         ("SortinoFixedWindowB", 4), ("SortinoFixedWindowB", 16), ("SortinoFixedWindowC", 6),
         ("SharpeEWMA", 10), ("SharpeEWMA", 3)]


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD))


@pytest.mark.parametrize("name,w", CASES)
def test_batched_matches_reference(gold, name, w):
    r, rs, ref = gold["rewards"], gold["resets"], gold[f"{name}_{w}"]
    S, T = r.shape
    obj = getattr(RN, name)(w, n_envs=S)
    out = np.zeros((S, T))
    for t in range(T):
        if rs[:, t].any():
            obj.reset(rs[:, t])
        out[:, t] = obj.stream(r[:, t])
    np.testing.assert_array_equal(out.view(np.int64), ref.view(np.int64), err_msg=name)


@pytest.mark.parametrize("name,w", CASES)
def test_scalar_matches_reference(gold, name, w):
    r, rs, ref = gold["rewards"], gold["resets"], gold[f"{name}_{w}"]
    for e in (0, 2, 3):
        obj = getattr(RN, name)(w)
        got = []
        for t in range(r.shape[1]):
            if rs[e, t]:
                obj.reset()
            v = obj.stream(float(r[e, t]))
            assert isinstance(v, float)
            got.append(v)
        np.testing.assert_array_equal(np.array(got).view(np.int64), ref[e].view(np.int64),
                                      err_msg=f"{name} stream {e}")


def test_make_reward_normalizer_dispatch():
    assert isinstance(RN.make_reward_normalizer({"reward_shaper_config": {"reward_shaper": "none"}}),
                      RN.NullShaper)
    s = RN.make_reward_normalizer({"reward_shaper_config": {"reward_shaper": "SortinoFixedWindowA",
                                                           "window": 9}}, n_envs=4)
    assert isinstance(s, RN.SortinoFixedWindowA) and s.window == 9 and s.N == 4
    with pytest.raises(NotImplementedError):
        RN.make_reward_normalizer({"reward_shaper_config": {"reward_shaper": "Nope"}})
    assert RN.NullShaper().stream(0.25) == 0.25


def test_sharpe_ewma_zero_variance_per_env():
    """A constant reward stream (an agent holding cash) has zero variance:
    the reference's checked division raises ZeroDivisionError for that env's
    shaper.  Batched, only that env's value is void: the error names it and
    carries the other envs' values, which equal independent scalar shapers'
    -- and every env's statistics have advanced, as the scalar shapers' have."""
    rng = np.random.default_rng(3)
    T, N = 6, 4
    r = rng.normal(0, 0.01, (T, N))
    r[:, 2] = 0.25  # env 2: constant
    batched = RN.SharpeEWMA(5, n_envs=N)
    scal = [RN.SharpeEWMA(5) for _ in range(N)]
    for t in range(T):
        want, raised = np.empty(N), []
        for e in range(N):
            try:
                want[e] = scal[e].stream(float(r[t, e]))
            except ZeroDivisionError:
                want[e] = np.nan
                raised.append(e)
        if raised:
            with pytest.raises(RN.ZeroVarianceError) as ei:
                batched.stream(r[t])
            assert isinstance(ei.value, ZeroDivisionError)
            assert ei.value.envs.tolist() == raised == [2]
            got = ei.value.out
        else:
            got = batched.stream(r[t])
        np.testing.assert_array_equal(np.isnan(got), np.isnan(want))
        ok = ~np.isnan(want)
        np.testing.assert_array_equal(got[ok].view(np.int64), want[ok].view(np.int64))
    for e in range(N):
        assert batched.count[e] == scal[e].count[0] == T
        assert batched.ewssq[e] == scal[e].ewssq[0]
