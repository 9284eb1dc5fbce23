"""Pin the oracle to golden vectors produced by the reference's own Python
(tests/golden/make_golden.py: madigan/utils/buffers/nstep_buffer.py DSR/DDR/
cosine PPC / sharpe_shaper / sortino_shaperA/B driven like ReplayBuffer.add,
and madigan/utils/preprocessor.py StackerDiscrete with its normalisers,
StackerDiscreteReturns, StackerDiscretePairs and MultiStackerDiscrete).  Tolerance rtol 1e-12: the restatement sums in a fixed
order, NumPy in its own pairwise order."""
import math
import os

import numpy as np
import pytest

from oracle import oracle as O

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "reference_vectors.npz"))
CASES = [str(c) for c in G["shaper_cases"]]


def test_eps_is_float32_eps():
    assert float(G["eps"]) == 1.1920928955078125e-07  # nstep_buffer.py:20


@pytest.mark.parametrize("case", CASES)
def test_nstep_shaper_matches_reference(case):
    shaper = str(G[case + "_shaper"]) if case + "_shaper" in G.files else case.split("_")[0]
    sexp = float(G[case + "_exp"]) if case + "_exp" in G.files else 2.0
    rewards = G[case + "_rewards"]
    ports = G[case + "_ports"]
    dones = G[case + "_dones"]
    n, gamma, eta, temp = G[case + "_cfg"]
    n = int(n)
    desired = G[case + "_desired"]
    discounts = np.array([math.pow(gamma, i) for i in range(n)])
    T, D = rewards.shape
    A = np.zeros(D)
    B = np.zeros(D)
    buf, outs = [], []

    def pop():  # NStepBuffer.pop_nstep_sarsd (nstep_buffer.py:337-356)
        r = np.array([rewards[t] for t in buf])
        if shaper == "DSR":
            out = O.dsr(r, discounts[:len(buf)], eta, A, B)
        elif shaper == "DDR":
            out = O.dsr(r, discounts[:len(buf)], eta, A, B, ddr=True)
        elif shaper in ("sharpe_shaper", "sortino_shaperA", "sortino_shaperB"):
            out = O.naive(shaper, r, discounts[:len(buf)], sexp)
        else:
            out = O.ppc(r, np.array([ports[t] for t in buf]), desired, temp, discounts[:len(buf)])
        buf.pop(0)
        return out

    for t in range(T):  # ReplayBuffer.add (replay_buffer.py:68-80)
        buf.append(t)
        if len(buf) >= n:
            outs.append(pop())
        if dones[t]:
            while buf:
                outs.append(pop())
    np.testing.assert_allclose(np.array(outs), G[case + "_out"], rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("norm", ["log", "lookback", "standard_normal", "lookback_log"])
def test_window_matches_reference_stacker(norm):
    prices, ports, W = G["win_prices"], G["win_ports"], int(G["win_W"])
    T, F = prices.shape
    r = O.Ring(1, F, F + 1, W, norm)
    for t in range(T):
        r.push(prices[t], ports[t], t + 2)
        pr, po, ts = r.gather()
        np.testing.assert_allclose(pr[0], G[f"win_{norm}_price"][t], rtol=1e-12, atol=1e-300,
                                   err_msg=f"t={t}")
        assert np.array_equal(po[0], G[f"win_{norm}_port"][t])
        assert np.array_equal(ts[0].astype(np.int64), G[f"win_{norm}_ts"][t])


def test_stacker_without_norm_type_raises_like_reference():
    assert bool(G["win_none_raises"])
    from madigan_amd.preprocessor import StackerDiscrete
    with pytest.raises(NotImplementedError):
        StackerDiscrete(8, 3, norm=False, norm_type=None)


def _golden_view(key, t):
    rows, cols, prow = G[key + "_shape"][t]
    return (G[key + "_price"][t, :rows, :cols], G[key + "_port"][t, :prow],
            G[key + "_ts"][t, :prow])


def test_window_log_standard_normal_matches_reference():
    prices, ports, W = G["var_prices"], G["var_ports"], int(G["var_W"])
    T, F = prices.shape
    r = O.Ring(1, F, F + 1, W, "log_standard_normal")
    for t in range(T):
        r.push(prices[t], ports[t], t + 2)
        pr, po, ts = r.gather()
        gp, gpo, gts = _golden_view("var_lsn", t)
        n = gp.shape[0]
        np.testing.assert_allclose(pr[0, :n], gp, rtol=1e-12, atol=1e-12, err_msg=f"t={t}")
        assert np.array_equal(po[0, :n], gpo) and np.array_equal(ts[0, :n].astype(np.int64), gts)


@pytest.mark.parametrize("norm", ["log", "lookback", "standard_normal"])
def test_stacker_returns_matches_reference(norm):
    prices, ports, W = G["var_prices"], G["var_ports"], int(G["var_W"])
    T, F = prices.shape
    r = O.Ring(1, F, F + 1, W, norm)
    for t in range(T):
        r.push(prices[t], ports[t], t + 2)
        pr, po, ts = O.returns_view(r)
        gp, gpo, gts = _golden_view(f"var_returns_{norm}", t)
        assert pr.shape == gp.shape  # (len, F - 1): diff across features (axis -1)
        np.testing.assert_allclose(pr, gp, rtol=1e-12, atol=1e-14, err_msg=f"t={t}")
        assert np.array_equal(po, gpo) and np.array_equal(ts, gts)


@pytest.mark.parametrize("norm", ["lookback", "log"])
def test_stacker_pairs_matches_reference(norm):
    prices, ports, W = G["var_prices"], G["var_ports"], int(G["var_W"])
    T = prices.shape[0]
    r = O.Ring(1, 1, ports.shape[1], W, norm)
    for t in range(T):
        r.push(O.pairs_row(prices[t, :2]), ports[t], t + 2)
        pr, po, ts = r.gather()
        gp, gpo, gts = _golden_view(f"var_pairs_{norm}", t)
        n = gp.shape[0]
        np.testing.assert_allclose(pr[0, :n], gp, rtol=1e-12, err_msg=f"t={t}")
        assert np.array_equal(po[0, :n], gpo) and np.array_equal(ts[0, :n].astype(np.int64), gts)


@pytest.mark.parametrize("norm", ["lookback", "standard_normal"])
def test_multi_stacker_matches_reference(norm):
    prices, ports, W = G["var_prices"], G["var_ports"], int(G["var_W"])
    T, F = prices.shape
    m = O.MultiRing(W, list(G["var_multi_dilations"]), F, F + 1, norm)
    ok = G[f"var_multi_{norm}_ok"]
    assert ok.sum() > 5 and not ok.all()
    for t in range(T):
        m.push(prices[t], ports[t], t + 2)
        v = m.view()
        assert (v is not None) == bool(ok[t]), f"t={t}"
        if v is None:
            continue
        gp, gpo, gts = _golden_view(f"var_multi_{norm}", t)
        np.testing.assert_allclose(v[0], gp, rtol=1e-12, atol=1e-14, err_msg=f"t={t}")
        assert np.array_equal(v[1], gpo) and np.array_equal(v[2], gts)


def test_expanding_norm_raises_like_reference():
    assert bool(G["win_expanding_raises"])
