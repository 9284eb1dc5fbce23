"""Pin the oracle to golden vectors produced by the reference's own Python
(tests/golden/make_golden.py: madigan/utils/buffers/nstep_buffer.py DSR/DDR/
cosine PPC driven like ReplayBuffer.add, and madigan/utils/preprocessor.py
StackerDiscrete).  Tolerance rtol 1e-12: the restatement sums in a fixed
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
    shaper = case.split("_")[0]
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
