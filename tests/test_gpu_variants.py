"""GPU parity for the naive n-step shapers and the StackerDiscrete variants.

* sharpe_shaper / sortino_shaperA / sortino_shaperB (nstep_buffer.py:207-312)
  inside the fused step kernel, n = 1 and n > 1 with done flushes, against the
  oracle (itself pinned to the reference's Python in tests/test_golden.py);
  rtol 1e-10 (x**(1/e) for e != 2 is libm pow vs ocml pow).
* log_standard_normal windows, StackerDiscreteReturns / StackerDiscretePairs /
  MultiStackerDiscrete (preprocessor.py:95-107, :202-327) through the device
  rings, against the golden vectors the reference's own classes produced.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.configs import ou_sources, trendou_sources
from tests.test_gpu_parity import assert_bits, close, make_pair, out_check, state_check

pytestmark = pytest.mark.gpu

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "reference_vectors.npz"))
TOU = [0.2, 2, 6, 0.05, 0.2, 5.0, 0.15, 0.3, 0.2, 0.99]


@pytest.mark.parametrize("shaper,sexp,mode,n", [
    ("sharpe_shaper", 2, "env_log", 1), ("sortino_shaperA", 2, "env_log", 1),
    ("sortino_shaperB", 3, "agent_per_asset", 1), ("sharpe_shaper", 2, "agent_per_asset", 5),
    ("sortino_shaperA", 3, "env_log", 4), ("sortino_shaperB", 2, "agent_sum", 20)])
def test_naive_shapers_rollout(gpu, shaper, sexp, mode, n):
    N, A, K = 128, 3, 48
    kw = dict(required_margin=0.02, maintenance_margin=0.25, transaction_cost_rel=0.02,
              unit_size=0.9, auto_reset=1, init_cash=1e5, reward_shaper=shaper, reward_mode=mode,
              sortino_exp=sexp, nstep_return=n, discount=0.97)
    g, orc = make_pair(trendou_sources(A, TOU), N, **kw)
    acts = g.generate_actions(2 * K, seed=31)
    D = A if mode == "agent_per_asset" else 1
    for half in range(2):
        a = acts[half * K:(half + 1) * K]
        out = g.rollout(a)
        ref = orc.rollout(a.cpu().numpy())
        host = {k: v.cpu().numpy() for k, v in out.items()}
        assert ref["done"].sum() > 0
        out_check({**host, "shaped": ref["shaped"]}, ref, f"{shaper}{half}", D)
        assert np.array_equal(host["n_shaped"], ref["n_shaped"]), "n_shaped"
        np.testing.assert_allclose(host["shaped"], ref["shaped"], rtol=1e-10, atol=1e-14,
                                   err_msg="shaped")
    state_check(g, orc, "end")


def test_sortino_needs_exp_like_reference(gpu):
    from madigan_amd import BatchedEnv
    from tests.configs import spec_from_sources
    with pytest.raises(KeyError):  # shaper_config["sortino_exp"] (nstep_buffer.py:392)
        BatchedEnv(spec_from_sources(ou_sources(2)), 4, reward_shaper="sortino_shaperA")


def test_env_window_log_standard_normal(gpu):
    N, A, K, W = 160, 4, 40, 16
    kw = dict(required_margin=1.0, maintenance_margin=0.25, transaction_cost_rel=0.02,
              reward_shaper="DSR", window=W, norm_type="log_standard_normal", auto_reset=1)
    g, orc = make_pair(ou_sources(A), N, **kw)
    g.reset()
    orc.reset()
    acts = g.generate_actions(K, seed=5)
    g.rollout(acts)
    orc.rollout(acts.cpu().numpy())
    pr, po, ts = g.window()
    rpr, rpo, rts = orc.window()
    np.testing.assert_allclose(pr.cpu().numpy(), rpr, rtol=1e-12, atol=1e-12)
    assert_bits(po.cpu().numpy(), rpo, "window portfolio")
    assert np.array_equal(ts.cpu().numpy().astype(np.uint64), rts)


def _golden_view(key, t):
    rows, cols, prow = G[key + "_shape"][t]
    return (G[key + "_price"][t, :rows, :cols], G[key + "_port"][t, :prow],
            G[key + "_ts"][t, :prow])


def _stream_and_check(pp, key, feed, tol=1e-12, ok=None):
    from madigan_amd import State
    ports = G["var_ports"]
    for t in range(feed.shape[0]):
        pp.stream_state(State(feed[t], ports[t], t + 2))
        if ok is not None and not ok[t]:
            with pytest.raises(ValueError):
                pp.current_data()
            continue
        cur = pp.current_data()
        gp, gpo, gts = _golden_view(key, t)
        price = np.asarray(cur.price)
        assert price.reshape(gp.shape[0], -1).shape == gp.shape, f"{key} t={t}"
        np.testing.assert_allclose(price.reshape(gp.shape), gp, rtol=tol, atol=1e-12,
                                   err_msg=f"{key} t={t}")
        assert np.array_equal(np.asarray(cur.portfolio), gpo), f"{key} t={t} port"
        assert np.array_equal(np.asarray(cur.timestamp).astype(np.int64), gts), f"{key} t={t} ts"


def test_stacker_log_standard_normal_golden(gpu):
    from madigan_amd import StackerDiscrete
    W = int(G["var_W"])
    F = G["var_prices"].shape[1]
    _stream_and_check(StackerDiscrete(W, F, norm=True, norm_type="log_standard_normal"), "var_lsn",
                      G["var_prices"])


@pytest.mark.parametrize("norm", ["log", "lookback", "standard_normal"])
def test_stacker_returns_golden(gpu, norm):
    from madigan_amd import StackerDiscreteReturns
    W = int(G["var_W"])
    F = G["var_prices"].shape[1]
    _stream_and_check(StackerDiscreteReturns(W, F, norm=True, norm_type=norm),
                      f"var_returns_{norm}", G["var_prices"])


@pytest.mark.parametrize("norm", ["lookback", "log"])
def test_stacker_pairs_golden(gpu, norm):
    from madigan_amd import StackerDiscretePairs
    W = int(G["var_W"])
    _stream_and_check(StackerDiscretePairs(W, 2, norm=True, norm_type=norm), f"var_pairs_{norm}",
                      G["var_prices"][:, :2])


@pytest.mark.parametrize("norm", ["lookback", "standard_normal"])
def test_multi_stacker_golden(gpu, norm):
    from madigan_amd import MultiStackerDiscrete
    W = int(G["var_W"])
    F = G["var_prices"].shape[1]
    ms = MultiStackerDiscrete(W, list(G["var_multi_dilations"]), F, norm=True, norm_type=norm)
    _stream_and_check(ms, f"var_multi_{norm}", G["var_prices"], ok=G[f"var_multi_{norm}_ok"])
    assert len(ms) == W


def test_batched_variants_match_oracle(gpu):
    """Batched States (N envs of device tensors) through Returns / Pairs /
    Multi against the oracle's per-env restatement."""
    import torch
    from madigan_amd import (MultiStackerDiscrete, State, StackerDiscretePairs,
                             StackerDiscreteReturns)
    rng = np.random.default_rng(2)
    N, F, W, T = 5, 3, 6, 17
    prices = 10 + np.cumsum(rng.normal(0, 0.3, (T, N, F)), axis=0)
    ports = rng.normal(0, 0.3, (T, N, F + 1))
    dil = [1, 2]
    ret = StackerDiscreteReturns(W, F, norm=True, norm_type="lookback")
    par = StackerDiscretePairs(W, 2, norm=True, norm_type="log")
    mul = MultiStackerDiscrete(W, dil, F, norm=True, norm_type="standard_normal")
    orr = [O.Ring(1, F, F + 1, W, "lookback") for _ in range(N)]
    orp = [O.Ring(1, 1, F + 1, W, "log") for _ in range(N)]
    orm = [O.MultiRing(W, dil, F, F + 1, "standard_normal") for _ in range(N)]
    dev = torch.device("cuda")
    for t in range(T):
        p = torch.tensor(prices[t], device=dev)
        q = torch.tensor(ports[t], device=dev)
        s = torch.full((N,), t + 2, dtype=torch.int64, device=dev)
        ret.stream_state(State(p, q, s))
        par.stream_state(State(p[:, :2].contiguous(), q, s))
        mul.stream_state(State(p, q, s))
        for e in range(N):
            orr[e].push(prices[t, e], ports[t, e], t + 2)
            orp[e].push(O.pairs_row(prices[t, e, :2]), ports[t, e], t + 2)
            orm[e].push(prices[t, e], ports[t, e], t + 2)
        n = min(t + 1, W)
        rp, rpo, rts = ret.current_data()
        pp, ppo, pts = par.current_data()
        for e in range(N):
            a, b, c = O.returns_view(orr[e])
            close(rp[e, :n].cpu().numpy(), a, f"returns t={t}", rtol=1e-14)
            assert_bits(rpo[e, :n - 1].cpu().numpy(), b, "returns port")
            x, y, z = orp[e].gather()
            close(pp[e, :n].cpu().numpy(), x[0, :n], f"pairs t={t}")
        v = orm[0].view()
        if v is None:
            with pytest.raises(ValueError):
                mul.current_data()
            continue
        mp, mpo, mts = mul.current_data()
        for e in range(N):
            v = orm[e].view()
            close(mp[e, :n].cpu().numpy(), v[0], f"multi t={t}", rtol=1e-14)
            assert np.array_equal(mts[e, :n].cpu().numpy(), v[2])
