"""GPU parity of the HDF replay DataSource: the file is read by
libmadigan_hdf.so, one period of HDFSourceSingle's cache walk is staged into
HBM (pinned double-buffered H2D), and the step kernel reads it in place.  The
oracle runs HDFSourceSingle's iterCache / loadData state machine
(DataSource.cpp:368-408) over the same arrays.  Everything that feeds back
into state is bit-exact; rewards at rtol 1e-12."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.test_gpu_parity import assert_bits, close

pytestmark = pytest.mark.gpu

KEYS = dict(price_key="price", feature_key="features", timestamp_key="timestamps")


def replay_file(tmp_path, T=300, A=3, F=5, seed=0):
    from madigan_amd import write_hdf
    rng = np.random.default_rng(seed)
    price = 10.0 * np.exp(np.cumsum(rng.normal(0, 0.05, (T, A)), axis=0))
    feats = rng.normal(0, 1, (T, F))
    ts = (1_600_000_000_000_000_000 + np.cumsum(rng.integers(1, 60, T)) * 1_000_000_000).astype(np.uint64)
    path = str(tmp_path / "replay.h5")
    codes = [f"FX{i}" for i in range(A)]
    write_hdf(path, "fx/minute", codes if A > 1 else codes[:1], price if A > 1 else price[:, 0],
              feats, ts, **KEYS)
    return path, price, feats, ts


def hdf_config(path, cache, start=None, end=None):
    d = dict(filepath=path, group_key="fx/minute", cache_size=cache, **KEYS)
    if start is not None:
        d["start_time"], d["end_time"] = int(start), int(end)
    return {"data_source_type": "HDFSourceSingle", "data_source_config": d}


@pytest.mark.parametrize("A,F,cache,stride,window,norm,sched", [
    (3, 5, 37, 7, 8, "lookback", "auto"), (1, 2, 300, 0, 0, None, "auto"),
    (8, 8, 64, 11, 16, "log", "auto"), (8, 8, 64, 11, 16, "log", "single"),
    (16, 3, 25, 5, 4, "standard_normal", "auto"), (16, 16, 25, 5, 0, None, "auto")])
def test_replay_rollout_bitwise(gpu, tmp_path, A, F, cache, stride, window, norm, sched):
    """Both step schedules: "auto" runs the two-role kernel for A >= 2 (tape
    rows prefetched by the generator lanes), "single" forces k_step."""
    from madigan_amd import BatchedEnv
    from madigan_amd import _lib as L
    from madigan_amd.config import spec_from_config
    path, price, feats, ts = replay_file(tmp_path, A=A, F=F, seed=A)
    # a bounded time range that is not a multiple of the cache
    start, end = int(ts[10]) + 1, int(ts[-20])
    spec = spec_from_config(hdf_config(path, cache, start, end))
    assert spec.n_assets == A and spec.n_feats == F
    N, K = 64, 160
    # leveraged (required margin .1, half the available margin per order) on a
    # volatile path, so margin calls end episodes and auto-reset runs
    kw = dict(required_margin=0.1, maintenance_margin=0.25, slippage_rel=1e-4,
              transaction_cost_rel=0.002, reward_shaper="DDR", adaptation_rate=0.001,
              unit_size=0.5, auto_reset=True, window=window, norm_type=norm, seed=5)
    g = BatchedEnv(spec, N, device=gpu, replay_stride=stride, **kw)
    if sched == "single":
        L.check(g.lib.mgn_set_schedule(g.h, L.SCHED_SINGLE), g.h)
    else:
        assert g.lib.mgn_get_schedule(g.h) == (L.SCHED_DUO if A >= 2 else L.SCHED_SINGLE)
    first, second, _, _ = O.hdf_bounds(ts, start, end)
    okw = dict(kw, n_envs=N, n_feats=F, auto_reset=1)
    orc = O.OracleBatch(okw, [(O.SRC_REPLAY, [])] * A)
    period = orc.set_replay(price, feats, ts, first, second, cache, stride)
    assert period == g._tape["ts"].shape[0]
    acts = g.generate_actions(K, seed=3)
    out = g.rollout(acts)
    ref = orc.rollout(acts.cpu().numpy())
    o = {k: v.cpu().numpy() for k, v in out.items()}
    for k in ("obs_price", "obs_port", "tprice", "tunits", "tcost"):
        assert_bits(o[k], ref[k], k)
    for k in ("risk", "done", "margin_call", "data_end"):
        assert np.array_equal(o[k], ref[k]), k
    assert np.array_equal(o["timestamp"].astype(np.uint64), ref["timestamp"])
    assert o["data_end"].any() or (stride == 0 and period > K + 1)  # the walk reached the end
    assert o["done"].any() or A == 1
    close(o["reward"], ref["reward"], "reward")
    close(o["shaped"], ref["shaped"], "shaped")
    assert_bits(g.ledger.cpu().numpy(), orc.field(O.F_LEDGER), "ledger")
    assert_bits(g.prices.cpu().numpy(), orc.field(O.F_PRICE), "prices")
    assert_bits(g.cash.cpu().numpy(), orc.scalar("cash"), "cash")
    assert np.array_equal(g.timestamp.cpu().numpy().astype(np.uint64),
                          orc.scalar("timestamp").astype(np.uint64))
    if window:
        wp, wq, wt = (t.cpu().numpy() for t in g.window())
        rp, rq, rt = orc.window()
        close(wp, rp, "window price")
        assert_bits(wq, rq, "window port")
        assert np.array_equal(wt.astype(np.uint64), rt)


def test_replay_dropin_env_kat(gpu, tmp_path):
    """Env("HDFSourceSingle", ...) on envTest.cpp's fixture: the constructor
    serves row 0, steps serve rows 1..8, dataEnd() after row 8 (currentIdx ==
    boundsIdx.second = 9), then the walk rewinds to row 0."""
    from madigan_amd import make_env, write_hdf
    i = np.arange(10)
    path = str(tmp_path / "test_envTest.h5")
    write_hdf(path, "group/dataset", ["Test"], i.astype(float), (i ** 3).astype(float).reshape(-1, 1),
              (i * i).astype(np.uint64), price_key="midprice", feature_key="feats",
              timestamp_key="timestamp")
    cfg = {"env_type": "Synth", "data_source_type": "HDFSourceSingle", "init_cash": 1_000_000,
           "required_margin": 1.0, "maintenance_margin": 0.25, "transaction_cost_rel": 0.0,
           "transaction_cost_abs": 0.0, "slippage_rel": 0.0, "slippage_abs": 0.0,
           "data_source_config": {"filepath": path, "group_key": "group/dataset",
                                  "price_key": "midprice", "feature_key": "feats",
                                  "timestamp_key": "timestamp", "cache_size": 10}}
    env = make_env(cfg)
    assert env.nAssets == 1 and env.nFeats == 1 and env.isDateTime
    assert env.currentPrices.tolist() == [0.0] and env.timestamp == 0
    seen = []
    for k in range(12):
        state, reward, done, info = env.step(np.array([0.0]))
        seen.append((state.price.tolist(), state.timestamp, info.dataEnd, env.dataEnd()))
    rows = [1, 2, 3, 4, 5, 6, 7, 8, 0, 1, 2, 3]
    assert [s[0] for s in seen] == [[float(r ** 3)] for r in rows]
    assert [s[1] for s in seen] == [r * r for r in rows]
    assert [s[2] for s in seen] == [r == 8 for r in rows] == [s[3] for s in seen]
    # a buy at row r's price, marked at r+1: the ledger sees the file's prices
    env.reset()  # HDFSourceSingle::reset carries on (DataSource.cpp:200-206)
    assert env.currentPrices.tolist() == [4.0]
    s, r, d, info = env.step(np.array([10.0]))
    assert info.brokerResponse.transactionPrice.tolist() == [4.0]
    assert env.ledger.tolist() == [10.0] and env.currentPrices.tolist() == [5.0]


def test_replay_tape_given_directly_and_sharding(gpu):
    """A device tape passed as tensors; two shards (env_offset) reproduce the
    unsharded run (cursor = (global env * stride) mod rows)."""
    import torch
    from madigan_amd import BatchedEnv, replay_spec
    rng = np.random.default_rng(9)
    P, A, F = 97, 4, 4
    price = 5.0 + rng.random((P, A))
    tape = dict(price=torch.tensor(price, device=gpu), feats=torch.tensor(price, device=gpu),
                ts=torch.arange(P, dtype=torch.int64, device=gpu) * 10,
                data_end=torch.zeros(P, dtype=torch.uint8, device=gpu))
    tape["data_end"][-1] = 1
    kw = dict(required_margin=1.0, maintenance_margin=0.25, transaction_cost_rel=0.01,
              auto_reset=True, replay_stride=13, replay_tape=tape, seed=1)
    N, K = 32, 50
    full = BatchedEnv(replay_spec(A, F), N, device=gpu, **kw)
    acts = full.generate_actions(K, seed=4)
    of = full.rollout(acts)
    halves = []
    for r in range(2):
        h = BatchedEnv(replay_spec(A, F), N // 2, device=gpu, env_offset=r * N // 2, **kw)
        halves.append(h.rollout(acts[:, r * N // 2:(r + 1) * N // 2].contiguous()))
    for k in ("obs_price", "obs_port", "tprice", "reward", "timestamp", "data_end"):
        cat = torch.cat([halves[0][k], halves[1][k]], dim=1)
        assert torch.equal(cat, of[k]), k
    # cursor of env e after construction + K steps: (e*13 + 1 + K) mod P (no resets consume
    # extra rows without a window)
    cur = full.replay_cursor.cpu().numpy()
    steps = 1 + K + (of["done"].cpu().numpy().sum(axis=0))  # each auto-reset ticks once
    assert np.array_equal(cur, (np.arange(N) * 13 + steps) % P)


@pytest.mark.parametrize("A,F,window,norm", [(16, 16, 8, None), (4, 3, 6, "log"), (3, 5, 8, "lookback")])
def test_replay_window_history(gpu, tmp_path, A, F, window, norm):
    """The windowed agent loop on a replay source (the C5 path): K steps in one
    launch with every step's window (mgn_rollout_hist / mgn_window_hist) equal
    the oracle's window after each step; feature columns come from the tape
    (prefetched one tick ahead when every feature has a lane)."""
    from madigan_amd import BatchedEnv
    from madigan_amd.config import spec_from_config
    path, price, feats, ts = replay_file(tmp_path, T=400, A=A, F=F, seed=A + 1)
    start, end = int(ts[3]) + 1, int(ts[-5])
    spec = spec_from_config(hdf_config(path, 50, start, end))
    N, K = 48, 20
    kw = dict(required_margin=0.1, maintenance_margin=0.25, slippage_rel=1e-4,
              transaction_cost_rel=0.002, reward_shaper="DDR", adaptation_rate=0.001,
              unit_size=0.5, auto_reset=True, window=window, norm_type=norm, seed=5)
    g = BatchedEnv(spec, N, device=gpu, replay_stride=13, **kw)
    first, second, _, _ = O.hdf_bounds(ts, start, end)
    okw = dict(kw, n_envs=N, n_feats=F, auto_reset=1)
    orc = O.OracleBatch(okw, [(O.SRC_REPLAY, [])] * A)
    orc.set_replay(price, feats, ts, first, second, 50, 13)
    acts = g.generate_actions(2 * K, seed=4)
    a = acts.cpu().numpy()
    dones = 0
    for half in range(2):  # two launches: the second starts from the first's ring
        out, (wp, wo, wt) = g.rollout_window(acts[half * K:(half + 1) * K], per_step=True)
        for k in range(K):
            r = orc.rollout(a[half * K + k:half * K + k + 1])
            dones += int(r["done"].sum())
            assert_bits(out["obs_price"][k].cpu().numpy(), r["obs_price"][0], f"obs_price {half}/{k}")
            rpr, rpo, rts = orc.window()
            if norm is None:
                assert_bits(wp[k].cpu().numpy(), rpr, f"window price {half}/{k}")
            else:
                close(wp[k].cpu().numpy(), rpr, f"window price {half}/{k}",
                      rtol=1e-14 if norm == "lookback" else 1e-12)
            assert_bits(wo[k].cpu().numpy(), rpo, f"window portfolio {half}/{k}")
            assert np.array_equal(wt[k].cpu().numpy().astype(np.uint64), rts)
    assert dones > 0 or A == 1


@pytest.mark.parametrize("F,window", [(16, 0), (20, 0), (16, 8)])
def test_replay_trio_equals_duo_sixteen_assets(gpu, F, window):
    """The three-role kernel on a replay tape (16 assets, the 256-lane layout:
    4096 envs) against the two-role kernel from the same construction: every
    output, the window and the final state bit for bit, through auto-resets
    (a leveraged, costly broker), 20- and 1-step launches; F > 16 features
    take the read-back-per-column path."""
    import torch
    from madigan_amd import BatchedEnv, replay_spec
    from madigan_amd import _lib as L
    rng = np.random.default_rng(21 + F)
    P, A, N = 503, 16, 4096
    price = 5.0 * np.exp(np.cumsum(rng.normal(0, 0.03, (P, A)), axis=0))
    feats = rng.normal(0, 1, (P, F))
    tape = dict(price=torch.tensor(price, device=gpu), feats=torch.tensor(feats, device=gpu),
                ts=torch.arange(P, dtype=torch.int64, device=gpu) * 60 + 7,
                data_end=torch.zeros(P, dtype=torch.uint8, device=gpu))
    tape["data_end"][-1] = 1
    kw = dict(required_margin=0.1, maintenance_margin=0.5, transaction_cost_rel=0.02, unit_size=0.9,
              auto_reset=True, replay_stride=29, replay_tape=tape, seed=3, reward_shaper="DDR",
              window=window, init_cash=1e5)
    res = []
    for sched in (L.SCHED_DUO, L.SCHED_TRIO):
        g = BatchedEnv(replay_spec(A, F), N, device=gpu, **kw)
        L.check(g.lib.mgn_set_schedule(g.h, sched), g.h)
        assert g.lib.mgn_get_schedule(g.h) == sched
        acts = g.generate_actions(41, seed=8)
        outs = [g.rollout(acts[:20]), g.rollout(acts[20:21]), g.rollout(acts[21:])]
        host = [{k: v.cpu().numpy() for k, v in o.items()} for o in outs]
        win = [t.cpu().numpy() for t in g.window()] if window else []
        state = [t.cpu().numpy() for t in (g.ledger, g.cash, g.prices, g.timestamp, g.replay_cursor,
                                           g.episode_stats, g.shaper_a, g.shaper_b)]
        res.append((host, win, state))
    (h0, w0, s0), (h1, w1, s1) = res
    assert sum(int(h["done"].sum()) for h in h0) > 0, "no episode ended"
    def same(x, y, what):
        if x.dtype == np.float64:
            assert_bits(y, x, what)
        else:
            np.testing.assert_array_equal(y, x, err_msg=what)
    for a, b in zip(h0, h1):
        for k in a:
            same(a[k], b[k], f"trio vs duo {k}")
    for i, (a, b) in enumerate(zip(w0 + s0, w1 + s1)):
        same(a, b, f"trio vs duo window/state {i}")
