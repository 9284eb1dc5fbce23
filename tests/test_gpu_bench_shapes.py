"""Parity at the benchmarked shapes where earlier tests left holes:

  * C3's full 8192 x 8 grid with episodes ending inside every launch: the
    three-role kernel speculates "the episode goes on" and rolls a step back
    when it ends; at the headline's own parameters no episode ends in the
    first few hundred steps, so a leveraged, volatile TrendOU variant of the
    same grid forces margin calls and auto-resets.  The bench's launch
    sequence (5, 20, 256 steps; the 20-step launch with the bench's output
    set) bit-exact against the oracle, `done` observed in every launch.
  * C5 at its bench shape: 8192 envs x 16 replay assets (bench.c5_paths, the
    HDFSourceSingle file the bench writes, cache 10000, env stride 997), W = 64,
    DDR, 64-step mgn_rollout_hist launches (until two launches with episode
    ends have run) with every output and the step windows (mgn_window_hist)
    against the oracle's StackerDiscrete.current_data after each step; the
    windows the auto-resets refill are all checked.
"""
import os
import sys

import numpy as np
import pytest

from oracle import oracle as O
from tests.configs import ou_sources, trendou_sources
from tests.test_gpu_parity import assert_bits, close, gen_state_check, make_pair, out_check, state_check

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
THREADS = 8
STD_FIELDS = ("reward", "shaped", "done", "obs_price", "obs_port", "timestamp", "tprice", "tunits",
              "tcost", "risk", "margin_call")


def _host(out):
    return {k: v.cpu().numpy() for k, v in out.items()}


def test_c3_full_grid_forced_resets(gpu):
    from madigan_amd import _lib as L
    N, A = 8192, 8
    # TrendOU with frequent, steep trends and 50x leverage: margin calls end
    # episodes every few steps on every part of the grid
    src = trendou_sources(A, [0.2, 2, 6, 0.05, 0.2, 5.0, 0.15, 0.3, 0.2, 0.99])
    kw = dict(required_margin=0.02, maintenance_margin=0.25, slippage_rel=1e-4, transaction_cost_rel=0.02,
              reward_shaper="DDR", adaptation_rate=0.001, unit_size=0.9, auto_reset=1, init_cash=1e5)
    g, orc = make_pair(src, N, seed=0x6D6164 + 3, **kw)
    assert g.lib.mgn_get_schedule(g.h) == L.SCHED_TRIO
    acts = g.generate_actions(5 + 20 + 256, seed=0x6D6164)
    a = acts.cpu().numpy()
    k0 = 0
    for K in (5, 20, 256):
        if K == 20:  # the bench's output set (the O_STD instantiation)
            out = g.alloc_traj(K, fields=STD_FIELDS)
            g.rollout(acts[k0:k0 + K], out)
            o = _host(out)
            ref = orc.rollout(a[k0:k0 + K], threads=THREADS)
            for k in ("obs_price", "obs_port", "tprice", "tunits", "tcost"):
                assert_bits(o[k], ref[k], f"K=20 {k}")
            for k in ("risk", "done", "margin_call"):
                assert np.array_equal(o[k], ref[k]), f"K=20 {k}"
            assert np.array_equal(o["timestamp"].astype(np.uint64), ref["timestamp"])
            close(o["reward"], ref["reward"], "K=20 reward")
            close(o["shaped"], ref["shaped"], "K=20 shaped", rtol=1e-10)
        else:
            o = _host(g.rollout(acts[k0:k0 + K]))
            ref = orc.rollout(a[k0:k0 + K], threads=THREADS)
            out_check(o, ref, f"C3 forced K={K}", shaped_rtol=1e-10)
        ends = int(o["done"].sum())
        assert ends > N // 10, f"K={K}: {ends} episode ends"  # rollbacks all over the grid
        k0 += K
        state_check(g, orc, f"after K={K}")
    gen_state_check(g, orc, "C3 forced")
    # one-step launches (the agent loop's K = 1) on the same grid: an episode
    # that ends at a launch's only step is a tail reset -- the generator's
    # candidate reset tick and the fresh Broker adopted after the loop
    # (mgn_trio.h TAIL) -- checked against the oracle after every launch
    n1 = 24
    acts1 = g.generate_actions(n1, seed=0x6D6164 + 11)
    a1 = acts1.cpu().numpy()
    out1 = g.alloc_traj(1, fields=STD_FIELDS)
    launch = g.rollout_launcher(out1, 1, acts1)
    tail_launches = 0
    for i in range(n1):
        assert launch(i) == 0
        o = _host(out1)
        ref = orc.rollout(a1[i:i + 1], threads=THREADS)
        for k in ("obs_price", "obs_port", "tprice", "tunits", "tcost"):
            assert_bits(o[k], ref[k], f"K=1 launch {i} {k}")
        for k in ("risk", "done", "margin_call"):
            assert np.array_equal(o[k], ref[k]), f"K=1 launch {i} {k}"
        assert np.array_equal(o["timestamp"].astype(np.uint64), ref["timestamp"]), f"K=1 launch {i} ts"
        close(o["reward"], ref["reward"], f"K=1 launch {i} reward")
        close(o["shaped"], ref["shaped"], f"K=1 launch {i} shaped", rtol=1e-10)
        state_check(g, orc, f"after K=1 launch {i}")
        gen_state_check(g, orc, f"after K=1 launch {i}")
        tail_launches += int(o["done"].any())
    assert tail_launches >= n1 - 2, f"only {tail_launches} of {n1} one-step launches ended an episode"
    st = g.episode_stats.cpu().numpy()
    for j, name in enumerate(("last_ret", "last_len", "last_equity", "n_done")):
        close(st[:, j], orc.scalar(name), name)


def test_c3_sliced_launcher_sequence_vs_oracle(gpu):
    """The bench's launch-length sweep on one handle at C3's shape: one-step
    launches through a launcher on [:1] views of a 256-step trajectory, then
    16- and 256-step launches on views of the same trajectory, each on fresh
    rows of one bound action tensor -- every output and the state against the
    oracle.  The launcher refuses action rows outside its tensor (round 4's
    bench fault: a K = 256 launch given a 25-step action buffer read past it)."""
    N, A = 8192, 8
    g, orc = make_pair(trendou_sources(A, [0.001, 100, 500, 0.001, 0.005, 5.0, 0.15, 0.04, 0.001, 0.99]), N,
                       seed=0x6D6164 + 3, required_margin=1.0, maintenance_margin=0.25, slippage_rel=1e-4,
                       transaction_cost_rel=0.02, reward_shaper="DDR", adaptation_rate=0.001,
                       unit_size=0.05, auto_reset=1, init_cash=1_000_000.0)
    T = 512
    acts = g.generate_actions(T, seed=0x6D6165)
    a = acts.cpu().numpy()
    big = g.alloc_traj(256, fields=STD_FIELDS)
    row = 0
    for K, n in ((1, 6), (16, 2), (256, 1)):
        view = {k: v[:K] for k, v in big.items()}
        launch = g.rollout_launcher(view, K, acts)
        with pytest.raises(IndexError):
            launch(T - K + 1)
        with pytest.raises(IndexError):
            launch(-1)
        for i in range(n):
            assert launch(row) == 0
            o = _host(view)
            ref = orc.rollout(a[row:row + K], threads=THREADS)
            out_check({**o, "agent_reward": ref["agent_reward"]}, ref, f"K={K} launch {i}")
            state_check(g, orc, f"K={K} launch {i}")
            row += K
    gen_state_check(g, orc, "sliced launcher")
    with pytest.raises(ValueError):
        g.rollout_launcher({k: v[:256] for k, v in big.items()}, 256, acts[:25])


def test_sixteen_assets_ou_window64_two_slots_vs_oracle(gpu):
    """16 OU assets with a W = 64 window at 4096 envs: the three-role kernel's
    two-slots-per-lane layout (trio_m2_ok: 4096 x 16 lanes) -- the automatic
    schedule since round 4 -- against the oracle: every output and every
    step's window over two 32-step launches, with a leveraged broker ending
    episodes inside them (the refill rows after each auto-reset)."""
    from madigan_amd import _lib as L
    from tests.test_gpu_configs import _check_windows
    N, A, W, K = 4096, 16, 64, 32
    g, orc = make_pair(ou_sources(A), N, seed=0x6D6164 + 12, required_margin=0.02, maintenance_margin=0.25,
                       slippage_rel=1e-4, transaction_cost_rel=0.02, unit_size=0.9, auto_reset=1,
                       init_cash=1e5, window=W, adaptation_rate=0.001, reward_shaper="DDR")
    assert g.lib.mgn_get_schedule(g.h) == L.SCHED_TRIO
    acts = g.generate_actions(2 * K, seed=0x6D6164 + 13)
    _check_windows(g, orc, acts[:K], K, None, "A16 W64 launch 0")
    _check_windows(g, orc, acts[K:], K, None, "A16 W64 launch 1")
    state_check(g, orc, "A16 W64")
    st = g.episode_stats.cpu().numpy()
    assert st[:, 3].sum() > N // 10, "too few episode ends"
    close(st[:, 3], orc.scalar("n_done"), "n_done")


@pytest.mark.parametrize("sched", ["auto", "duo"])
def test_c5_bench_shape_windows(gpu, tmp_path, sched):
    import torch
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    from madigan_amd import BatchedEnv
    from madigan_amd.config import spec_from_config
    N, A, T, W, K = 8192, 16, 200_000, 64, 64
    path = str(tmp_path / "c5.h5")
    bench.c5_replay_file(A, T, path)
    price, ts = bench.c5_paths(A, T)
    cfg = {"data_source_type": "HDFSourceSingle",
           "data_source_config": {"filepath": path, "group_key": "synth/ou", "price_key": "price",
                                  "feature_key": "features", "timestamp_key": "timestamps",
                                  "cache_size": 10_000}}
    kw = dict(required_margin=1.0, maintenance_margin=0.25, transaction_cost_rel=0.02, unit_size=0.05,
              auto_reset=True, init_cash=1_000_000.0, window=W, adaptation_rate=0.001,
              reward_shaper="DDR", seed=0x6D6164 + 5)
    g = BatchedEnv(spec_from_config(cfg), N, device=gpu, replay_stride=997, **kw)
    from madigan_amd import _lib as L
    if sched == "duo":  # the two-role kernel (explicit); auto: the three-role kernel
        L.check(g.lib.mgn_set_schedule(g.h, L.SCHED_DUO), g.h)
    assert g.lib.mgn_get_schedule(g.h) == (L.SCHED_DUO if sched == "duo" else L.SCHED_TRIO)
    first, second, _, _ = O.hdf_bounds(ts, 0, 0)
    orc = O.OracleBatch(dict(kw, n_envs=N, n_feats=A, auto_reset=1), [(O.SRC_REPLAY, [])] * A)
    assert orc.set_replay(price, price, ts, first, second, 10_000, 997) == g._tape["ts"].shape[0]
    # C5's first episodes end after a few hundred steps (the 2 % cost drains
    # equity below 0.1 initCash): launches run until two launches with episode
    # ends have been checked; every output of every step is checked, and every
    # step's window in the first launch and from the first launch with resets on
    MAXL = 16
    acts = g.generate_actions(MAXL * K, seed=0x6D6164)
    a = acts.cpu().numpy()
    dones, checked = [], 0
    for launch in range(MAXL):  # each launch starts from the previous one's ring
        out, (wp, wo, wt) = g.rollout_window(acts[launch * K:(launch + 1) * K], per_step=True)
        torch.cuda.synchronize()
        windows = launch == 0 or any(dones)
        d = 0
        for k in range(K):
            r = orc.rollout(a[launch * K + k:launch * K + k + 1], threads=THREADS)
            tag = f"C5 launch {launch} step {k}"
            for f in ("obs_price", "obs_port", "tprice", "tunits", "tcost"):
                assert_bits(out[f][k].cpu().numpy(), r[f][0], f"{tag} {f}")
            for f in ("risk", "done", "margin_call", "data_end"):
                assert np.array_equal(out[f][k].cpu().numpy(), r[f][0]), f"{tag} {f}"
            close(out["reward"][k].cpu().numpy(), r["reward"][0], f"{tag} reward")
            close(out["shaped"][k].cpu().numpy(), r["shaped"][0], f"{tag} shaped", rtol=1e-10)
            d += int(r["done"].sum())
            if windows or d:
                rpr, rpo, rts = orc.window()
                assert_bits(wp[k].cpu().numpy(), rpr, f"{tag} window price")
                assert_bits(wo[k].cpu().numpy(), rpo, f"{tag} window portfolio")
                assert np.array_equal(wt[k].cpu().numpy().astype(np.uint64), rts), f"{tag} window ts"
        dones.append(d)
        del out, wp, wo, wt
        checked += 1 if d and any(dones[:-1]) else 0
        if checked >= 1 and sum(1 for x in dones if x) >= 2:
            break
    assert sum(1 for x in dones if x) >= 2, dones
    state_check(g, orc, "C5 end")
