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
from tests.configs import trendou_sources
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
    st = g.episode_stats.cpu().numpy()
    for j, name in enumerate(("last_ret", "last_len", "last_equity", "n_done")):
        close(st[:, j], orc.scalar(name), name)


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
