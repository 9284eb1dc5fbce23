"""BASELINE.json configs at their benchmarked shapes, end to end on the GPU
against the oracle:

  C3  8192 envs x 8 TrendOU (config.yaml:116-138), slippage 1e-4 + 2 % cost,
      DDR, discrete actions, auto-reset: the bench's launch sequence (a 5-step
      warm launch, a 20-step launch, a 256-step launch), every output of every
      step and the final state bit-exact;
  C2  4096 envs x 4 OU, W = 64 window (norm none), DSR: every step's window
      of a 16-step launch (mgn_rollout_hist / mgn_window_hist, as bench.py);
  C4  Composite Synth(2) + OU(3) + TrendOU(3), W = 64 log window, PPC over the
      env log reward, the bench's 64-step windowed launches;
plus the automatic layout at a large batch that is not a multiple of the
two-role kernel's envs per workgroup (32768 + 17 envs), against the
single-role kernel at the layout the old rule picked.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.configs import TRENDOU_P, composite_sources, ou_sources, trendou_sources
from tests.test_gpu_parity import (assert_bits, close, gen_state_check, make_pair, out_check,
                                   state_check)

pytestmark = pytest.mark.gpu

C3_KW = dict(required_margin=1.0, maintenance_margin=0.25, slippage_rel=1e-4,
             transaction_cost_rel=0.02, reward_shaper="DDR", adaptation_rate=0.001, unit_size=0.05,
             auto_reset=1, init_cash=1_000_000.0)
THREADS = 8


def _host(out):
    return {k: v.cpu().numpy() for k, v in out.items()}


def test_c3_bench_shape_launches(gpu):
    N, A = 8192, 8
    g, orc = make_pair(trendou_sources(A, TRENDOU_P), N, seed=0x6D6164 + 3, **C3_KW)
    acts = g.generate_actions(5 + 20 + 256, seed=0x6D6164)
    a = acts.cpu().numpy()
    k0 = 0
    for K in (5, 20, 256):
        out = _host(g.rollout(acts[k0:k0 + K]))
        ref = orc.rollout(a[k0:k0 + K], threads=THREADS)
        out_check(out, ref, f"C3 K={K}")
        k0 += K
        state_check(g, orc, f"C3 after K={K}")
    gen_state_check(g, orc, "C3")
    close(g.shaper_a.cpu().numpy(), orc.scalar("shaperA"), "DDR A")
    close(g.shaper_b.cpu().numpy(), orc.scalar("shaperB"), "DDR B")
    st = g.episode_stats.cpu().numpy()
    for j, name in enumerate(("last_ret", "last_len", "last_equity", "n_done")):
        close(st[:, j], orc.scalar(name), name)


STD_FIELDS = ("reward", "shaped", "done", "obs_price", "obs_port", "timestamp", "tprice", "tunits",
              "tcost", "risk", "margin_call")


@pytest.mark.parametrize("fields,misalign", [
    ("std", False),     # the agent loop's / bench's output set: the fixed-set instantiation
    ("all", False),     # every field: the fixed-set instantiation
    ("std", True),      # the same set in buffers offset by one element
    ("subset", False),  # no timestamps / costs: the runtime-mask instantiation
])
def test_c3_output_sets(gpu, fields, misalign):
    """Every output set the three-role kernel serves, at the bench shape
    (8192 x 8, 20-step launches), bit-exact against the oracle for every field
    present (mgn_trio.h instantiates the kernel per fixed output set, with
    the runtime-mask kernel for every other set)."""
    import torch
    N, A, K = 8192, 8, 20
    g, orc = make_pair(trendou_sources(A, TRENDOU_P), N, seed=0x6D6164 + 3, **C3_KW)
    acts = g.generate_actions(2 * K, seed=0x6D6164)
    names = {"std": STD_FIELDS, "all": None,
             "subset": ("reward", "shaped", "done", "obs_price", "obs_port", "tprice", "tunits", "risk")}[fields]
    for rep in range(2):
        traj = g.alloc_traj(K, fields=names)
        if misalign:  # the same fields, each one element into a larger buffer
            shp = g._traj_shapes(K)
            traj = {k: torch.empty(v.numel() + 1, dtype=v.dtype, device=v.device)[1:].view(shp[k][0])
                    for k, v in traj.items()}
        out = _host(g.rollout(acts[rep * K:(rep + 1) * K], out=traj))
        ref = orc.rollout(acts[rep * K:(rep + 1) * K].cpu().numpy(), threads=THREADS)
        for f, v in out.items():
            if v.dtype == np.float64 and f not in ("reward", "shaped", "agent_reward"):
                assert_bits(v, ref[f], f"{fields} {f} launch {rep}")
            elif f in ("reward", "shaped", "agent_reward"):
                close(v, ref[f], f"{fields} {f} launch {rep}")
            else:
                assert np.array_equal(v.astype(np.uint64) if f == "timestamp" else v,
                                      ref[f]), f"{fields} {f} launch {rep}"
    state_check(g, orc, f"C3 {fields}")


def _windowed_pair(sources, N, W, norm, shaper, **kw):
    base = dict(required_margin=1.0, maintenance_margin=0.25, transaction_cost_rel=0.02,
                unit_size=0.05, auto_reset=1, init_cash=1_000_000.0, window=W, norm_type=norm,
                adaptation_rate=0.001, reward_shaper=shaper)
    base.update(kw)
    g, orc = make_pair(sources, N, **base)
    return g, orc


def _check_windows(g, orc, acts, K, norm, tag):
    import ctypes as C
    import torch
    from madigan_amd import _lib as L
    N, W, A, F = g.N, g.W, g.A, g.F
    traj = g.alloc_traj(K)
    wp = torch.empty((K, N, W, F), dtype=torch.float64, device=g.device)
    wo = torch.empty((K, N, W, A + 1), dtype=torch.float64, device=g.device)
    wt = torch.empty((K, N, W), dtype=torch.int64, device=g.device)
    t = g._traj_struct(traj)
    L.check(g.lib.mgn_rollout_hist(g.h, C.c_void_p(acts.data_ptr()), K, C.byref(t)), g.h)
    L.check(g.lib.mgn_window_hist(g.h, *[C.c_void_p(x.data_ptr()) for x in (wp, wo, wt)]), g.h)
    a = acts.cpu().numpy()
    host = _host(traj)
    for k in range(K):
        r = orc.rollout(a[k:k + 1], threads=THREADS)
        for f in ("obs_price", "obs_port", "tunits", "tcost", "risk", "done"):
            if host[f].dtype == np.float64:
                assert_bits(host[f][k], r[f][0], f"{tag} {f} step {k}")
            else:
                assert np.array_equal(host[f][k], r[f][0]), f"{tag} {f} step {k}"
        close(host["reward"][k], r["reward"][0], f"{tag} reward step {k}")
        close(host["shaped"][k], r["shaped"][0], f"{tag} shaped step {k}")
        rpr, rpo, rts = orc.window()
        if norm is None:
            assert_bits(wp[k].cpu().numpy(), rpr, f"{tag} window price step {k}")
        else:
            close(wp[k].cpu().numpy(), rpr, f"{tag} window price step {k}")
        assert_bits(wo[k].cpu().numpy(), rpo, f"{tag} window portfolio step {k}")
        assert np.array_equal(wt[k].cpu().numpy().astype(np.uint64), rts), f"{tag} window ts {k}"


def test_c2_window64_4096(gpu):
    N, A, W, K = 4096, 4, 64, 16
    g, orc = _windowed_pair(ou_sources(A), N, W, None, "DSR", seed=0x6D6164 + 2)
    acts = g.generate_actions(2 * K, seed=0x6D6164)
    _check_windows(g, orc, acts[:K], K, None, "C2 launch 0")
    _check_windows(g, orc, acts[K:], K, None, "C2 launch 1")
    state_check(g, orc, "C2")


@pytest.mark.parametrize("N", [2048, 8192])
def test_c4_composite_ppc_log_window(gpu, N):
    """2048 envs run the three-role kernel at one wave per role, 8192 (the
    bench shape) at 256 lanes per role."""
    from madigan_amd import _lib as L
    W, K = 64, 64
    src = composite_sources()
    A = len(src)
    g, orc = _windowed_pair(src, N, W, "log", "PPC", cosine_temp=0.01,
                            desired_portfolio=[1.0] + [0.0] * A, seed=0x6D6164 + 4)
    assert g.lib.mgn_get_schedule(g.h) == L.SCHED_TRIO
    acts = g.generate_actions(K, seed=0x6D6164)
    _check_windows(g, orc, acts, K, "log", "C4")
    state_check(g, orc, "C4")
    gen_state_check(g, orc, "C4")


def test_large_batch_auto_layout_tail_block(gpu):
    """the automatic layout runs a multi-role kernel at large N
    (k_step_trio here, k_step_duo where the three-role one is not eligible);
    32768 + 17 envs (a partial last workgroup), auto-reset forced by high
    leverage, against k_step at 4 assets per lane bit for bit."""
    from madigan_amd import BatchedEnv
    from madigan_amd import _lib as L
    from tests.configs import spec_from_sources
    N, A, K = 32768 + 17, 8, 12
    spec = spec_from_sources(trendou_sources(A, [0.2, 2, 6, 0.05, 0.2, 5.0, 0.15, 0.3, 0.2, 0.99]))
    kw = dict(required_margin=0.02, maintenance_margin=0.25, transaction_cost_rel=0.02,
              slippage_rel=1e-4, unit_size=0.9, auto_reset=True, init_cash=1e5, seed=31,
              reward_shaper="DDR")
    res = []
    for mode in ("auto", "single4"):
        g = BatchedEnv(spec, N, **kw)
        if mode == "auto":
            assert g.lib.mgn_get_schedule(g.h) in (L.SCHED_DUO, L.SCHED_TRIO)
        else:
            L.check(g.lib.mgn_set_schedule(g.h, L.SCHED_SINGLE), g.h)
            L.check(g.lib.mgn_set_layout(g.h, 4), g.h)
            assert g.lib.mgn_get_layout(g.h) == 4
        acts = g.generate_actions(K, seed=5)
        out = _host(g.rollout(acts))
        out["ledger"] = g.ledger.cpu().numpy()
        out["cash"] = g.cash.cpu().numpy()
        out["stats"] = g.episode_stats.cpu().numpy()
        res.append(out)
    assert res[0]["done"].sum() > 0
    for k, v in res[0].items():
        if v.dtype == np.float64:
            assert_bits(res[1][k], v, f"auto vs single {k}")
        else:
            assert np.array_equal(res[1][k], v), k


def test_state_dict_resume_bit_exact(gpu):
    """Checkpoint / resume: save mid-run, run on, restore into a
    fresh handle, run the same actions: identical to the uninterrupted run and
    to the oracle (windowed DSR env with auto-resets)."""
    from madigan_amd import BatchedEnv
    from tests.configs import spec_from_sources
    N, A, W, K = 300, 4, 8, 24
    kw = dict(required_margin=0.02, maintenance_margin=0.25, transaction_cost_rel=0.02,
              unit_size=0.9, auto_reset=1, init_cash=1e5, reward_shaper="DSR", window=W, seed=12)
    src = trendou_sources(A, [0.2, 2, 6, 0.05, 0.2, 5.0, 0.15, 0.3, 0.2, 0.99])
    g, orc = make_pair(src, N, **kw)
    acts = g.generate_actions(2 * K, seed=3)
    g.rollout(acts[:K])
    orc.rollout(acts[:K].cpu().numpy())
    sd = g.state_dict()
    o1 = _host(g.rollout(acts[K:]))
    h = BatchedEnv(spec_from_sources(src), N, **{k: v for k, v in kw.items() if k != "seed"},
                   seed=999)
    h.load_state_dict(sd)
    o2 = _host(h.rollout(acts[K:]))
    ref = orc.rollout(acts[K:].cpu().numpy())
    assert ref["done"].sum() > 0
    for k in o1:
        if o1[k].dtype == np.float64:
            assert_bits(o2[k], o1[k], f"resume {k}")
        else:
            assert np.array_equal(o2[k], o1[k]), k
    out_check(o2, ref, "resume vs oracle")
    state_check(h, orc, "resume")
    with pytest.raises(ValueError):
        BatchedEnv(spec_from_sources(src), N + 1, **kw).load_state_dict(sd)


def test_stats_allgather_rccl_single_rank(gpu):
    """mgn_stats_allgather over torch's RCCL communicator (world size 1 on the
    one leased GPU): the gathered table equals the handle's statistics, padded
    rows are zero."""
    import os
    import torch
    import torch.distributed as dist
    from madigan_amd.distributed import allgather_env_stats, rccl_comm
    from madigan_amd import _lib as L
    import ctypes as C
    N, A, K = 200, 4, 40
    kw = dict(required_margin=0.02, maintenance_margin=0.25, transaction_cost_rel=0.02,
              unit_size=0.9, auto_reset=1, init_cash=1e5)
    g, _ = make_pair(trendou_sources(A, [0.2, 2, 6, 0.05, 0.2, 5.0, 0.15, 0.3, 0.2, 0.99]), N, **kw)
    g.rollout(g.generate_actions(K, seed=2))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29400 + os.getpid() % 500))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=g.device)
    try:
        assert rccl_comm(device=g.device) != 0
        got = allgather_env_stats(g, n_total=N)
        from madigan_amd import distributed as D
        assert D.last_allgather_path == "mgn_stats_allgather"
        torch.cuda.synchronize()
        ref = g.episode_stats.cpu().numpy()
        assert ref[:, 3].sum() > 0
        assert_bits(got.cpu().numpy(), ref, "allgather")
        out = torch.full((N + 9, 4), 7.0, dtype=torch.float64, device=g.device)
        L.check(g.lib.mgn_stats_allgather(g.h, C.c_void_p(rccl_comm(device=g.device)), N + 9,
                                          C.c_void_p(out.data_ptr())), g.h)
        torch.cuda.synchronize()
        o = out.cpu().numpy()
        assert_bits(o[:N], ref, "padded allgather")
        assert not o[N:].any()
        with pytest.raises(ValueError):
            L.check(g.lib.mgn_stats_allgather(g.h, C.c_void_p(rccl_comm(device=g.device)), N - 1,
                                              C.c_void_p(out.data_ptr())), g.h)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("binding", ["pycall", "ctypes"])
def test_rollout_launcher_matches_rollout(gpu, binding, monkeypatch):
    """BatchedEnv.rollout_launcher (bench.py's timed loop) through the CPython
    binding and through ctypes: the same launches as rollout() into the same
    output buffers, bit-exact against the oracle (C3 shape, 1- and 20-step);
    the stream waits (polling and plain) through the same binding."""
    from madigan_amd import _lib as L
    if binding == "ctypes":
        monkeypatch.setattr(L, "pycall", lambda: None)
    elif os.environ.get("MADIGAN_LIB_PATH"):
        pytest.skip("another library build is loaded (MADIGAN_LIB_PATH): the binding links the in-tree one")
    else:
        assert L.pycall() is not None, "_mgn_pycall not built"
    N, A = 8192, 8
    g, orc = make_pair(trendou_sources(A, TRENDOU_P), N, seed=0x6D6164 + 5, **C3_KW)
    acts = g.generate_actions(1 + 20, seed=0x6D6164)
    a = acts.cpu().numpy()
    k0 = 0
    for K in (1, 20):
        out = g.alloc_traj(K, fields=list(STD_FIELDS))
        launch = g.rollout_launcher(out, K)
        assert launch(acts[k0:k0 + K].data_ptr()) == 0
        # the handle's stream waits (the one-step launch's by polling it,
        # mgn_synchronize_spin; then the plain one on an idle stream)
        assert g.stream_synchronizer(spin=(K == 1))() == 0
        assert g.stream_synchronizer(spin=(K != 1))() == 0
        ref = orc.rollout(a[k0:k0 + K], threads=THREADS)
        o = _host(out)
        for f in ("obs_price", "obs_port", "tprice", "tunits", "tcost"):
            assert_bits(o[f], ref[f], f"launcher {binding} K={K} {f}")
        for f in ("risk", "done", "margin_call"):
            assert np.array_equal(o[f], ref[f]), f"launcher {binding} K={K} {f}"
        assert np.array_equal(o["timestamp"].astype(np.uint64), ref["timestamp"])
        close(o["reward"], ref["reward"], f"launcher {binding} K={K} reward")
        close(o["shaped"], ref["shaped"], f"launcher {binding} K={K} shaped")
        k0 += K
    state_check(g, orc, f"launcher {binding}")


@pytest.mark.parametrize("N", [2048, 4096])
def test_sixteen_assets_auto_schedule_vs_oracle(gpu, N):
    """16 TrendOU assets at the automatic schedule (the three-role kernel since
    round 3; at 4096 envs its two-slots-per-lane layout, launch_trio_m2), 20-
    and 64-step launches against the oracle: every output and the final state."""
    from madigan_amd import _lib as L
    A = 16
    g, orc = make_pair(trendou_sources(A, TRENDOU_P), N, seed=0x6D6164 + 7, **C3_KW)
    assert g.lib.mgn_get_schedule(g.h) == L.SCHED_TRIO
    acts = g.generate_actions(20 + 64, seed=0x6D6164)
    a = acts.cpu().numpy()
    k0 = 0
    for K in (20, 64):
        out = _host(g.rollout(acts[k0:k0 + K]))
        ref = orc.rollout(a[k0:k0 + K], threads=THREADS)
        out_check(out, ref, f"A16 K={K}")
        k0 += K
        state_check(g, orc, f"A16 after K={K}")
    gen_state_check(g, orc, "A16")
