"""The reference's own experiment shape ("What's missing" 2): one
OU asset (mean 10, theta .08, phi .04), a W = 64 StackerDiscrete window
(norm false: raw prices), n = 20 step returns (discount .99) over the summed
agent reward (reduce_rewards), DDR (eta .001) or sortino_shaperB (exp 1.1),
2 % transaction cost, unit .05 of the available margin, discrete actions
(scripts/ou_ddr_.001_nstep20.yaml:27,280,286; ou_sortinoB_exp_1.1_nstep20.yaml).

A one-asset env runs on the three-role kernel with two lanes per env and role
(ONE: the second lane a pad; the env's sums are lane 0's one leaf) -- n-step
rings, the window and the naive shaper in its finish role.  Against the
oracle at the bench's batch: every output, the n-step rows and every step's
window of 64-step launches with auto-resets inside them."""
import numpy as np
import pytest

from tests.configs import ou_sources
from tests.test_gpu_parity import assert_bits, close, make_pair, state_check

pytestmark = pytest.mark.gpu
THREADS = 8

REF_KW = dict(required_margin=1.0, maintenance_margin=0.25, transaction_cost_rel=0.02, unit_size=0.05,
              auto_reset=1, init_cash=1_000_000.0, window=64, adaptation_rate=0.001, nstep_return=20,
              discount=0.99, reward_mode="agent_sum")


# the bench's output set for the windowed workloads (bench.py windowed(): the
# agent loop's State / EnvInfo, data_end and the popped counts), which the
# one-asset OU n-step window handles instantiate with the set at compile time
BENCH_FIELDS = ["reward", "shaped", "done", "obs_price", "obs_port", "timestamp", "tprice", "tunits", "tcost",
                "risk", "margin_call", "data_end", "n_shaped"]


def _launch_vs_oracle(g, orc, acts, tag, shaped_rtol, fields=None, atol=1e-14):
    import ctypes as C
    import torch
    from madigan_amd import _lib as L
    K, N, W, A, F = acts.shape[0], g.N, g.W, g.A, g.F
    traj = g.alloc_traj(K, fields=fields)
    wp = torch.empty((K, N, W, F), dtype=torch.float64, device=g.device)
    wo = torch.empty((K, N, W, A + 1), dtype=torch.float64, device=g.device)
    wt = torch.empty((K, N, W), dtype=torch.int64, device=g.device)
    t = g._traj_struct(traj)
    L.check(g.lib.mgn_rollout_hist(g.h, C.c_void_p(acts.data_ptr()), K, C.byref(t)), g.h)
    L.check(g.lib.mgn_window_hist(g.h, *[C.c_void_p(x.data_ptr()) for x in (wp, wo, wt)]), g.h)
    torch.cuda.synchronize()
    a = acts.cpu().numpy()
    host = {k: v.cpu().numpy() for k, v in traj.items()}
    ends = 0
    for k in range(K):
        r = orc.rollout(a[k:k + 1], threads=THREADS)
        for f in ("obs_price", "obs_port", "tprice", "tunits", "tcost"):
            assert_bits(host[f][k], r[f][0], f"{tag} {f} step {k}")
        for f in ("risk", "done", "margin_call", "n_shaped"):
            assert np.array_equal(host[f][k], r[f][0]), f"{tag} {f} step {k}"
        close(host["reward"][k], r["reward"][0], f"{tag} reward step {k}")
        if "agent_reward" in host:
            close(host["agent_reward"][k], r["agent_reward"][0], f"{tag} agent reward step {k}")
        np.testing.assert_allclose(host["shaped"][k], r["shaped"][0], rtol=shaped_rtol, atol=atol,
                                   err_msg=f"{tag} n-step row step {k}")
        rpr, rpo, rts = orc.window()
        assert_bits(wp[k].cpu().numpy(), rpr, f"{tag} window price step {k}")
        assert_bits(wo[k].cpu().numpy(), rpo, f"{tag} window portfolio step {k}")
        assert np.array_equal(wt[k].cpu().numpy().astype(np.uint64), rts), f"{tag} window ts step {k}"
        ends += int(r["done"].sum())
    return ends


@pytest.mark.parametrize("N,shaper,extra,rtol", [
    (8192, "DDR", {}, 1e-10),
    (8192, "sortino_shaperB", dict(sortino_exp=1.1), 1e-10),
    (65536, "DDR", {}, 1e-10),
    (2048, "sortino_shaperB", dict(sortino_exp=1.5), 1e-10),
])
def test_reference_shape_vs_oracle(gpu, N, shaper, extra, rtol):
    from madigan_amd import _lib as L
    # (a leveraged variant ends episodes inside the launches: margin calls)
    kw = dict(REF_KW, reward_shaper=shaper, **extra, seed=0x6D6164 + 21)
    kw.update(required_margin=0.05, unit_size=0.9)
    g, orc = make_pair(ou_sources(1), N, **kw)
    # (beyond 16384 one-asset window envs the automatic schedule takes the
    # single-role kernel, measured faster there)
    assert g.lib.mgn_get_schedule(g.h) == (L.SCHED_TRIO if N <= 16384 else L.SCHED_SINGLE)
    K = 64 if N <= 8192 else 24
    acts = g.generate_actions(2 * K, seed=0x6D6164 + 22)
    ends = _launch_vs_oracle(g, orc, acts[:K], f"{shaper} N={N} launch 0", rtol)
    ends += _launch_vs_oracle(g, orc, acts[K:], f"{shaper} N={N} launch 1", rtol)
    assert ends > N // 20, f"{ends} episode ends"
    state_check(g, orc, f"{shaper} N={N}")
    close(g.shaper_a.cpu().numpy(), orc.scalar("shaperA"), "A")
    close(g.shaper_b.cpu().numpy(), orc.scalar("shaperB"), "B")
    # a units step on the same handle (no three-role instantiation: another
    # kernel, the same state) and a discrete launch after it
    u = np.random.default_rng(5).normal(0, 2e3, (N, 1))
    g.step(u)
    ref = orc.step(u)
    o = g.host_outputs()
    assert_bits(o["tunits"], ref["tunits"], "units step tunits")
    acts2 = g.generate_actions(8, seed=0x6D6164 + 23)
    _launch_vs_oracle(g, orc, acts2, f"{shaper} N={N} after units", rtol)
    state_check(g, orc, f"{shaper} N={N} end")


@pytest.mark.parametrize("shaper,extra", [("DDR", {}), ("sortino_shaperB", dict(sortino_exp=1.1))])
def test_reference_shape_bench_outputs_vs_oracle(gpu, shaper, extra):
    """The bench's output set (BENCH_FIELDS) at 8192 envs: the instantiation
    with that set and the OU generator at compile time
    (mgn_launch_impl.h launch_trio_one_impl) against the oracle, every
    output, n-step row and window of two 64-step launches with auto-resets."""
    kw = dict(REF_KW, reward_shaper=shaper, **extra, seed=0x6D6164 + 31)
    kw.update(required_margin=0.05, unit_size=0.9)
    g, orc = make_pair(ou_sources(1), 8192, **kw)
    K = 64
    acts = g.generate_actions(2 * K, seed=0x6D6164 + 32)
    ends = _launch_vs_oracle(g, orc, acts[:K], f"{shaper} bench set launch 0", 1e-10, BENCH_FIELDS)
    ends += _launch_vs_oracle(g, orc, acts[K:], f"{shaper} bench set launch 1", 1e-10, BENCH_FIELDS)
    assert ends > 8192 // 20, f"{ends} episode ends"


@pytest.mark.parametrize("shaper,extra", [("DDR", {}), ("sortino_shaperB", dict(sortino_exp=1.1))])
def test_reference_shape_trio_equals_single_bitwise(gpu, shaper, extra):
    """At the bench's batch (8192 envs) the ONE layout's outputs -- the n-step
    rows (`shaped`) included, which the oracle tests hold to rtol 1e-10 --
    and every step's window equal the single-role kernel's bit for bit, over
    two 64-step launches with auto-resets (the same pop summands in the same
    order on both kernels)."""
    import ctypes as C
    import torch
    from madigan_amd import BatchedEnv
    from madigan_amd import _lib as L
    from tests.configs import spec_from_sources
    kw = dict(REF_KW, reward_shaper=shaper, **extra, seed=0x6D6164 + 51)
    kw.update(required_margin=0.05, unit_size=0.9)
    res = []
    for sched in (L.SCHED_TRIO, L.SCHED_SINGLE):
        g = BatchedEnv(spec_from_sources(ou_sources(1)), 8192, **kw)
        L.check(g.lib.mgn_set_schedule(g.h, sched), g.h)
        acts = g.generate_actions(128, seed=0x6D6164 + 52)
        outs = []
        for half in range(2):
            K = 64
            traj = g.alloc_traj(K)
            wp = torch.empty((K, g.N, g.W, g.F), dtype=torch.float64, device=g.device)
            wo = torch.empty((K, g.N, g.W, g.A + 1), dtype=torch.float64, device=g.device)
            wt = torch.empty((K, g.N, g.W), dtype=torch.int64, device=g.device)
            t = g._traj_struct(traj)
            a = acts[half * K:(half + 1) * K]
            L.check(g.lib.mgn_rollout_hist(g.h, C.c_void_p(a.data_ptr()), K, C.byref(t)), g.h)
            L.check(g.lib.mgn_window_hist(g.h, *[C.c_void_p(x.data_ptr()) for x in (wp, wo, wt)]), g.h)
            o = {k: v.cpu().numpy() for k, v in traj.items()}
            o.update(win_price=wp.cpu().numpy(), win_port=wo.cpu().numpy(), win_ts=wt.cpu().numpy())
            outs.append(o)
        assert g.lib.mgn_get_schedule(g.h) == sched
        res.append(outs)
    ends = 0
    for half, (a, b) in enumerate(zip(*res)):
        for k, v in a.items():
            if v.dtype == np.float64:
                assert_bits(b[k], v, f"{shaper} launch {half} trio vs single {k}")
            else:
                assert np.array_equal(b[k], v), f"{shaper} launch {half} trio vs single {k}"
        ends += int(a["done"].sum())
    assert ends > 8192 // 20
