"""The running-sum n-step pop on the GPU (MGN_NSTEP_POP_RUNNING: the
three-role kernel's NST == 2 instantiations, csrc/mgn_trio.h NRUN) against the
oracle's exact pop (nstep_buffer.py:62-91 DSR, :128-162 DDR, :182-204 PPC,
:23-27 none): every popped value within north_star's 1e-6 relative, over
>= 1e4 steps with done flushes, clip saturation and the A = B = 0 start
(the EPS-dominated denominators); everything else -- ledger, State,
responses, done, the popped counts, the shaper state A / B -- exactly as the
exact pop leaves it (the running pop changes only how a pop is summed)."""
import numpy as np
import pytest

from tests.configs import ou_sources, spec_from_sources, trendou_sources
from tests.test_gpu_parity import assert_bits, close, make_pair, state_check
from tests.test_gpu_reference_shape import REF_KW, _launch_vs_oracle

pytestmark = pytest.mark.gpu

RTOL, ATOL = 1e-6, 1e-10
TOU = [0.2, 2, 6, 0.05, 0.2, 5.0, 0.15, 0.3, 0.2, 0.99]
STD = ["reward", "shaped", "done", "obs_price", "obs_port", "timestamp", "tprice", "tunits", "tcost", "risk",
       "margin_call", "n_shaped"]


def _check_launch(host, ref, tag):
    for k, v in host.items():
        if k == "shaped":
            continue
        if k == "reward":
            close(v, ref[k], f"{tag} {k}")
        elif k == "timestamp":
            assert np.array_equal(v.astype(np.uint64), ref[k]), tag
        elif v.dtype == np.float64:
            assert_bits(v, ref[k], f"{tag} {k}")
        else:
            assert np.array_equal(v, np.asarray(ref[k]).astype(v.dtype)), f"{tag} {k}"
    np.testing.assert_allclose(host["shaped"], ref["shaped"], rtol=RTOL, atol=ATOL, err_msg=f"{tag} shaped")


@pytest.mark.parametrize("A,N,src,shaper,n,gamma,launches", [
    # the n = 20 DDR bench shape (256-lane TrendOU agent-loop instantiation,
    # O_STDN), 20-step launches then 256-step launches (re-sums inside them)
    (8, 8192, "trendou", "DDR", 20, 0.99, [20] * 6 + [256] * 4),
    # one wave per role (the 64-lane layout), OU, DSR: >= 1e4 steps
    (4, 512, "ou", "DSR", 5, 0.9, [256] * 40),
    (2, 1024, "trendou", "PPC", 20, 0.97, [64] * 20),
    (8, 512, "trendou", None, 16, 0.99, [256] * 8),
    # sortino_shaperB's running form (one wave per role): exp 1.1 and 3
    (4, 512, "ou", "sortino_shaperB", 20, 0.99, [256] * 8),
    (2, 1024, "trendou", "sortino_shaperB3", 12, 0.95, [64] * 20),
])
def test_running_pop_vs_oracle(gpu, A, N, src, shaper, n, gamma, launches):
    from madigan_amd import _lib as L
    kw = dict(required_margin=0.02, maintenance_margin=0.25, transaction_cost_rel=0.02, unit_size=0.9,
              auto_reset=1, init_cash=1e5, reward_shaper=shaper, adaptation_rate=0.01, nstep_return=n,
              discount=gamma, seed=0x6E7275 + A)
    if shaper == "PPC":
        kw.update(cosine_temp=0.05, desired_portfolio=[0.5] + [0.5 / A] * A)
    if shaper and shaper.startswith("sortino_shaperB"):
        kw.update(reward_shaper="sortino_shaperB", sortino_exp=3.0 if shaper.endswith("3") else 1.1)
    sources = trendou_sources(A, TOU) if src == "trendou" else ou_sources(A)
    g, orc = make_pair(sources, N, nstep_pop="running", **kw)
    L.check(g.lib.mgn_set_schedule(g.h, L.SCHED_TRIO), g.h)
    acts = g.generate_actions(sum(launches), seed=0x6E7276)
    k0, ends, sat, diff = 0, 0, 0, 0
    for i, K in enumerate(launches):
        a = acts[k0:k0 + K]
        k0 += K
        o = g.alloc_traj(K, fields=STD)
        g.rollout(a, o)
        host = {k: v.cpu().numpy() for k, v in o.items()}
        ref = orc.rollout(a.cpu().numpy(), threads=8)
        _check_launch(host, ref, f"{shaper} n={n} A{A} launch {i}")
        ends += int(host["done"].sum())
        sat += int((np.abs(ref["shaped"]) == 1.0).sum())
        diff += int((bits_of(host["shaped"]) != bits_of(ref["shaped"])).sum())
        state_check(g, orc, f"{shaper} launch {i}")
    assert N * k0 >= 1e6  # (the OU DSR case: 10240 steps)
    assert ends > 0 and int(ref["n_shaped"].max()) > 1, "done flushes"
    if shaper in ("DSR", "DDR") or (shaper or "").startswith("sortino"):
        assert sat > 0, "clip saturation"
    # the running pop sums differently: its values are not the exact pop's bits
    assert diff > 0, "the running-sum kernel ran"
    close(g.shaper_a.cpu().numpy(), orc.scalar("shaperA"), "A")
    close(g.shaper_b.cpu().numpy(), orc.scalar("shaperB"), "B")


def bits_of(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64)).view(np.int64)


@pytest.mark.parametrize("N,K,shaper", [(2048, 64, "DDR"), (65536, 24, "DDR"), (2048, 64, "sortino_shaperB"),
                                         (8192, 32, "sortino_shaperB")])
def test_running_pop_reference_shape_vs_oracle(gpu, N, K, shaper):
    """The reference's experiment shape (R1: one OU asset, W = 64 window, n =
    20 DDR on the summed agent reward) on the ONE layout's running-sum
    instantiation -- which the automatic schedule keeps at every batch (the
    exact pop's handles beyond 16384 envs take the single-role kernel):
    every output, n-step row (1e-6) and window of two launches with
    auto-resets against the oracle."""
    from madigan_amd import _lib as L
    sx = dict(sortino_exp=1.1) if shaper.startswith("sortino") else {}  # ou_sortinoB_exp_1.1_nstep20.yaml
    kw = dict(REF_KW, reward_shaper=shaper, seed=0x6D6164 + 41, nstep_pop="running", **sx)
    kw.update(required_margin=0.05, unit_size=0.9)
    g, orc = make_pair(ou_sources(1), N, **kw)
    assert g.lib.mgn_get_schedule(g.h) == L.SCHED_TRIO
    acts = g.generate_actions(2 * K, seed=0x6D6164 + 42)
    ends = _launch_vs_oracle(g, orc, acts[:K], f"R1 {shaper} running N={N} launch 0", RTOL, atol=ATOL)
    ends += _launch_vs_oracle(g, orc, acts[K:], f"R1 {shaper} running N={N} launch 1", RTOL, atol=ATOL)
    assert ends > N // 20
    state_check(g, orc, f"R1 {shaper} running N={N}")


def test_running_pop_not_granted_pops_exactly(gpu):
    """nstep_pop="running" is a permission: where the kernel has no running
    form (sortino_shaperB at the 256-lane layout: it has one at one wave per
    role only) or the discount would amplify the slides' rounding (gamma^n <
    1e-3), the pops stay the exact ones -- bit for bit the handle without the
    switch."""
    from madigan_amd import BatchedEnv
    for extra in (dict(reward_shaper="sortino_shaperB", sortino_exp=1.1, discount=0.99),
                  dict(reward_shaper="DDR", discount=0.5)):
        base = dict(required_margin=0.02, maintenance_margin=0.25, transaction_cost_rel=0.02, unit_size=0.9,
                    auto_reset=True, init_cash=1e5, nstep_return=20, seed=5, **extra)
        outs = []
        for pop in ("exact", "running"):
            g = BatchedEnv(spec_from_sources(trendou_sources(8, TOU)), 8192, nstep_pop=pop, **base)
            a = g.generate_actions(40, seed=3)
            outs.append(g.rollout(a)["shaped"].cpu().numpy())
        assert_bits(outs[1], outs[0], f"{extra} running == exact")
