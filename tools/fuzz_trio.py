"""Randomised schedule-equivalence check (diagnostic, GPU): random handles --
2..16 assets, generator kinds (one kind or mixed), batch sizes on both sides
of the 256-lane and two-slot thresholds, windows, n-step, shapers, reward
modes, leveraged brokers that end episodes -- each run on the three-role
kernel and on the two-role kernel from the same construction, launch lengths
1 / 3 / 17, a unit step in between; every output, the window and the whole
state compared bit for bit.

    python tools/fuzz_trio.py [n_cases] [seed]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from tests.configs import composite_sources, spec_from_sources, trendou_sources  # noqa: E402

P_TOU = [0.2, 2, 6, 0.05, 0.2, 5.0, 0.15, 0.3, 0.2, 0.99]


def sources_for(rng, A, mixed):
    if not mixed:
        kind = rng.integers(0, 2)
        return trendou_sources(A, P_TOU) if kind == 0 else [(O.SRC_OU, [10.0, 0.15, 0.04])] * A
    pool = composite_sources()[:5] + trendou_sources(3, P_TOU)
    return [pool[int(i)] for i in rng.integers(0, len(pool), A)]


def state(g):
    names = ["ledger", "mean_entry", "borrowed", "cash", "prices", "timestamp", "episode_stats", "shaper_a",
             "shaper_b", "draw_skip"]
    return {n: getattr(g, n).cpu().numpy() for n in names}


def same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.dtype == np.float64:
        return np.array_equal(a.view(np.int64), b.view(np.int64))
    return np.array_equal(a, b)


def one_case(rng, i):
    from madigan_amd import BatchedEnv
    from madigan_amd import _lib as L
    A = int(rng.choice([2, 3, 4, 5, 8, 9, 12, 13, 16]))
    N = int(rng.choice([64, 300, 1024, 4096, 8192]))
    mixed = bool(rng.integers(0, 2))
    kw = dict(required_margin=float(rng.choice([1.0, 0.1, 0.02])), maintenance_margin=0.25,
              transaction_cost_rel=0.02, slippage_rel=1e-4, unit_size=float(rng.choice([0.05, 0.9])),
              auto_reset=True, init_cash=1e5, seed=int(rng.integers(1, 1 << 30)),
              reward_shaper=str(rng.choice(["DDR", "DSR", "PPC"])), cosine_temp=0.05)
    r = rng.random()
    if r < 0.3:
        kw.update(window=int(rng.choice([4, 8, 16])), norm_type=[None, "log"][int(rng.integers(0, 2))])
    elif r < 0.5 and kw["reward_shaper"] in ("DDR", "DSR"):
        kw.update(nstep_return=int(rng.choice([3, 5, 20])), discount=0.97)
    if rng.random() < 0.2 and "nstep_return" not in kw:
        kw["reward_mode"] = "agent_sum"
    spec = spec_from_sources(sources_for(rng, A, mixed))
    Ks = [int(k) for k in rng.choice([1, 3, 17], 3)]
    units = rng.normal(0, 3e3, (N, A))
    res = []
    for sched in (L.SCHED_DUO, L.SCHED_TRIO):
        g = BatchedEnv(spec, N, **kw)
        if g.lib.mgn_set_schedule(g.h, sched) != 0 or g.lib.mgn_get_schedule(g.h) != sched:
            return None  # not eligible for one of the kernels
        acts = g.generate_actions(sum(Ks), seed=i)
        out, k0 = [], 0
        for j, K in enumerate(Ks):
            o = {k: v.cpu().numpy() for k, v in g.rollout(acts[k0:k0 + K]).items()}
            k0 += K
            o.update({"st_" + k: v for k, v in state(g).items()})
            if g.W:
                o.update({"w_" + str(q): t.cpu().numpy() for q, t in enumerate(g.window())})
            out.append(o)
            if j == 0:
                g.step(units)
                out.append({"u_" + k: v for k, v in g.host_outputs().items()})
        res.append(out)
    bad = []
    for j, (a, b) in enumerate(zip(*res)):
        for k in a:
            if not same(a[k], b[k]):
                bad.append(f"launch {j} {k}")
    desc = f"A={A} N={N} mixed={mixed} Ks={Ks} {kw}"
    return desc, bad


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 7)
    t0 = time.time()
    fails = ran = 0
    for i in range(n):
        r = one_case(rng, i)
        if r is None:
            print(f"case {i}: skipped (schedule refused)", flush=True)
            continue
        ran += 1
        desc, bad = r
        print(f"case {i}: {'OK' if not bad else 'MISMATCH ' + ', '.join(bad[:6])} | {desc}", flush=True)
        fails += bool(bad)
    print(f"fuzz: {ran} cases, {fails} mismatches, {time.time() - t0:.0f} s", flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
