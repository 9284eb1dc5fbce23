"""Randomised schedule-equivalence check (diagnostic, GPU): random handles --
1..16 assets, generator kinds (one kind or mixed), batch sizes on both sides
of the 256-lane and two-slot thresholds, windows, n-step (with windows, and
the naive shapers), shapers, reward modes, auto-reset on or off, leveraged
brokers that end episodes -- each run on the three-role kernel and on the
two-role kernel (the single-role kernel for one asset) from the same
construction: discrete launches of 1 / 3 / 17 steps with a units step, a
single-asset step or a discrete launch between them; every output, the window
and the whole state (draw_skip included) compared bit for bit.  Every
ORACLE_EVERY-th case also runs the oracle (oracle/) beside the three-role
kernel: the same outputs (rewards at rtol 1e-12, shaped rewards 1e-10) and
state after every launch.

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

ORACLE_EVERY = int(os.environ.get("ORACLE_EVERY", 4))

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
    A = int(rng.choice([1, 2, 3, 4, 5, 8, 9, 12, 13, 16]))
    N = int(rng.choice([64, 300, 1024, 4096, 8192]))
    mixed = bool(rng.integers(0, 2)) and A > 1
    kw = dict(required_margin=float(rng.choice([1.0, 0.1, 0.02])), maintenance_margin=0.25,
              transaction_cost_rel=0.02, slippage_rel=1e-4, unit_size=float(rng.choice([0.05, 0.9])),
              auto_reset=bool(rng.random() < 0.85), init_cash=1e5, seed=int(rng.integers(1, 1 << 30)),
              reward_shaper=str(rng.choice(["DDR", "DSR", "PPC", "sortino_shaperB", "sharpe_shaper"])),
              cosine_temp=0.05)
    if kw["reward_shaper"].startswith("sortino"):
        kw["sortino_exp"] = float(rng.choice([1.1, 2.0]))
    r = rng.random()
    if r < 0.3:
        kw.update(window=int(rng.choice([4, 8, 16])), norm_type=[None, "log"][int(rng.integers(0, 2))])
    if (r < 0.15 or 0.3 <= r < 0.55) and kw["reward_shaper"] != "PPC":
        kw.update(nstep_return=int(rng.choice([3, 5, 20])), discount=0.97)
    if rng.random() < 0.2 and "nstep_return" not in kw:
        kw["reward_mode"] = "agent_sum"
    elif "nstep_return" in kw and rng.random() < 0.5:
        kw["reward_mode"] = "agent_sum"
    srcs = sources_for(rng, A, mixed)
    spec = spec_from_sources(srcs)
    Ks = [int(k) for k in rng.choice([1, 3, 17], 3)]
    between = str(rng.choice(["units", "single", "discrete"]))
    units = rng.normal(0, 3e3, (N, A))
    aidx = rng.integers(0, A, N).astype(np.int32)
    u1 = rng.normal(0, 3e3, N)
    ref_sched = L.SCHED_DUO if A >= 2 else L.SCHED_SINGLE
    use_oracle = i % ORACLE_EVERY == 0
    res = []
    for sched in (ref_sched, L.SCHED_TRIO):
        g = BatchedEnv(spec, N, **kw)
        if g.lib.mgn_set_schedule(g.h, sched) != 0 or g.lib.mgn_get_schedule(g.h) != sched:
            return None  # not eligible for one of the kernels
        orc = None
        if use_oracle and sched == L.SCHED_TRIO:
            okw = dict(kw, n_envs=N)
            okw["auto_reset"] = int(okw["auto_reset"])
            orc = O.OracleBatch(okw, srcs)
        acts = g.generate_actions(sum(Ks), seed=i)
        a_host = acts.cpu().numpy()
        out, k0, obad = [], 0, []
        for j, K in enumerate(Ks):
            o = {k: v.cpu().numpy() for k, v in g.rollout(acts[k0:k0 + K]).items()}
            if orc is not None:
                ref = orc.rollout(a_host[k0:k0 + K], threads=8)
                obad += oracle_diff(o, ref, g, orc, f"launch {j}")
            k0 += K
            o.update({"st_" + k: v for k, v in state(g).items()})
            if g.W:
                o.update({"w_" + str(q): t.cpu().numpy() for q, t in enumerate(g.window())})
            out.append(o)
            if j == 0:
                if between == "units":
                    g.step(units)
                    ref = orc.step(units) if orc is not None else None
                elif between == "single":
                    g.step(u1, aidx)
                    ref = orc.step(u1, aidx) if orc is not None else None
                else:
                    g.step()
                    ref = orc.step() if orc is not None else None
                ho = g.host_outputs()
                if orc is not None:
                    obad += oracle_diff(ho, ref, g, orc, f"{between} step")
                out.append({"u_" + k: v for k, v in ho.items()})
        res.append((out, obad))
    bad = []
    for j, (a, b) in enumerate(zip(res[0][0], res[1][0])):
        for k in a:
            if not same(a[k], b[k]):
                bad.append(f"launch {j} {k}")
    bad += ["oracle: " + x for x in res[1][1]]
    desc = f"A={A} N={N} mixed={mixed} Ks={Ks} between={between} oracle={use_oracle} {kw}"
    return desc, bad


def oracle_diff(o, ref, g, orc, tag):
    """The outputs and state that differ from the oracle's (bit for bit; the
    rewards within rtol 1e-12, shaped rewards 1e-10, as the parity tests)."""
    bad = []
    for k in ("obs_price", "obs_port", "tprice", "tunits", "tcost", "risk", "done", "margin_call"):
        if k in o and k in ref and not same(np.asarray(o[k]).reshape(np.shape(ref[k])), ref[k]):
            bad.append(f"{tag} {k}")
    for k, rt in (("reward", 1e-12), ("shaped", 1e-10)):
        if k in o and k in ref and not np.allclose(np.asarray(o[k]).reshape(np.shape(ref[k])), ref[k], rtol=rt,
                                                   atol=1e-14, equal_nan=True):
            bad.append(f"{tag} {k}")
    for name, f in (("ledger", O.F_LEDGER), ("mean_entry", O.F_MEP), ("borrowed", O.F_BORROWED),
                    ("prices", O.F_PRICE)):
        if not same(getattr(g, name).cpu().numpy(), orc.field(f)):
            bad.append(f"{tag} state {name}")
    if not same(g.cash.cpu().numpy(), orc.scalar("cash")):
        bad.append(f"{tag} state cash")
    if not np.array_equal(g.draw_skip.cpu().numpy(), orc.scalar("draw_skip").astype(np.int64)):
        bad.append(f"{tag} state draw_skip")
    return bad


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
