"""Diagnostic: the three-role kernel at 16 lanes per env against the
single-role kernel, field by field (which envs / assets / steps differ first).

    python tools/dbg_trio16.py [A] [N] [K]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    A = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    from madigan_amd import BatchedEnv, _lib as L
    from tests.configs import ou_sources, spec_from_sources, trendou_sources
    kind = sys.argv[4] if len(sys.argv) > 4 else 'trendou'
    base = dict(required_margin=0.02, maintenance_margin=0.25, transaction_cost_rel=0.02,
                slippage_rel=1e-4, unit_size=0.9, auto_reset=True, init_cash=1e5, seed=17,
                reward_shaper="DDR")
    if kind == 'ou':
        spec = spec_from_sources(ou_sources(A))
    else:
        spec = spec_from_sources(trendou_sources(A, [0.2, 2, 6, 0.05, 0.2, 5.0, 0.15, 0.3, 0.2, 0.99]))
    res = {}
    for name, sched in (("single", L.SCHED_SINGLE), ("duo", L.SCHED_DUO), ("trio", L.SCHED_TRIO)):
        g = BatchedEnv(spec, N, **base)
        L.check(g.lib.mgn_set_schedule(g.h, sched), g.h)
        acts = g.generate_actions(K, seed=9)
        p0 = g.prices.cpu().numpy().copy()
        out = {k: v.cpu().numpy() for k, v in g.rollout(acts).items()}
        out["ledger"] = g.ledger.cpu().numpy()
        out["prices"] = g.prices.cpu().numpy()
        out["cash"] = g.cash.cpu().numpy()
        out["acts"] = acts.cpu().numpy()
        out["p0"] = p0
        res[name] = out
    for other in ("duo", "trio"):
        for k, v in res["single"].items():
            w = res[other][k]
            a, b = np.asarray(v), np.asarray(w)
            if a.dtype == np.float64:
                diff = a.view(np.uint64) != b.view(np.uint64)
            else:
                diff = a != b
            if diff.any():
                idx = np.argwhere(diff)
                print(f"{other} {k} shape {a.shape}: {len(idx)} differ; first {idx[:6].tolist()}")
                i = tuple(idx[0])
                print(f"   single {a[i]!r} {other} {b[i]!r}")
    np.set_printoptions(linewidth=200, precision=5)
    for nm in ("single", "trio"):
        print(nm, "p0", res[nm]["p0"][0])
        print(nm, "obs0", res[nm]["obs_price"][0, 0])
        print(nm, "tunits0", res[nm]["tunits"][0, 0])
        print(nm, "prices", res[nm]["prices"][0])
    print("acts[0]", res["single"]["acts"][0].reshape(N, -1)[:4])
    print("done")


if __name__ == "__main__":
    main()
