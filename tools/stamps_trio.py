"""Per-role cycles of k_step_trio (diagnostic build with -DMGN_STAMPS).

    MADIGAN_LIB_PATH=tools/_var/stamps/libmadigan_hip.so FUSE=64 python tools/stamps_trio.py

Prints, per role (generator / ledger / finish), the mean cycles per
iteration spent working before the iteration's barrier and waiting at it
(s_memtime, one wave per role and block), the ledger's Broker parts, and the
launch time.
"""
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from madigan_amd import _lib as L  # noqa: E402


def main():
    N = int(os.environ.get("N", 8192))
    fuse = int(os.environ.get("FUSE", 64))
    nst = int(os.environ.get("NSTEP", 1))
    extra = dict(nstep_return=nst, discount=0.99, nstep_pop=os.environ.get("NSTEP_POP", "exact")) if nst > 1 else {}
    wl = os.environ.get("WORKLOAD", "C3")
    A = int(os.environ.get("ASSETS", 8))
    env, _, _ = bench.workload_env(wl, N, A, 0, "cuda:0", **(extra if wl == "C3" else {}))
    assert int(env.lib.mgn_get_schedule(env.h)) == L.SCHED_TRIO
    # the two-slot kernels (9..16 assets at >= 4096 envs) keep their stamps in
    # their own unit (mgn_launch_a16m2.hip)
    # (and the n-step kernels at APAD 8 in mgn_launch_a8nst.hip)
    if env.A > 8 and N * 16 >= 65536:
        fn = env.lib.mgn_diag_stamps_m2
    elif nst > 1 and env.A == 8:
        fn = env.lib.mgn_diag_stamps_nst
    else:
        fn = env.lib.mgn_diag_stamps
    fn.argtypes = [C.POINTER(C.c_ulonglong)]
    acts = env.generate_actions(fuse, seed=5)
    out = env.alloc_traj(fuse, fields=["reward", "shaped", "done", "obs_price", "obs_port", "timestamp",
                                       "tprice", "tunits", "tcost", "risk", "margin_call"])
    for _ in range(3):
        env.rollout(acts, out)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * 24)()
    fn(buf)
    reps = 10
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        env.rollout(acts, out)
    e1.record()
    torch.cuda.synchronize()
    fn(buf)
    v = list(buf)
    it = max(v[8], 1)
    res = {"workload": wl, "assets": env.A, "N": N, "fuse": fuse, "us_per_launch": e0.elapsed_time(e1) * 1000 / reps,
           "iters_per_block": v[8] / max(v[10], 1),
           "gen": {"work": round(v[0] / it, 1), "wait": round(v[1] / it, 1)},
           "ledger": {"work": round(v[4] / it, 1), "wait": round(v[5] / it, 1),
                      "broker_parts": {k: round(v[13 + i] / it, 1)
                                       for i, k in enumerate(("order_prep", "spec_loop", "post"))}},
           "ledger_phases": {k: round(v[20 + i] / it, 1) for i, k in
                             enumerate(("prices_and_pre_sums", "units", "broker", "records"))},
           "broker_first_pass": {"trees": round(v[2] / it, 1), "cash_chain": round(v[3] / it, 1),
                                 "checks_and_more_passes": round(v[6] / it, 1)},
           "finish": {"work": round(v[16] / it, 1), "wait": round(v[17] / it, 1),
                      # per iteration that evaluated a step (averaged over all
                      # iterations): records to reward / shaping / outputs
                      "phases": {k: round(v[i] / it, 1) for k, i in
                                 (("to_reward", 9), ("shaping", 11), ("outputs", 12))}},
           "ledger_passes_per_broker_call": round(v[19] / max(v[18], 1), 3)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
