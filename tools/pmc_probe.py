"""A bare launch sequence of the step kernel for rocprofv3 --pmc passes (no
bench bookkeeping, no other kernels between the timed launches).

    MADIGAN_LIB_PATH=... WORKLOAD=C3 N=8192 FUSE=20 REPS=8 AGE=0 \
        rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU ... -- python3 tools/pmc_probe.py

AGE steps are stepped first (64-step launches), so that the measured launches
run on episodes of that age; then 3 warm launches and REPS measured launches
of FUSE steps, each on fresh actions.  Prints one JSON line naming the
configuration; tools/pmc_brief.py reads the last REPS step-kernel dispatches.
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    N = int(os.environ.get("N", 8192))
    fuse = int(os.environ.get("FUSE", 20))
    reps = int(os.environ.get("REPS", 8))
    age = int(os.environ.get("AGE", 0))
    nst = int(os.environ.get("NSTEP", 1))
    wl = os.environ.get("WORKLOAD", "C3")
    A = int(os.environ.get("ASSETS", 8))
    extra = dict(nstep_return=nst, discount=0.99, nstep_pop=os.environ.get("NSTEP_POP", "exact")) if nst > 1 else {}
    env, _, _ = bench.workload_env(wl, N, A, 0, "cuda:0", **(extra if wl == "C3" else {}))
    if os.environ.get("SCHED"):  # force a schedule (single / duo / trio)
        from madigan_amd import _lib as L
        L.check(env.lib.mgn_set_schedule(env.h, {"single": L.SCHED_SINGLE, "duo": L.SCHED_DUO,
                                                 "trio": L.SCHED_TRIO}[os.environ["SCHED"]]), env.h)
    fields = ["reward", "shaped", "done", "obs_price", "obs_port", "timestamp", "tprice", "tunits", "tcost",
              "risk", "margin_call"]
    if age:
        a64 = env.generate_actions(64, seed=11)
        o64 = env.alloc_traj(64, fields=fields)
        for _ in range(age // 64):
            env.rollout(a64, o64)
        del o64
    acts = env.generate_actions(fuse * (reps + 3), seed=5)
    out = env.alloc_traj(fuse, fields=fields)
    if env.W > 0 and os.environ.get("GATHER", "0") == "1":
        # windowed workloads: each launch's K steps (mgn_rollout_hist) then
        # every step's window (mgn_window_hist) -- the bench's windowed() pair;
        # PMC_KERNEL=k_hist_gather selects the gather's dispatches
        import ctypes as C
        from madigan_amd import _lib as L
        W, F = env.W, env.F
        wp = torch.empty((fuse, N, W, F), dtype=torch.float64, device="cuda:0")
        wo = torch.empty((fuse, N, W, A + 1), dtype=torch.float64, device="cuda:0")
        wt = torch.empty((fuse, N, W), dtype=torch.int64, device="cuda:0")
        t = env._traj_struct(out)
        per = N * A
        for r in range(reps + 3):
            L.check(env.lib.mgn_rollout_hist(env.h, C.c_void_p(acts.data_ptr() + r * fuse * per), fuse, C.byref(t)),
                    env.h)
            L.check(env.lib.mgn_window_hist(env.h, *[C.c_void_p(x.data_ptr()) for x in (wp, wo, wt)]), env.h)
    else:
        for r in range(reps + 3):
            env.rollout(acts[r * fuse:(r + 1) * fuse], out)
    torch.cuda.synchronize()
    print(json.dumps({"workload": wl, "N": N, "assets": env.A, "fuse": fuse, "reps": reps, "age": age,
                      "nstep": nst, "sched": os.environ.get("SCHED", "auto"),
                      "lib": os.environ.get("MADIGAN_LIB_PATH", "product")}))


if __name__ == "__main__":
    main()
