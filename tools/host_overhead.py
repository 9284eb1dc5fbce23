"""Host overhead of the driver's timed region (diagnostic): one 20-step launch
at C3 (8192 x 8) bracketed by torch.cuda.synchronize(), repeated; the median
wall time by launcher (ctypes / the CPython binding) and kernel-timing mode
(0 none, 1 marker events, 2 events recorded by the launch).  Run it once with
the default environment and once with HSA_ENABLE_INTERRUPT=0 to see the
completion-signal wait.

    python tools/host_overhead.py [--reps 300]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--k", type=int, default=20)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from madigan_amd import _lib as L
    dev = torch.device("cuda:0")
    env, _, _ = bench.workload_env("C3", 8192, 8, 0, dev)
    K = a.k
    acts = env.generate_actions(K * 4, seed=0x6D6164)
    traj = env.alloc_traj(K, fields=["reward", "shaped", "done", "obs_price", "obs_port", "timestamp",
                                     "tprice", "tunits", "tcost", "risk", "margin_call"])
    lib, h = env.lib, env.h
    t = env._traj_for(traj, K)
    ref = C.byref(t)
    fn = lib.mgn_rollout
    pc = L.pycall()
    ptr = acts.data_ptr()

    def via_ctypes():
        return fn(h, ptr, K, ref)

    def via_pycall():
        return pc.rollout(int(h), ptr, K, C.addressof(t))

    res = {"HSA_ENABLE_INTERRUPT": os.environ.get("HSA_ENABLE_INTERRUPT", "(default)")}
    for name, call in (("ctypes", via_ctypes), ("pycall", via_pycall)):
        if call is via_pycall and pc is None:
            continue
        for mode in (0, 1, 2):
            L.check(lib.mgn_set_timing(h, mode), h)
            for _ in range(20):
                call()
            torch.cuda.synchronize()
            wall, host = [], []
            for _ in range(a.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                rc = call()
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                L.check(rc, h)
                wall.append((t2 - t0) * 1e6)
                host.append((t1 - t0) * 1e6)
            tm = (C.c_double * 4)()
            L.check(lib.mgn_get_timing(h, tm), h)
            kus = tm[0] / max(tm[1], 1) * 1e3 if mode else None
            res[f"{name}_mode{mode}"] = {"wall_us_median": float(np.median(wall)),
                                         "wall_us_p10": float(np.percentile(wall, 10)),
                                         "launch_call_us_median": float(np.median(host)),
                                         "kernel_us": kus}
            print(name, mode, json.dumps(res[f"{name}_mode{mode}"]), flush=True)
    L.check(lib.mgn_set_timing(h, 0), h)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
