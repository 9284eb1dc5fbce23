"""K = 1 launch time on the C3 handle by how the launch is set up (diagnostic):
own-size trajectory vs a slice of a 256-step one, fresh vs reused actions.

    python tools/k1_diag.py
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


def timed(env, fn, ptrs, reps):
    lib, h = env.lib, env.h
    fn(ptrs[0])
    torch.cuda.synchronize()
    L.check(lib.mgn_set_timing(h, 2), h)
    for r in range(reps):
        fn(ptrs[r % len(ptrs)])
    torch.cuda.synchronize()
    tk = (C.c_double * 4)()
    L.check(lib.mgn_get_timing(h, tk), h)
    L.check(lib.mgn_set_timing(h, 0), h)
    return tk[0] / max(int(tk[1]), 1) * 1e3


def main():
    N, A = 8192, 8
    env, _, _ = bench.workload_env("C3", N, A, 0, "cuda:0")
    fields = ["reward", "shaped", "done", "obs_price", "obs_port", "timestamp", "tprice", "tunits", "tcost",
              "risk", "margin_call"]
    res = {}
    for K in (1, 16):
        acts = env.generate_actions(512 * K, seed=3)
        per = N * A
        base = acts.data_ptr()
        own = env.alloc_traj(K, fields=fields)
        big = env.alloc_traj(256, fields=fields)
        f_own = env.rollout_launcher(own, K)
        f_big = env.rollout_launcher({k: v[:K] for k, v in big.items()}, K)
        fresh = [base + i * K * per for i in range(512)]
        same = [base]
        res[K] = {"own_fresh": timed(env, f_own, fresh, 256), "own_same": timed(env, f_own, same, 256),
                  "slice_fresh": timed(env, f_big, fresh, 256), "slice_same": timed(env, f_big, same, 256),
                  "own_fresh_again": timed(env, f_own, fresh, 256)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
