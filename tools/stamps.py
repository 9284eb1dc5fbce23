"""Phase balance of k_step_duo at C3 (diagnostic build with -DMGN_STAMPS).

    MADIGAN_LIB_PATH=tools/_var/stamps/libmadigan_hip.so python tools/stamps.py

Prints, per role, the mean cycles per iteration spent working before barrier
A, waiting at A, working before B, waiting at B (s_memtime, one wave per role
and block), and the launch time.
"""
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    N = int(os.environ.get("N", 8192))
    fuse = int(os.environ.get("FUSE", 64))
    env, _, _ = bench.workload_env("C3", N, 8, 0, "cuda:0")
    lib = env.lib
    fn = getattr(lib, "mgn_diag_stamps")
    fn.argtypes = [C.POINTER(C.c_ulonglong)]
    acts = env.generate_actions(fuse, seed=5)
    for _ in range(3):
        env.rollout(acts)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * 16)()
    fn(buf)
    reps = 10
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        env.rollout(acts)
    e1.record()
    torch.cuda.synchronize()
    fn(buf)
    v = list(buf)
    blocks = v[10]
    it_g, it_l = v[8], v[9]
    res = {"N": N, "fuse": fuse, "us_per_launch": e0.elapsed_time(e1) * 1000 / reps,
           "iters_per_block": it_g / max(blocks, 1)}
    for role, base, it in (("gen", 0, it_g), ("ledger", 4, it_l)):
        res[role] = {k: round(v[base + i] / max(it, 1), 1)
                     for i, k in enumerate(("work1", "waitA", "work2", "waitB"))}
    res["ledger"]["action"] = round(v[11] / max(it_l, 1), 1)
    res["ledger"]["broker"] = round(v[12] / max(it_l, 1), 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
