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
    # the bench's output set unless STAMPS_FIELDS names one (comma separated)
    fields = os.environ.get("STAMPS_FIELDS", "reward,shaped,done,obs_price,obs_port,timestamp,tprice,"
                                             "tunits,tcost,risk,margin_call").split(",")
    out = env.alloc_traj(fuse, fields=[f for f in fields if f])
    for _ in range(3):
        env.rollout(acts, out)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * 24)()
    fn(buf)
    wall = getattr(lib, "mgn_diag_wall")
    wall.argtypes = [C.POINTER(C.c_ulonglong)]
    wb = (C.c_ulonglong * (2048 * 32))()
    reps = 10
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        env.rollout(acts, out)
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
    res["ledger"]["broker_parts"] = {k: round(v[13 + i] / max(it_l, 1), 1)
                                     for i, k in enumerate(("order_prep", "spec_loop", "post"))}
    res["ledger"]["phase2_parts"] = {k: round(v[16 + i] / max(it_l, 1), 1)
                                     for i, k in enumerate(("sums_done", "finish"))}
    # one more launch for the wall-clock phases (us from the first block entry)
    env.rollout(acts, out)
    torch.cuda.synchronize()
    wall(wb)
    import numpy as np
    nb = min(2048, (N + 31) // 32)
    raw = np.frombuffer(wb, dtype=np.uint64).reshape(2048, 32)[:nb].copy()
    if os.environ.get("STAMPS_RAW"):
        np.save(os.environ["STAMPS_RAW"], raw)
    w = raw[:, :8].astype(np.int64)
    t0 = w[:, :2].min()
    names = ("gen_entry", "led_entry", "led_loop_start", "led_loop_end", "gen_loop_end", "gen_exit",
             "led_iter0_end", "led_iter2_end")
    res["wall_us"] = {k: [round(float(w[:, i].min() - t0) / 100, 2),
                          round(float(np.median(w[:, i]) - t0) / 100, 2),
                          round(float(w[:, i].max() - t0) / 100, 2)] for i, k in enumerate(names)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
