"""Per-launch, per-block wall stamps of k_step_duo (diagnostic build -DMGN_WALLX).

    MADIGAN_LIB_PATH=tools/_var/wallx/libmadigan_hip.so FUSE=20 LAUNCHES=20 \
        python tools/wallx.py OUT.npz

Saves wall[launch, block, 32] (see mgn_duo.h: [0..7] phase stamps, [8] HW_ID,
[9] XCC_ID, [10]/[11] writeback ends, [12]/[13] slowest generator store phase
and its iteration, [14]/[15] slowest ledger phase 1 and its iteration, [16..21] prologue points: generator / ledger after the
state loads issue, after the staging barrier, after the drain) and the
launch durations (HIP events) for the C3 workload.
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    N = int(os.environ.get("N", 8192))
    fuse = int(os.environ.get("FUSE", 20))
    launches = int(os.environ.get("LAUNCHES", 20))
    env, _, _ = bench.workload_env("C3", N, 8, 0, "cuda:0")
    fields = os.environ.get("FIELDS", "reward,shaped,done,obs_price,obs_port,timestamp,tprice,"
                                      "tunits,tcost,risk,margin_call").split(",")
    out = env.alloc_traj(fuse, fields=[f for f in fields if f])
    acts = env.generate_actions(fuse * (launches + 3), seed=5)
    wall = env.lib.mgn_diag_wall
    wall.argtypes = [C.POINTER(C.c_ulonglong)]
    wb = (C.c_ulonglong * (2048 * 32))()
    nb = min(2048, (N + 31) // 32)
    for i in range(3):
        env.rollout(acts[i * fuse:(i + 1) * fuse], out)
    torch.cuda.synchronize()
    walls, durs = [], []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(3, launches + 3):
        e0.record()
        env.rollout(acts[i * fuse:(i + 1) * fuse], out)
        e1.record()
        torch.cuda.synchronize()
        durs.append(e0.elapsed_time(e1) * 1000)
        wall(wb)
        walls.append(np.frombuffer(wb, dtype=np.uint64).reshape(2048, 32)[:nb].copy())
    np.savez(sys.argv[1], wall=np.stack(walls), dur_us=np.array(durs), N=N, fuse=fuse)
    print(f"N {N} fuse {fuse} launch us: median {np.median(durs):.1f} min {min(durs):.1f} max {max(durs):.1f}")


if __name__ == "__main__":
    main()
