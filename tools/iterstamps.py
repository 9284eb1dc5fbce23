"""Per-iteration timeline of the three-role kernel (diagnostic build -DMGN_ITERSTAMP).

    MGN_VARIANT_UNITS=8t,8k1 python tools/build_variant.py iter -DMGN_ITERSTAMP
    MADIGAN_LIB_PATH=tools/_var/iter/libmadigan_hip.so python tools/iterstamps.py [FUSE] [LAUNCHES]

Runs the driver's C3 shape (a 5-step warm launch, then FUSE-step launches),
reads the s_memtime stamps of the first 256 blocks and prints, as medians
over blocks and launches (cycles of s_memtime, and us at the measured rate):
entry -> prologue barrier, each iteration, the last iteration -> each role's
epilogue stores complete; beside the launch's event-timed duration.
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    fuse = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    env, _, _ = bench.workload_env("C3", 8192, 8, 0, "cuda:0")
    fields = ["reward", "shaped", "done", "obs_price", "obs_port", "timestamp", "tprice", "tunits",
              "tcost", "risk", "margin_call"]
    out = env.alloc_traj(fuse, fields=fields)
    acts = env.generate_actions(5 + fuse * launches, seed=0x6D6164)
    # (one-step launches run in mgn_launch_a8k1.hip, with its own stamp buffer)
    fn = env.lib.mgn_diag_iter_k1 if fuse == 1 else env.lib.mgn_diag_iter
    fn.argtypes = [C.POINTER(C.c_ulonglong)]
    buf = (C.c_ulonglong * (256 * 64))()
    w5 = env.alloc_traj(5, fields=fields)
    env.rollout(acts[:5], w5)
    torch.cuda.synchronize()
    fn(buf)
    # s_memtime rate: stamp a known wall interval
    rows, durs = [], []
    for i in range(launches):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        env.rollout(acts[5 + i * fuse:5 + (i + 1) * fuse], out)
        e1.record()
        torch.cuda.synchronize()
        durs.append(e0.elapsed_time(e1) * 1e3)
        fn(buf)
        rows.append(np.frombuffer(buf, dtype=np.uint64).reshape(256, 64).astype(np.int64).copy())
    st = np.stack(rows)  # (launches, 256, 64)
    base = st[:, :, 0:1]
    rel = st - base
    it = rel[:, :, 2:2 + fuse + 2]  # iterations 0..fuse (+1 spare)
    med = lambda x: float(np.median(x))  # noqa: E731
    res = {"fuse": fuse, "launch_us_event_median": med(durs),
           "prologue_cycles": med(rel[:, :, 1]),
           "iter0_cycles": med(it[:, :, 0] - rel[:, :, 1]),
           "iter_cycles_median": [med(it[:, :, j] - it[:, :, j - 1]) for j in range(1, fuse + 1)],
           "last_iter_to_g_epilogue": med(rel[:, :, 44] - it[:, :, fuse]),
           "last_iter_to_l_epilogue": med(rel[:, :, 45] - it[:, :, fuse]),
           "last_iter_to_f_epilogue": med(rel[:, :, 46] - it[:, :, fuse]),
           "entry_to_f_epilogue": med(rel[:, :, 46]),
           # from entry (finer stamps): kernel arguments, prologue barrier,
           # G tick published (iteration 0), L records published (iteration
           # 0), the iteration-0 barrier, F outputs issued (iteration 1), the
           # iteration-1 barrier, each role's epilogue
           "timeline_from_entry": {n: med(rel[:, :, i]) for n, i in (
               ("kernargs", 47), ("prologue_barrier", 1), ("g_state_loaded", 54),
               ("l_state_loaded", 51), ("l_prev_eq_it0", 58), ("l_orders_start_it0", 52),
               ("l_orders_done_it0", 53),
               ("g_tick_done_it0", 48),
               ("l_records_done_it0", 49), ("barrier_it0", 2), ("f_sums_it1", 55), ("f_reward_it1", 56),
               ("f_shaped_it1", 57), ("f_outputs_issued_it1", 50),
               ("barrier_it1", 3), ("g_epilogue", 44), ("l_epilogue", 45), ("f_epilogue", 46))},
           "block_entry_spread_cycles": med(st[:, :, 0].max(1) - st[:, :, 0].min(1))}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
