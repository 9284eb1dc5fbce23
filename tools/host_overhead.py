"""Diagnostic: host-side cost around one 20-step C3 launch (the driver's
bench shape): wall time of [launch; synchronize] with and without the
library's kernel events, with one or two synchronizes, against the kernel
time itself (events) and an idle synchronize."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from madigan_amd import _lib as L  # noqa: E402

env, _, _ = bench.workload_env("C3", 8192, 8, 0, torch.device("cuda:0"))
lib, h = env.lib, env.h
K = int(os.environ.get("K", 20))
acts = env.generate_actions(K * 40, seed=5)
traj = env.alloc_traj(K, fields=["reward", "shaped", "done", "obs_price", "obs_port", "timestamp",
                                 "tprice", "tunits", "tcost", "risk", "margin_call"])
fn = env.rollout_launcher(traj, K)
base, per = acts.data_ptr(), env.N * env.A
res = {}


def trial(name, timing, syncs, reps=30):
    ts = []
    L.check(lib.mgn_set_timing(h, 1 if timing else 0), h)
    for r in range(reps):
        torch.cuda.synchronize()
        time.sleep(0.002)
        t0 = time.perf_counter()
        fn(base + (r % 40) * K * per)
        for _ in range(syncs):
            torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    if timing:
        tm = (C.c_double * 4)()
        L.check(lib.mgn_get_timing(h, tm), h)
        res[name + "_kernel_us"] = tm[0] / tm[1] * 1e3
    res[name + "_wall_us"] = float(np.median(ts[3:])) * 1e6


trial("events_2sync", True, 2)
trial("events_1sync", True, 1)
trial("noevents_1sync", False, 1)
trial("noevents_2sync", False, 2)
ts = []
for r in range(30):
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
res["idle_sync_us"] = float(np.median(ts)) * 1e6
ts = []
for r in range(30):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn(base)
    ts.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
res["launch_call_us"] = float(np.median(ts)) * 1e6
print(json.dumps(res))
