"""Diagnostic: the host's share of the driver's timed region -- one 20-step
C3 launch (bench.py's shape) and the wait for it -- by wait method and with
or without the launch's own timing events.  Wall time of [launch; wait]
(median of `reps`, each from an idle device), the launch call alone, and the
kernel time by the launch events.  Wait methods: torch.cuda.synchronize
(device), mgn_synchronize (hipStreamSynchronize on the handle's stream), a
spin on hipStreamQuery, a spin on hipEventQuery of an event recorded after the
launch."""
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

hip = C.CDLL("libamdhip64.so")
hip.hipStreamQuery.argtypes = [C.c_void_p]
hip.hipEventQuery.argtypes = [C.c_void_p]
hip.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
hip.hipEventCreateWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
env, _, _ = bench.workload_env("C3", 8192, 8, 0, torch.device("cuda:0"))
lib, h = env.lib, env.h
K = int(os.environ.get("K", 20))
T = 40 * K
acts = env.generate_actions(T, seed=5)
traj = env.alloc_traj(K, fields=["reward", "shaped", "done", "obs_price", "obs_port", "timestamp",
                                 "tprice", "tunits", "tcost", "risk", "margin_call"])
fn = env.rollout_launcher(traj, K, acts)
st = C.c_void_p(env.stream.cuda_stream)
msync = env.stream_synchronizer()
ev = C.c_void_p()
hip.hipEventCreateWithFlags(C.byref(ev), C.c_uint(2))  # hipEventDisableTiming
res = {"stream": env.stream.cuda_stream}


def spin_stream():
    while hip.hipStreamQuery(st) != 0:
        pass


def spin_event():
    hip.hipEventRecord(ev, st)
    while hip.hipEventQuery(ev) != 0:
        pass


WAITS = {"device_sync": torch.cuda.synchronize, "mgn_synchronize": msync, "spin_stream_query": spin_stream,
         "spin_event_query": spin_event}


def trial(name, timing, wait, reps=40, sleep=0.002):
    ts, tl = [], []
    L.check(lib.mgn_set_timing(h, 2 if timing else 0), h)
    for r in range(reps):
        torch.cuda.synchronize()
        if sleep:
            time.sleep(sleep)
        t0 = time.perf_counter()
        fn((r % 40) * K)
        t1 = time.perf_counter()
        wait()
        ts.append(time.perf_counter() - t0)
        tl.append(t1 - t0)
    out = {"wall_us": float(np.median(ts[4:])) * 1e6, "wall_min_us": float(np.min(ts[4:])) * 1e6,
           "launch_call_us": float(np.median(tl[4:])) * 1e6}
    if timing:
        tm = (C.c_double * 4)()
        L.check(lib.mgn_get_timing(h, tm), h)
        out["kernel_us"] = tm[0] / tm[1] * 1e3
        out["host_share_us"] = out["wall_us"] - out["kernel_us"]
    L.check(lib.mgn_set_timing(h, 0), h)
    res[name] = out


for wname, w in WAITS.items():
    trial(f"events_{wname}", True, w)
    trial(f"noevents_{wname}", False, w)
trial("events_mgn_synchronize_nosleep", True, msync, sleep=0)
# the floor: launch + wait of a trivial kernel (k_gen_actions)
ga = env.generate_actions(1, seed=1)
for wname in ("device_sync", "spin_stream_query"):
    ts = []
    for r in range(40):
        torch.cuda.synchronize()
        time.sleep(0.002)
        t0 = time.perf_counter()
        lib.mgn_generate_actions(h, C.c_void_p(ga.data_ptr()), 1, C.c_uint64(r))
        WAITS[wname]()
        ts.append(time.perf_counter() - t0)
    res[f"trivial_kernel_{wname}_wall_us"] = float(np.median(ts[4:])) * 1e6
print(json.dumps(res, indent=1))
