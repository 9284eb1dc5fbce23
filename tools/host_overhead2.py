"""Diagnostic: what the host adds around one K-step C3 launch (the driver's
bench shape, K = 20).  Wall time of [launch; synchronize] against the kernel
time (events), for: the handle on torch's null stream vs a created stream,
synchronising the device (torch.cuda.synchronize) vs the stream, with and
without the library's kernel-timing events, before and after switching the
device to spin-wait synchronisation (hipSetDeviceFlags(hipDeviceScheduleSpin))."""
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
env, _, _ = bench.workload_env("C3", 8192, 8, 0, torch.device("cuda:0"))
lib, h = env.lib, env.h
K = int(os.environ.get("K", 20))
acts = env.generate_actions(K * 40, seed=5)
traj = env.alloc_traj(K, fields=["reward", "shaped", "done", "obs_price", "obs_port", "timestamp",
                                 "tprice", "tunits", "tcost", "risk", "margin_call"])
fn = env.rollout_launcher(traj, K)
base, per = acts.data_ptr(), env.N * env.A
side = torch.cuda.Stream()
res = {}


def trial(name, timing, sync, reps=40):
    ts, tl = [], []
    L.check(lib.mgn_set_timing(h, 1 if timing else 0), h)
    for r in range(reps):
        torch.cuda.synchronize()
        time.sleep(0.002)
        t0 = time.perf_counter()
        fn(base + (r % 40) * K * per)
        t1 = time.perf_counter()
        sync()
        ts.append(time.perf_counter() - t0)
        tl.append(t1 - t0)
    out = {"wall_us": float(np.median(ts[4:])) * 1e6, "launch_call_us": float(np.median(tl[4:])) * 1e6}
    if timing:
        tm = (C.c_double * 4)()
        L.check(lib.mgn_get_timing(h, tm), h)
        out["kernel_us"] = tm[0] / tm[1] * 1e3
    res[name] = out


def sweep(tag):
    L.check(lib.mgn_set_stream(h, C.c_void_p(0)), h)
    trial(tag + "null_events_devsync", True, torch.cuda.synchronize)
    trial(tag + "null_noevents_devsync", False, torch.cuda.synchronize)
    L.check(lib.mgn_set_stream(h, C.c_void_p(side.cuda_stream)), h)
    ssync = lambda: hip.hipStreamSynchronize(C.c_void_p(side.cuda_stream))  # noqa: E731
    trial(tag + "side_events_streamsync", True, ssync)
    trial(tag + "side_noevents_streamsync", False, ssync)
    trial(tag + "side_events_devsync", True, torch.cuda.synchronize)
    ts = []
    for r in range(30):
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    res[tag + "idle_devsync_us"] = float(np.median(ts)) * 1e6


sweep("")
# the floor: a trivial kernel (k_gen_actions, 256 workgroups) launched and synchronised
ga = env.generate_actions(1, seed=1)
ts, tl = [], []
for r in range(40):
    torch.cuda.synchronize()
    time.sleep(0.002)
    t0 = time.perf_counter()
    lib.mgn_generate_actions(h, C.c_void_p(ga.data_ptr()), 1, C.c_uint64(r))
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
    tl.append(t1 - t0)
res["trivial_kernel"] = {"wall_us": float(np.median(ts[4:])) * 1e6, "launch_call_us": float(np.median(tl[4:])) * 1e6}
# back-to-back (no sleep): the timed launch right after another
ts = []
for r in range(40):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn(base + (r % 40) * K * per)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
res["nosleep_null_noevents_devsync_wall_us"] = float(np.median(ts[4:])) * 1e6
if os.environ.get("SPIN"):
    rc = hip.hipSetDeviceFlags(C.c_uint(1))  # hipDeviceScheduleSpin
    res["setflags_spin_rc"] = rc
    sweep("spin_")
res["env"] = {k: os.environ.get(k) for k in ("HIP_FORCE_DEV_KERNARG", "GPU_MAX_HW_QUEUES", "AMD_DIRECT_DISPATCH")}
L.check(lib.mgn_set_stream(h, C.c_void_p(0)), h)
print(json.dumps(res, indent=1))
