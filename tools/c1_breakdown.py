"""Diagnostic: where the drop-in Env.step's time goes (C1: one 1-asset Sine
env, units from numpy): the whole step, the launch alone + synchronise, the
host snapshot alone (valuation launch, copies, synchronise), and pieces."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from madigan_amd import Env  # noqa: E402
from madigan_amd import _lib as L  # noqa: E402

cfg = {"data_source_type": "Synth",
       "data_source_config": {"freq": [1.0], "mu": [2.0], "amp": [1.0], "phase": [0.0],
                              "dX": 0.01, "noise": 0.0}}
env = Env("Synth", 1_000_000.0, cfg, device=torch.device("cuda:0"), seed=5)
b = env.batched
u = np.array([10.0])
res = {}


def timed(name, f, reps=400):
    for _ in range(20):
        f()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        t.append(time.perf_counter() - t0)
    res[name] = float(np.median(t)) * 1e6


timed("env_step_units", lambda: env.step(u))
timed("env_step_none", lambda: env.step())


def launch_sync():
    b.step(units=u.reshape(1, -1))
    torch.cuda.synchronize()


timed("batched_step_units_plus_sync", launch_sync)


def launch_only_sync():
    L.check(b.lib.mgn_step(b.h, L.STEP_NONE, None, None), b.h)
    torch.cuda.synchronize()


timed("mgn_step_none_plus_sync", launch_only_sync)


def snap():
    env._dirty()
    env._snapshot()


timed("snapshot", snap)


def val_only():
    L.check(b.lib.mgn_valuation(b.h, C.c_void_p(b._val.data_ptr())), b.h)
    b.stream.synchronize()


timed("valuation_launch_plus_sync", val_only)


def copy1():
    hip = L.hip()
    st = C.c_void_p(b.stream.cuda_stream)
    hip.hipMemcpyAsync(C.c_void_p(env._h_buf.data_ptr()), C.c_void_p(b._arena_buf.data_ptr()),
                       C.c_size_t(env._h_buf.numel()), 2, st)
    hip.hipStreamSynchronize(st)


timed("one_d2h_copy_plus_sync", copy1)
res["arena_bytes"] = int(b.arena.numel())
print(json.dumps(res, indent=1))
