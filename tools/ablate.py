"""Diagnostic: attribute the fused step's time by ablation (outputs wrong in
ablated variants; never used for reported numbers).  Variants are interleaved
in one process (cdna_hip_programming.md 5.4 rule 24)."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import TRENDOU_P, c3_kwargs  # noqa: E402
from madigan_amd import BatchedEnv  # noqa: E402
from madigan_amd.config import trendou_spec  # noqa: E402

N = int(os.environ.get("N", 8192))
A, F = 8, 64
env = BatchedEnv(trendou_spec(*[[p] * A for p in TRENDOU_P]), N, seed=1, **c3_kwargs())
acts = env.generate_actions(F, seed=3)
traj = env.alloc_traj(F, fields=["reward", "shaped", "done", "obs_price", "obs_port", "timestamp",
                                 "tprice", "tunits", "tcost", "risk", "margin_call"])
if os.environ.get("LAYOUT"):
    env.lib.mgn_set_layout(env.h, int(os.environ["LAYOUT"]))
variants = {"full": 0, "no_rounds": 1, "no_gen": 2, "no_store": 4, "no_log": 8,
            "rounds_only": 2 | 4 | 8, "gen_only": 1 | 4 | 8, "none": 15}
times = {k: [] for k in variants}
for rep in range(6):
    for name, flags in variants.items():
        env.lib.mgn_set_ablation(env.h, flags)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        env.rollout(acts, out=traj)
        e.record()
        torch.cuda.synchronize()
        if rep:
            times[name].append(s.elapsed_time(e) * 1e3 / F)
env.lib.mgn_set_ablation(env.h, 0)
print(json.dumps({"N": N, "layout": int(env.lib.mgn_get_layout(env.h)), "us_per_step":
                  {k: round(float(np.median(v)), 3) for k, v in times.items()}}))
