"""Diagnostic: dynamic VALU / SALU / LDS instruction counts of k_step_duo per
ablation variant (run under rocprofv3 --pmc; dispatch order = variant order).
Outputs of ablated variants are wrong; never used for reported numbers."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import TRENDOU_P, c3_kwargs  # noqa: E402
from madigan_amd import BatchedEnv  # noqa: E402
from madigan_amd.config import trendou_spec  # noqa: E402

N, A, F = 8192, 8, 64
env = BatchedEnv(trendou_spec(*[[p] * A for p in TRENDOU_P]), N, seed=1, **c3_kwargs())
acts = env.generate_actions(F, seed=3)
traj = env.alloc_traj(F, fields=["reward", "shaped", "done", "obs_price", "obs_port", "timestamp",
                                 "tprice", "tunits", "tcost", "risk", "margin_call"])
variants = {"full": 0, "no_rounds": 1, "no_gen": 2, "no_finish": 4, "none": 7}
order = []
for name, flags in variants.items():
    env.lib.mgn_set_ablation(env.h, flags)
    env.rollout(acts, out=traj)
    order.append(name)
torch.cuda.synchronize()
env.lib.mgn_set_ablation(env.h, 0)
print(json.dumps({"order": order, "steps": F}))
