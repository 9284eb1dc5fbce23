import numpy as np, torch, sys
sys.path.insert(0, '.')
from madigan_amd import BatchedEnv, _lib as L
from madigan_amd.config import trendou_spec
P = [0.02, 100, 500, 0.001, 0.005, 5.0, 0.15, 0.04, 0.001, 0.99]
kw = dict(required_margin=1.0, maintenance_margin=0.25, slippage_rel=1e-4, transaction_cost_rel=0.02,
          reward_shaper="DDR", adaptation_rate=0.001, unit_size=0.05, auto_reset=True)
g = BatchedEnv(trendou_spec(*[[p] * 8 for p in P]), 100, seed=1, **kw)
print("sched", g.lib.mgn_get_schedule(g.h), flush=True)
a = g.generate_actions(4, seed=2)
o = g.rollout(a); torch.cuda.synchronize(); print("duo ok", o["reward"][0, :4].tolist(), flush=True)
