"""C5 step-launch probe (diagnostic): how much of C5's 64-step launch is the
auto-reset refill tail?  Times mgn_rollout_hist (HIP events on the handle's
stream) for the bench's C5 env and for variants with fewer episode ends
(transaction cost 0) or shorter refills (W = 8), and counts episode ends.

    python tools/c5_probe.py [--launches 6]
"""
import argparse
import ctypes as C
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=6)
    ap.add_argument("--warm", type=int, default=8)
    a = ap.parse_args()
    import torch
    import bench
    from madigan_amd import BatchedEnv, _lib as L
    from madigan_amd.config import spec_from_config
    N, A, T, K = 8192, 16, 200_000, 64
    dev = torch.device("cuda:0")
    path = os.path.join(tempfile.mkdtemp(), "c5.h5")
    bench.c5_replay_file(A, T, path)
    cfg = {"data_source_type": "HDFSourceSingle",
           "data_source_config": {"filepath": path, "group_key": "synth/ou", "price_key": "price",
                                  "feature_key": "features", "timestamp_key": "timestamps",
                                  "cache_size": 10_000}}
    spec = spec_from_config(cfg)
    base = dict(required_margin=1.0, maintenance_margin=0.25, transaction_cost_rel=0.02, unit_size=0.05,
                auto_reset=True, init_cash=1_000_000.0, window=64, adaptation_rate=0.001,
                reward_shaper="DDR", seed=0x6D6164 + 5)
    variants = [("C5", {}), ("C5_cost0", {"transaction_cost_rel": 0.0}), ("C5_W8", {"window": 8}),
                ("C5_W8_cost0", {"window": 8, "transaction_cost_rel": 0.0})]
    res = {}
    for name, over in variants:
        kw = dict(base, **over)
        env = BatchedEnv(spec, N, device=dev, replay_stride=997, **kw)
        lib, h = env.lib, env.h
        total = (a.warm + a.launches) * K
        acts = env.generate_actions(total, seed=0x6D6164)
        traj = env.alloc_traj(K, fields=["reward", "done"])
        ts = C.byref(env._traj_struct(traj))
        per = N * A
        for l in range(a.warm):
            L.check(lib.mgn_rollout_hist(h, C.c_void_p(acts.data_ptr() + l * K * per), K, ts), h)
        torch.cuda.synchronize()
        L.check(lib.mgn_set_timing(h, 1), h)
        ends = 0
        for l in range(a.warm, a.warm + a.launches):
            L.check(lib.mgn_rollout_hist(h, C.c_void_p(acts.data_ptr() + l * K * per), K, ts), h)
            ends += int(traj["done"].sum().item())
        torch.cuda.synchronize()
        tm = (C.c_double * 4)()
        L.check(lib.mgn_get_timing(h, tm), h)
        L.check(lib.mgn_set_timing(h, 0), h)
        us = tm[0] / max(tm[1], 1) * 1e3
        res[name] = {"step_launch_us": us, "us_per_step": us / K, "launches": int(tm[1]),
                     "episode_ends_per_env_step": ends / (N * K * a.launches),
                     "schedule": int(lib.mgn_get_schedule(h))}
        print(name, json.dumps(res[name]), flush=True)
        del env, traj
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
