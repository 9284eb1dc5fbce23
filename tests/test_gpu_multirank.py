"""The bench's multi-rank path rehearsed on the one leased GPU (VERDICT r1
#9): `torch.distributed.run --nproc-per-node 2 bench.py --dist-backend gloo`
puts two ranks on the same device, each stepping its contiguous shard
(env_offset = rank * N) and all-gathering the (N, 4) episode statistics;
rank 0's gathered table must equal one unsharded run over both shards'
envs bit for bit (same launches, same global-env-keyed actions and
variates).  Covers the sharding offsets, the gather order and the elapsed
MAX-reduce of bench.py."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("launcher", ["torchrun", "spawn"])
def test_bench_two_ranks_gloo_matches_unsharded(gpu, tmp_path, launcher):
    """launcher "spawn": `bench.py --gpus 2` with no launcher starts its two
    ranks itself (bench.spawn_ranks) -- the form of the driver's scaling run."""
    N, steps, warmup = 512, 1000, 24  # first margin-call dones come after ~500 steps
    dump = str(tmp_path / "stats.npy")
    port = 29600 + os.getpid() % 300
    pre = ([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
            "--master-addr", "127.0.0.1", "--master-port", str(port)] if launcher == "torchrun"
           else [sys.executable])
    cmd = pre + [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", str(steps), "--warmup", str(warmup), "--n-envs", str(N),
           "--dist-backend", "gloo", "--no-cpu-baseline", "--no-probe", "--dump-stats", dump]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 2 and res["value"] > 0
    assert res["config"]["n_envs_total"] == 2 * N
    got = np.load(dump)
    assert got.shape == (2 * N, 4)

    sys.path.insert(0, ROOT)
    import bench
    from madigan_amd import BatchedEnv
    from madigan_amd.config import trendou_spec
    spec = trendou_spec(*[[p] * 8 for p in bench.TRENDOU_P])
    full = BatchedEnv(spec, 2 * N, seed=0x6D6164 + 3, env_offset=0, **bench.c3_kwargs())
    acts = full.generate_actions(warmup + steps, seed=0x6D6164)
    full.rollout(acts[:warmup])
    full.rollout(acts[warmup:])
    ref = full.episode_stats.cpu().numpy()
    assert ref[:, 3].sum() > 0, "the run should complete episodes"
    assert np.array_equal(got.view(np.int64), ref.view(np.int64))
