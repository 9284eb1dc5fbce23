"""bench.py's rank launcher (CPU, no GPU call): `bench.py --gpus N` without a
launcher starts N ranks itself, each with RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR 127.0.0.1 / MASTER_PORT, and a launcher's WORLD_SIZE that
differs from --gpus is refused.  The ranks' data path (gathered statistics ==
the unsharded run) is tests/test_gpu_multirank.py's, through both launchers."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def clean_env(**kw):
    env = dict(os.environ, **kw)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        if k not in kw:
            env.pop(k, None)
    return env


def test_spawn_starts_every_rank():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--dist-backend", "gloo", "--rank-probe"],
                       capture_output=True, text=True, timeout=120, env=clean_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1, 2, 3]
    assert {d["world"] for d in lines} == {4}
    assert all(d["local_rank"] == d["rank"] for d in lines)
    masters = {d["master"] for d in lines}
    assert len(masters) == 1 and masters.pop().startswith("127.0.0.1:")


def test_one_rank_runs_in_process():
    r = subprocess.run([sys.executable, BENCH, "--rank-probe"], capture_output=True, text=True, timeout=120,
                       env=clean_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["rank"] == 0 and d["world"] == 1


def test_launcher_world_mismatch_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--rank-probe"], capture_output=True, text=True,
                       timeout=120, env=clean_env(WORLD_SIZE="2", RANK="0"), cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_nccl_needs_a_gpu_per_rank():
    """--dist-backend nccl (RCCL) with fewer visible GPUs than ranks: refused by
    the parent before any rank starts (this container has none)."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--rank-probe"], capture_output=True, text=True,
                       timeout=120, env=clean_env(), cwd=ROOT)
    assert r.returncode == 2 and "one rank per GPU" in r.stderr
