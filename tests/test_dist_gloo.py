"""world_size-2 gloo test of the sharded path (CPU).

Each rank runs its contiguous shard of the C3-family workload (the oracle
stands in for the device on a CPU host; the GPU equivalence of shards is
tests/test_gpu_parity.py::test_sharded_equals_unsharded), then the product's
all-gather of episode statistics assembles the global table.  Rank 0 checks
it against one unsharded run over all envs: sharding by global env index is
exact, so the tables must be identical.
"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from madigan_amd.distributed import allgather_episode_stats, shard, summarize

N_TOTAL, A, K = 37, 4, 60
PARAMS = [0.2, 2, 6, 0.05, 0.2, 5.0, 0.15, 0.3, 0.2, 0.99]


def _cfg(n, off):
    return dict(n_envs=n, env_offset=off, seed=5, required_margin=0.02, maintenance_margin=0.25,
                transaction_cost_rel=0.02, unit_size=0.9, auto_reset=1, init_cash=1e5)


def _actions(total):
    return np.random.default_rng(1).integers(0, 3, (K, total, A)).astype(np.int8)


def _stats(b):
    return np.stack([b.scalar(k) for k in ("last_ret", "last_len", "last_equity", "n_done")], 1)


def _worker(rank, world, port, q):
    from oracle import oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    off, n = shard(N_TOTAL, rank, world)
    b = O.OracleBatch(_cfg(n, off), [(O.SRC_TRENDOU, PARAMS)] * A)
    b.rollout(_actions(N_TOTAL)[:, off:off + n])
    gathered = allgather_episode_stats(torch.from_numpy(_stats(b)))
    if rank == 0:
        q.put(gathered.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_shard_partition():
    for world in (1, 2, 3, 8):
        spans = [shard(N_TOTAL, r, world) for r in range(world)]
        assert spans[0][0] == 0
        assert sum(n for _, n in spans) == N_TOTAL
        for (o1, n1), (o2, _) in zip(spans, spans[1:]):
            assert o1 + n1 == o2
    with pytest.raises(ValueError):
        shard(10, 2, 2)


def test_gloo_allgather_matches_unsharded():
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = O.OracleBatch(_cfg(N_TOTAL, 0), [(O.SRC_TRENDOU, PARAMS)] * A)
    full.rollout(_actions(N_TOTAL))
    ref = _stats(full)
    assert ref[:, 3].sum() > 0, "workload must complete episodes"
    assert np.array_equal(got.view(np.int64), ref.view(np.int64))
    s = summarize(torch.from_numpy(got))
    assert s["episodes"] == int(ref[:, 3].sum())


def test_nccl_without_communicator_fails_loudly(monkeypatch):
    """Over "nccl" the statistics all-gather is the C ABI's
    mgn_stats_allgather; a torch whose ProcessGroupNCCL hides the RCCL
    communicator raises instead of silently taking torch's all-gather."""
    from madigan_amd import distributed as D

    class NoComm:
        def _get_backend(self, dev):
            raise AttributeError("_comm_ptr")

    monkeypatch.setattr(dist, "get_backend", lambda g=None: "nccl")
    with pytest.raises(D.CollectiveUnavailable):
        D.rccl_comm(NoComm(), device=torch.device("cpu"))
    monkeypatch.setattr(dist, "get_backend", lambda g=None: "gloo")
    assert D.rccl_comm(NoComm(), device=torch.device("cpu")) == 0
