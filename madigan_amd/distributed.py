"""Multi-GPU sharding of the batched env (one process per GPU).

Envs are independent (no cross-env term anywhere on the step), so
N_total envs are split contiguously: rank r owns global envs
[offset_r, offset_r + n_r).  The generators key their Philox streams by the
global env index (``env_offset``), so a sharded run produces exactly the
per-env trajectories of a single-device run.  The only collective is an
all-gather of per-env episode statistics (RCCL over xGMI with the "nccl"
backend; gloo in CPU tests), issued at log intervals, never per step.
"""
from __future__ import annotations

from typing import Tuple


def shard(n_total: int, rank: int, world: int) -> Tuple[int, int]:
    """(env_offset, n_local) of rank's contiguous slice; remainders go to the
    lowest ranks so every rank's slice differs by at most one env."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, rem = divmod(int(n_total), world)
    n_local = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, n_local


def allgather_episode_stats(stats, group=None):
    """All-gather the (n_local, S) per-env episode statistics of every rank into
    (n_total, S) in global env order.  Equal shard sizes use one
    all_gather_into_tensor; ragged shards pad to the largest and trim."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return stats
    world = dist.get_world_size(group)
    n_local = torch.tensor([stats.shape[0]], dtype=torch.int64, device=stats.device)
    sizes = [torch.zeros_like(n_local) for _ in range(world)]
    dist.all_gather(sizes, n_local, group=group)
    sizes = [int(s.item()) for s in sizes]
    n_max = max(sizes)
    if stats.shape[0] < n_max:
        pad = torch.zeros((n_max - stats.shape[0],) + tuple(stats.shape[1:]), dtype=stats.dtype,
                          device=stats.device)
        stats = torch.cat([stats, pad])
    out = torch.empty((world * n_max,) + tuple(stats.shape[1:]), dtype=stats.dtype,
                      device=stats.device)
    dist.all_gather_into_tensor(out, stats.contiguous(), group=group)
    if all(s == n_max for s in sizes):
        return out
    return torch.cat([out[r * n_max:r * n_max + sizes[r]] for r in range(world)])


class CollectiveUnavailable(RuntimeError):
    """An "nccl" process group whose RCCL communicator cannot be reached, so
    the C ABI's mgn_stats_allgather cannot run on it."""


def rccl_comm(group=None, device=None) -> int:
    """The raw RCCL communicator (ncclComm_t) of a torch "nccl" process group,
    for mgn_stats_allgather; 0 for other backends (gloo).  Over "nccl" a
    communicator that cannot be reached raises CollectiveUnavailable -- it is
    taken through a private accessor of torch's ProcessGroupNCCL, and a torch
    without it must not silently route the sharded path's collective around
    the library."""
    import torch
    import torch.distributed as dist
    g = group if group is not None else dist.group.WORLD
    if dist.get_backend(g) != "nccl":
        return 0
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    try:
        comm = int(g._get_backend(dev)._comm_ptr())
    except (AttributeError, RuntimeError) as e:
        raise CollectiveUnavailable(
            "nccl process group without a reachable RCCL communicator (ProcessGroupNCCL._comm_ptr): "
            f"{e!r}; pass allow_torch_fallback=True to all-gather through torch.distributed") from e
    if not comm:
        raise CollectiveUnavailable("nccl process group returned a null RCCL communicator")
    return comm


# which path the last allgather_env_stats took: "mgn_stats_allgather" (the
# C ABI's ncclAllGather on the caller's RCCL communicator), "torch" (torch's
# all-gather: gloo, or nccl with allow_torch_fallback), "local" (one process)
last_allgather_path = None


def allgather_env_stats(env, n_total=None, group=None, allow_torch_fallback=False):
    """All-gather a BatchedEnv's (N_local, 4) episode statistics into
    (n_total, 4) in global env order.  Over "nccl" the collective is the C
    ABI's mgn_stats_allgather on the handle's stream (one ncclAllGather of
    ceil(n_total / world) rows per rank; ragged shards are zero-padded by the
    library and trimmed here); gloo uses torch's all-gather.  An nccl group
    whose communicator cannot be reached raises CollectiveUnavailable unless
    allow_torch_fallback.  The path taken is recorded in
    ``last_allgather_path``.  With n_total given (the shard() partition) no
    size exchange is needed."""
    import ctypes as C
    import torch
    import torch.distributed as dist
    from . import _lib as L
    global last_allgather_path
    stats = env.episode_stats
    if not (dist.is_available() and dist.is_initialized()):
        last_allgather_path = "local"
        return stats
    world = dist.get_world_size(group)
    try:
        comm = rccl_comm(group, env.device)
    except CollectiveUnavailable:
        if not allow_torch_fallback:
            raise
        comm = 0
    if not comm:
        last_allgather_path = "torch"
        return allgather_episode_stats(stats.cpu() if dist.get_backend(group) == "gloo" else stats,
                                       group)
    last_allgather_path = "mgn_stats_allgather"
    if n_total is None:
        n = torch.tensor([env.N], dtype=torch.int64, device=env.device)
        sizes = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(sizes, n, group=group)
        sizes = [int(s.item()) for s in sizes]
    else:
        sizes = [shard(n_total, r, world)[1] for r in range(world)]
    rows = max(sizes)
    out = torch.empty((world * rows, 4), dtype=torch.float64, device=env.device)
    L.check(env.lib.mgn_stats_allgather(env.h, C.c_void_p(comm), rows, C.c_void_p(out.data_ptr())),
            env.h)
    if all(s == rows for s in sizes):
        return out
    return torch.cat([out[r * rows:r * rows + sizes[r]] for r in range(world)])


def summarize(stats):
    """Episode summary over all envs from gathered (n_total, 4) statistics:
    {last return, last length, last final equity, done count}."""
    import torch
    done = stats[:, 3] > 0
    n = int(done.sum().item())
    if n == 0:
        return {"episodes": int(stats[:, 3].sum().item()), "mean_return": float("nan"),
                "mean_length": float("nan"), "mean_final_equity": float("nan")}
    return {"episodes": int(stats[:, 3].sum().item()),
            "mean_return": float(stats[done, 0].mean().item()),
            "mean_length": float(stats[done, 1].mean().item()),
            "mean_final_equity": float(stats[done, 2].mean().item()),
            "envs_with_episode": n, "std_return": float(torch.std(stats[done, 0]).item())
            if n > 1 else 0.0}
