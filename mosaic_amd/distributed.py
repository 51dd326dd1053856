"""Multi-GPU plumbing for the chip join: one process per GPU, torch.distributed over RCCL.

The path shards naturally: every point is independent, chips are
replicated on every GPU, and the only exchange is one all-reduce of the per-polygon int64 counts
(P = 263 for the NYC zones: a latency-bound 2 KB message over xGMI).  Backend "nccl" is RCCL on
ROCm; "gloo" is used for CPU tests of the same code path.
"""
import os

import torch
import torch.distributed as dist


def env_ranks():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend=None):
    """Initialise the process group from the torchrun environment; returns (rank, world, local_rank)."""
    rank, world, local = env_ranks()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def shard_bounds(n_total, rank, world):
    """Contiguous [lo, hi) point range owned by `rank` (sizes differ by at most one)."""
    base, extra = divmod(int(n_total), int(world))
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def allreduce_counts(counts):
    """Sum per-polygon counts over ranks in place (no-op for a single process)."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(counts, op=dist.ReduceOp.SUM)
    return counts


def max_over_ranks(value, device=None):
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sharded_join_count(count_fn, x, y, n_polygons, device=None):
    """Run count_fn(x_shard, y_shard) -> int64[n_polygons] on this rank's shard of (x, y) and
    all-reduce.  x, y are the full arrays (the caller may instead pass pre-sharded arrays with
    world == 1 semantics by not initialising a group)."""
    rank, world = (dist.get_rank(), dist.get_world_size()) if dist.is_initialized() else (0, 1)
    lo, hi = shard_bounds(len(x), rank, world)
    local = count_fn(x[lo:hi], y[lo:hi])
    counts = torch.as_tensor(local, dtype=torch.int64, device=device).clone()
    allreduce_counts(counts)
    return counts[:n_polygons]


def finalize():
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
