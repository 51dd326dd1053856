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


def broadcast_chip_set(chips, src=0, device=None):
    """Replicate a chip set (tessellate()'s columns) from rank `src` to every rank as raw buffers --
    one size message, then is_core, index_id, polygon_key, the WKB offsets and the WKB bytes, each a
    single broadcast -- instead of a pickled object (C4: 12 M chips, GBs of WKB).  The chip table is
    then built on every rank from identical columns (chips replicated per
    GPU).  `device`: where the collective's tensors live (a CUDA device for RCCL, None for gloo).
    Returns the chip set on every rank (numpy columns; on `src` the input itself)."""
    import numpy as np

    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return chips
    me = dist.get_rank()
    sizes = torch.zeros(2, dtype=torch.int64, device=device)
    if me == src:
        sizes[0] = len(chips["index_id"])
        sizes[1] = int(chips["wkb"][0][-1])
    dist.broadcast(sizes, src=src)
    n, nb = int(sizes[0]), int(sizes[1])
    cols = [("is_core", torch.uint8, n), ("index_id", torch.int64, n), ("polygon_key", torch.int32, n),
            ("wkb_offsets", torch.int64, n + 1), ("wkb", torch.uint8, nb)]
    out = {}
    for name, dt, m in cols:
        if me == src:
            src_arr = chips["wkb"][0] if name == "wkb_offsets" else (chips["wkb"][1][:nb] if name == "wkb" else chips[name])
            npdt = {torch.uint8: np.uint8, torch.int64: np.int64, torch.int32: np.int32}[dt]
            t = torch.from_numpy(np.ascontiguousarray(src_arr, dtype=npdt)).to(device) if m else torch.empty(0, dtype=dt, device=device)
        else:
            t = torch.empty(m, dtype=dt, device=device)
        if m:
            dist.broadcast(t, src=src)
        out[name] = t.cpu().numpy() if me != src else None
    if me == src:
        return chips
    return dict(is_core=out["is_core"], index_id=out["index_id"], polygon_key=out["polygon_key"],
                wkb=(out["wkb_offsets"], out["wkb"]))


def finalize():
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
