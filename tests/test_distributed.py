"""Multi-process (gloo, world_size 2) test of the sharded join + count all-reduce (CPU only).

Each rank runs the join on its contiguous shard of the points -- here with the CPU oracle standing
in for the GPU kernel, since this container has no GPU -- and the per-polygon counts are summed
with one all-reduce: the result must equal the single-process join over all points.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import oracle
    from mosaic_amd import distributed as D
    from mosaic_amd.data import PolygonSet, quickstart_points
    from tests.helpers import chips_to_oracle, synthetic_chips

    D.init("gloo")
    zones = PolygonSet.load("nyc_taxi_zones_35")
    rng = np.random.default_rng(0)
    ids = list(range(35))
    chips = synthetic_chips(zones, ids, 9, lambda a, b, r: oracle.h3_point_to_index(a, b, r), rng, pts_per_zone=60)
    oc = chips_to_oracle(chips)
    x, y = quickstart_points(zones, 40_000, seed=3)
    counts = D.sharded_join_count(lambda xs, ys: oracle.pip_join(oc, oracle.GRID_H3, 9, xs, ys, 35)[0], x, y, 35)
    lo, hi = D.shard_bounds(len(x), rank, world)
    elapsed = D.max_over_ranks(float(rank + 1))
    if rank == 0:
        full, _ = oracle.pip_join(oc, oracle.GRID_H3, 9, x, y, 35)
        q.put((counts.numpy().tolist(), full.tolist(), elapsed, hi - lo))
    D.finalize()


def test_shard_bounds():
    from mosaic_amd.distributed import shard_bounds

    for n in (0, 1, 7, 100, 10**9 + 3):
        for w in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1


@pytest.mark.timeout(300)
def test_gloo_world2_sharded_join_equals_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, want, elapsed, shard = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == want
    assert elapsed == 2.0  # max over ranks
    assert shard == 20_000


class _HostTessellator:
    """Stands in for the GPU context in bench.build_chips on CPU: the host producer."""

    def grid_tessellateexplode(self, zones, res):
        from mosaic_amd.context import tessellate

        return tessellate("H3", zones, res)


def _bench_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from mosaic_amd import distributed as D

    D.init("gloo")
    # only rank 0 may tessellate: the other ranks get the chip rows over the process group
    ctx = _HostTessellator() if rank == 0 else None
    zones, chips, _ = bench.build_chips(ctx, 9, rank, world)
    offs, data = chips["wkb"]
    q.put((rank, len(zones), chips["index_id"].tobytes(), chips["is_core"].tobytes(),
           chips["polygon_key"].tobytes(), bytes(np.asarray(offs).tobytes()), bytes(np.asarray(data).tobytes())))
    D.finalize()


@pytest.mark.timeout(300)
def test_gloo_world2_bench_chip_broadcast():
    """bench.py's multi-rank build: rank 0 tessellates the 263 zones and
    broadcasts the chip set; every rank ends with identical chip rows (ids, is_core, keys, WKB)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict((r[0], r[1:]) for r in (q.get(timeout=240), q.get(timeout=240)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0] == got[1]
    assert got[0][0] == 263 and len(got[0][1]) > 8 * 10_000


def _c4_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch

    from mosaic_amd import distributed as D
    from mosaic_amd.context import tessellate
    from mosaic_amd.data import synthetic_buildings

    D.init("gloo")
    # C4's shape at CPU-test scale: building footprints chipped at res 11 (all border chips), the
    # chip set replicated from rank 0 as raw buffers
    chips = None
    if rank == 0:
        b = synthetic_buildings(20_000, bbox=(-74.02, 40.70, -73.95, 40.77), n_centres=8, sigma=0.01)
        chips = tessellate("H3", b, 11)
    got = D.broadcast_chip_set(chips, src=0)
    offs, data = got["wkb"]
    digest = (got["index_id"].tobytes(), got["is_core"].tobytes(), got["polygon_key"].tobytes(),
              np.asarray(offs).tobytes(), np.asarray(data[:offs[-1]]).tobytes())
    # C4's count exchange: int64[5e6] per-building counts, one all-reduce
    P = 5_000_000
    counts = torch.arange(P, dtype=torch.int64) * (rank + 1)
    D.allreduce_counts(counts)
    ok = bool(torch.equal(counts, torch.arange(P, dtype=torch.int64) * 3))
    import hashlib
    q.put((rank, hashlib.sha256(b"".join(digest)).hexdigest(), len(got["index_id"]), ok))
    D.finalize()


@pytest.mark.timeout(300)
def test_gloo_world2_c4_chip_set_and_counts():
    """C4's multi-GPU shape: a building-scale chip set replicated as raw
    buffers (no pickling) arrives byte-identical on every rank, and the per-building int64 counts
    (P = 5e6, 40 MB) are summed with one all-reduce."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c4_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict((r[0], r[1:]) for r in (q.get(timeout=240), q.get(timeout=240)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0] == got[1]
    assert got[0][1] > 20_000 and got[0][2]
