"""The point raster classified on the GPU (k_raster_sub / k_raster_line / k_raster_cells, option
"raster_build" = 1, the default) is byte-identical to the host-thread build (option 0) -- the
build whose every pure code tests/test_raster_selfcheck.py checks against the exact answer -- and
joins to the oracle's counts.  Runs on the MI355X box only."""
import numpy as np
import pytest

import oracle
from mosaic_amd import MosaicContext
from mosaic_amd.context import tessellate
from mosaic_amd.data import PolygonSet, quickstart_points

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = MosaicContext.build("H3", "JTS")
    yield c
    c.close()


@pytest.fixture(scope="module")
def zones():
    return PolygonSet.load("nyc_taxi_zones")


def _build(ctx, chips, res, npoly, gpu, **opts):
    ctx.set_option("raster_build", 1 if gpu else 0)
    for k, v in opts.items():
        ctx.set_option(k, v)
    try:
        return ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], res,
                              n_polygons=npoly)
    finally:
        ctx.set_option("raster_build", 1)
        for k in opts:
            ctx.set_option(k, {"raster_sub": 64, "raster_cell": 16, "raster_lines": 1, "raster_leaf_lines": 1}[k])


@pytest.mark.parametrize("res,ids,opts", [
    (9, None, {}),
    (10, None, {}),
    (8, None, {"raster_lines": 0}),
    (10, range(0, 263, 5), {"raster_sub": 16, "raster_cell": 8}),
    (11, range(0, 263, 29), {"raster_sub": 32, "raster_cell": 4}),
    (9, None, {"raster_leaf_lines": 0}),
    (10, range(0, 263, 5), {"raster_sub": 16, "raster_cell": 8, "raster_leaf_lines": 1}),
])
def test_gpu_raster_equals_host_raster(ctx, zones, res, ids, opts):
    z = zones if ids is None else zones.subset(list(ids))
    chips = tessellate("H3", z, res)
    tg = _build(ctx, chips, res, len(z), True, **opts)
    th = _build(ctx, chips, res, len(z), False, **opts)
    ig, ih = tg.build_info(), th.build_info()
    sg, sh = tg.tiles(), th.tiles()
    assert sg["raster"] == 1 and sg == sh, (sg, sh)
    assert ig["raster_digest"] != 0 and ig["raster_digest"] == ih["raster_digest"], (ig, ih)
    print(f"res {res} zones {len(z)} {opts}: classify GPU {ig['raster_classify_ms']:.1f} ms host "
          f"{ih['raster_classify_ms']:.1f} ms, assemble {ig['raster_assemble_ms']:.1f} ms, directory "
          f"{ig['directory_ms']:.1f} ms, core {ig['core_ms']:.1f} ms")
    x, y = quickstart_points(z, 300_000, sigma=0.002, seed=res)
    offs, data = chips["wkb"]
    oc = dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
              wkb_offsets=offs, wkb=data)
    want, total = oracle.pip_join(oc, oracle.GRID_H3, res, x, y, len(z), threads=8)
    assert total > 10_000
    assert np.array_equal(ctx.pip_join_count(tg, x, y), want)
    tg.close()
    th.close()


def test_leaf_lines_join(ctx, zones):
    """Leaf lines (option raster_leaf_lines): the stream kernels send leaf-line rows to the mixed
    queue, k_join_leaf answers them from the line record (option leaf_join) and passes the rest on to
    k_join_mixed.  Counts and pairs equal the oracle's with k_join_leaf on and off, on uniform points
    plus points on and next to chip vertices and segments (the line bands)."""
    import torch

    from tests.test_gpu_parity import _chip_boundary_points

    chips = tessellate("H3", zones, 9)
    t = _build(ctx, chips, 9, len(zones), True, raster_leaf_lines=1)
    try:
        info = t.tiles()
        assert info["leaf_lines"] > 100_000 and info["stream"] == 1, info
        rng = np.random.default_rng(41)
        x0, y0, x1, y1 = zones.bbox()
        bx, by = _chip_boundary_points(chips, rng)
        x = np.concatenate([rng.uniform(x0, x1, 2_000_000), bx])
        y = np.concatenate([rng.uniform(y0, y1, 2_000_000), by])
        offs, data = chips["wkb"]
        oc = dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
                  wkb_offsets=offs, wkb=data)
        want, _, orow, okey = oracle.pip_join(oc, oracle.GRID_H3, 9, x, y, len(zones), pairs=True, threads=8)
        want_pairs = np.sort(orow.astype(np.int64) * len(zones) + okey)
        xd, yd = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
        tests = {}
        for lj in (0, 1):
            ctx.set_option("leaf_join", lj)
            got = ctx.pip_join_count(t, xd, yd)
            assert ctx.last_kernel() == "k_join_stream_cpt"
            assert np.array_equal(got.cpu().numpy(), want), lj
            tests[lj] = ctx.last_stats()["contains_tests"]
            rows, keys = ctx.pip_join_pairs(t, xd, yd)
            rows = rows.cpu().numpy() if hasattr(rows, "cpu") else rows
            keys = keys.cpu().numpy() if hasattr(keys, "cpu") else keys
            assert np.array_equal(np.sort(rows.astype(np.int64) * len(zones) + keys), want_pairs), lj
        # the leaf-line rows no longer reach the chip loop (most of these points lie on chip
        # boundaries, in the bands, and still do)
        assert tests[1] < tests[0], tests
    finally:
        ctx.set_option("leaf_join", 1)
        t.close()
