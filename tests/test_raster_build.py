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
            ctx.set_option(k, {"raster_sub": 64, "raster_cell": 16, "raster_lines": 1}[k])


@pytest.mark.parametrize("res,ids,opts", [
    (9, None, {}),
    (10, None, {}),
    (8, None, {"raster_lines": 0}),
    (10, range(0, 263, 5), {"raster_sub": 16, "raster_cell": 8}),
    (11, range(0, 263, 29), {"raster_sub": 32, "raster_cell": 4}),
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
