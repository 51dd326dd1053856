"""BASELINE.json configs at (or near) full size on one MI355X, checked against the oracle.

* C1 (configs[0], the Quickstart shape): 1e7 points -- 80 % Gaussian mixture around
  32 zone centres (sigma 0.005 deg), 20 % uniform, rounded to 1e-6 deg like the taxi GPS -- plus 0.1 %
  adversarial points on the zones' vertices and edge midpoints, the 263 zones tessellated at H3 res
  9: cells of every point, counts and pairs equal the oracle's; the WKT geometry column of the first
  1e6 points gives the same cells (grid_pointascellid over pickup_geom, QuickstartNotebook.py:162-165).
* C2 (configs[1], the bench workload): 1e9 uniform points over the NYC bbox, 263 zones at H3 res 9.
  Counts of the point-raster path (k_join_stream) equal those of the generic path (tile directory
  and point raster off: hash probe + per-chip rasters) on all 1e9 points, and the oracle's on a
  1e8-point prefix (reference: the Quickstart count, notebooks/examples/python/
  QuickstartNotebook.py:207-219).
* C3 shape: all 263 zones at H3 res 10 (grid_tessellateexplode on the GPU), clustered points
  (sigma 0.002 deg) -- counts equal the oracle's.
* C4 shape at scale: 1e6 OSM-style buildings chipped at H3 res 11 (~2.4 M chips), 1e7 points
  (70 % near buildings) -- counts equal the oracle's.
Full size (VERDICT r2 "full-size checks"), each the raster / dense-table path against the generic
path (tile directory and point raster off) on every point plus the oracle on a prefix:
* C3: 1e9 clustered device points (80 % around 32 zone centres, sigma 0.002 deg), all 263 zones at
  H3 res 10; oracle on the first 1e8.
* C5: 1e9 uniform points over the 177 London postcode zones in EPSG:27700, BNG res 4 (dense cell
  table + LDS cell level + line records); oracle on the first 1e8.
* C4: 5e6 buildings chipped at H3 res 11, 2.5e8 points (70 % within 25 m of a building); oracle on
  the first 1e7 (reference: notebooks/examples/python/QuickstartNotebook.py:207-219).
Runs on the MI355X box only.
"""
import numpy as np
import pytest

import oracle
from mosaic_amd import MosaicContext
from mosaic_amd.data import PolygonSet

pytestmark = pytest.mark.gpu


def chips_to_oracle(chips):
    offs, data = chips["wkb"]
    return dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
                wkb_offsets=offs, wkb=data)


@pytest.fixture(scope="module")
def h3ctx():
    ctx = MosaicContext.build("H3", "JTS")
    yield ctx
    ctx.close()


@pytest.fixture(scope="module")
def zones():
    return PolygonSet.load("nyc_taxi_zones")


def test_c1_quickstart_shape_vs_oracle(h3ctx, zones):
    from mosaic_amd.data import quickstart_points

    chips = h3ctx.grid_tessellateexplode(zones, 9)
    table = h3ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 9,
                             n_polygons=len(zones))
    x, y = quickstart_points(zones, 10_000_000, config=1)
    # 0.1 %: zone vertices and edge midpoints (boundary points: JTS leaves them out of both zones)
    rng = np.random.default_rng(1)
    vi = rng.choice(len(zones.xy) - 1, 5_000, replace=False)
    vx, vy = zones.xy[vi, 0], zones.xy[vi, 1]
    mx, my = 0.5 * (zones.xy[vi, 0] + zones.xy[vi + 1, 0]), 0.5 * (zones.xy[vi, 1] + zones.xy[vi + 1, 1])
    x = np.concatenate([x, vx, mx])
    y = np.concatenate([y, vy, my])
    perm = rng.permutation(len(x))
    x, y = np.ascontiguousarray(x[perm]), np.ascontiguousarray(y[perm])
    cells = h3ctx.grid_longlatascellid(x, y, 9, raw=True)
    assert np.array_equal(cells, oracle.h3_point_to_index(x, y, 9))
    oc = chips_to_oracle(chips)
    want, total, orow, okey = oracle.pip_join(oc, oracle.GRID_H3, 9, x, y, len(zones), pairs=True, threads=16)
    assert total > 6e6
    assert np.array_equal(h3ctx.pip_join_count(table, x, y), want)
    rows, keys = h3ctx.pip_join_pairs(table, x, y)
    o = np.lexsort((okey, orow))
    assert np.array_equal(rows, orow[o]) and np.array_equal(keys, okey[o])
    m = 1_000_000
    wkt = [f"POINT ({a!r} {b!r})" for a, b in zip(x[:m].tolist(), y[:m].tolist())]
    assert np.array_equal(h3ctx.grid_pointascellid(wkt, 9, raw=True), cells[:m])
    table.close()


def test_c2_full_size_raster_vs_generic_vs_oracle(h3ctx, zones):
    import torch

    from mosaic_amd.data import SEED_BASE, uniform_points_device

    chips = h3ctx.grid_tessellateexplode(zones, 9)
    table = h3ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 9,
                             n_polygons=len(zones))
    assert table.tiles()["stream"] == 1
    n = 1_000_000_000
    x, y = uniform_points_device(zones.bbox(), n, seed=SEED_BASE + 2, device=torch.device("cuda:0"))
    fast = h3ctx.pip_join_count(table, x, y).cpu().numpy()
    try:
        h3ctx.set_option("tiles", 0)
        h3ctx.set_option("point_raster", 0)
        generic = h3ctx.pip_join_count(table, x, y).cpu().numpy()
    finally:
        h3ctx.set_option("tiles", 1)
        h3ctx.set_option("point_raster", 1)
    assert fast.sum() > 3e8
    assert np.array_equal(fast, generic)
    m = 100_000_000
    prefix = h3ctx.pip_join_count(table, x[:m], y[:m]).cpu().numpy()
    hx, hy = x[:m].cpu().numpy(), y[:m].cpu().numpy()
    del x, y
    torch.cuda.empty_cache()
    want, total = oracle.pip_join(chips_to_oracle(chips), oracle.GRID_H3, 9, hx, hy, len(zones), threads=16)
    assert np.array_equal(prefix, want) and total > 3e7
    table.close()


def test_c3_all_zones_res10_vs_oracle(h3ctx, zones):
    from mosaic_amd.data import quickstart_points

    chips = h3ctx.grid_tessellateexplode(zones, 10)
    table = h3ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 10,
                             n_polygons=len(zones))
    t = table.tiles()
    assert t["raster"] == 1 and t["stream"] == 1, t
    x, y = quickstart_points(zones, 4_000_000, sigma=0.002, seed=103)
    want, total = oracle.pip_join(chips_to_oracle(chips), oracle.GRID_H3, 10, x, y, len(zones), threads=16)
    assert total > 1_000_000
    assert np.array_equal(h3ctx.pip_join_count(table, x, y), want)
    table.close()


def test_c4_million_buildings_vs_oracle(h3ctx):
    import torch

    from mosaic_amd.data import building_points_device, synthetic_buildings

    nb = 1_000_000
    b = synthetic_buildings(nb, bbox=(-74.05, 40.60, -73.80, 40.85), n_centres=64, sigma=0.02)
    chips = h3ctx.grid_tessellateexplode(b, 11)
    assert len(chips["index_id"]) > 1_500_000
    table = h3ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 11,
                             n_polygons=nb)
    xd, yd = building_points_device(b, 10_000_000, seed=79)
    got = h3ctx.pip_join_count(table, xd, yd).cpu().numpy()
    x, y = xd.cpu().numpy(), yd.cpu().numpy()
    del xd, yd
    torch.cuda.empty_cache()
    want, total = oracle.pip_join(chips_to_oracle(chips), oracle.GRID_H3, 11, x, y, nb, threads=16)
    assert total > 1_000_000
    assert np.array_equal(got, want)
    table.close()


def _fast_vs_generic(ctx, table, x, y):
    """Counts of the default path and of the generic path (tile directory / dense table and point
    raster off: hash probe + per-chip rasters) on the same device points."""
    fast = ctx.pip_join_count(table, x, y).cpu().numpy()
    try:
        ctx.set_option("tiles", 0)
        ctx.set_option("point_raster", 0)
        generic = ctx.pip_join_count(table, x, y).cpu().numpy()
    finally:
        ctx.set_option("tiles", 1)
        ctx.set_option("point_raster", 1)
    return fast, generic


def _oracle_prefix(ctx, table, chips, grid, res, x, y, m, n_polygons):
    import torch

    got = ctx.pip_join_count(table, x[:m], y[:m]).cpu().numpy()
    hx, hy = x[:m].cpu().numpy(), y[:m].cpu().numpy()
    torch.cuda.empty_cache()
    want, total = oracle.pip_join(chips_to_oracle(chips), grid, res, hx, hy, n_polygons, threads=16)
    return got, want, total


def test_c3_full_size_clustered_res10(h3ctx, zones):
    import torch

    from mosaic_amd.data import SEED_BASE, clustered_points_device

    chips = h3ctx.grid_tessellateexplode(zones, 10)
    table = h3ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 10,
                             n_polygons=len(zones))
    t = table.tiles()
    assert t["raster"] == 1 and t["stream"] == 1, t
    n = 1_000_000_000
    x, y = clustered_points_device(zones, n, seed=SEED_BASE + 3, sigma=0.002, device=torch.device("cuda:0"))
    fast, generic = _fast_vs_generic(h3ctx, table, x, y)
    assert fast.sum() > 5e8
    assert np.array_equal(fast, generic)
    got, want, total = _oracle_prefix(h3ctx, table, chips, oracle.GRID_H3, 10, x, y, 100_000_000, len(zones))
    del x, y
    torch.cuda.empty_cache()
    assert total > 5e7 and np.array_equal(got, want)
    table.close()


def test_c5_full_size_bng_res4():
    import torch

    from mosaic_amd.context import tessellate
    from mosaic_amd.data import uniform_points_device

    proj = PolygonSet.load("london_postcodes_bng")
    assert len(proj) == 177
    ctx = MosaicContext.build("BNG")
    try:
        chips = tessellate("BNG", proj, 4)
        table = ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 4,
                               n_polygons=len(proj))
        assert table.tiles()["built"] == 1
        n = 1_000_000_000
        x, y = uniform_points_device(proj.bbox(), n, seed=5, device=torch.device("cuda:0"))
        fast, generic = _fast_vs_generic(ctx, table, x, y)
        assert fast.sum() > 3e8
        assert np.array_equal(fast, generic)
        got, want, total = _oracle_prefix(ctx, table, chips, oracle.GRID_BNG, 4, x, y, 100_000_000, len(proj))
        del x, y
        torch.cuda.empty_cache()
        assert total > 3e7 and np.array_equal(got, want)
        table.close()
    finally:
        ctx.close()


def test_c4_full_size_five_million_buildings(h3ctx):
    import time

    import torch

    from mosaic_amd.data import building_points_device, synthetic_buildings

    nb = 5_000_000
    b = synthetic_buildings(nb, bbox=(-74.05, 40.60, -73.80, 40.85), n_centres=320, sigma=0.02)
    t0 = time.perf_counter()
    chips = h3ctx.grid_tessellateexplode(b, 11)
    t_tess = time.perf_counter() - t0
    assert len(chips["index_id"]) > 7_500_000
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    t0 = time.perf_counter()
    table = h3ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 11,
                             n_polygons=nb)
    t_table = time.perf_counter() - t0
    dev_bytes = free0 - torch.cuda.mem_get_info()[0]
    print(f"C4 full size: {len(chips['index_id'])} chips, tessellate {t_tess:.2f} s, table {t_table:.2f} s, "
          f"device {dev_bytes / 2**30:.2f} GiB, info {table.info()}")
    n = 250_000_000
    x, y = building_points_device(b, n, seed=81)
    fast, generic = _fast_vs_generic(h3ctx, table, x, y)
    assert fast.sum() > 5e7
    assert np.array_equal(fast, generic)
    got, want, total = _oracle_prefix(h3ctx, table, chips, oracle.GRID_H3, 11, x, y, 10_000_000, nb)
    del x, y
    torch.cuda.empty_cache()
    assert total > 2e6 and np.array_equal(got, want)
    table.close()
