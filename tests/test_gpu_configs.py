"""BASELINE.json configs at (or near) full size on one MI355X, checked against the oracle.

* C2 (configs[1], the bench workload): 1e9 uniform points over the NYC bbox, 263 zones at H3 res 9.
  Counts of the point-raster path (k_join_stream) equal those of the generic path (tile directory
  and point raster off: hash probe + per-chip rasters) on all 1e9 points, and the oracle's on a
  1e8-point prefix (reference: the Quickstart count, notebooks/examples/python/
  QuickstartNotebook.py:207-219).
* C3 shape: all 263 zones at H3 res 10 (grid_tessellateexplode on the GPU), clustered points
  (sigma 0.002 deg) -- counts equal the oracle's.
* C4 shape at scale: 1e6 OSM-style buildings chipped at H3 res 11 (~2.4 M chips), 1e7 points
  (70 % near buildings) -- counts equal the oracle's.
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
