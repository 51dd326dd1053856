"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the same inputs.

Bit-exact for cell ids, contains booleans, join counts and pairs.  Runs on the MI355X box only.
"""
import json
import math
import os

import numpy as np
import pytest

import oracle
from mosaic_amd import IllegalStateException, MosaicContext
from mosaic_amd import wkb as W
from mosaic_amd.data import PolygonSet, quickstart_points

from .helpers import boundary_points, chips_to_oracle, synthetic_chips

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_vectors.json")))


@pytest.fixture(scope="module")
def h3ctx():
    ctx = MosaicContext.build("H3", "JTS")
    yield ctx
    ctx.close()


@pytest.fixture(scope="module")
def bngctx():
    ctx = MosaicContext.build("BNG", "JTS")
    yield ctx
    ctx.close()


@pytest.fixture(scope="module")
def zones():
    return PolygonSet.load("nyc_taxi_zones")


# ---------------- (a) point -> cell ----------------
def test_h3_known_answers_gpu(h3ctx):
    for c in GOLD["h3_point_to_cell"]:
        got = h3ctx.grid_longlatascellid(np.array([c["lon"]]), np.array([c["lat"]]), c["res"])
        assert int(got[0]) == c["cell"], c["source"]


def _sphere_points(rng, n):
    lon = rng.uniform(-180, 180, n)
    lat = np.degrees(np.arcsin(rng.uniform(-1, 1, n)))
    return lon, lat


@pytest.mark.parametrize("res", list(range(16)))
def test_h3_cells_match_oracle_global(h3ctx, res):
    rng = np.random.default_rng(100 + res)
    lon, lat = _sphere_points(rng, 200_000)
    got = h3ctx.grid_longlatascellid(lon, lat, res)
    want = oracle.h3_point_to_index(lon, lat, res)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, [(lon[i], lat[i], hex(got[i]), hex(want[i])) for i in bad[:5]]


@pytest.mark.parametrize("res", [8, 9, 10, 11])
def test_h3_cells_match_oracle_nyc(h3ctx, zones, res):
    x, y = quickstart_points(zones, 1_000_000, config=1)
    got = h3ctx.grid_longlatascellid(x, y, res)
    want = oracle.h3_point_to_index(x, y, res)
    assert np.array_equal(got, want)


def test_h3_cells_adversarial(h3ctx):
    """Points at hexagon vertices / edge midpoints of every face and resolution (forces the exact
    path) must still match the oracle bit for bit; the stats counter shows the exact path ran."""
    rng = np.random.default_rng(5)
    # vertices of res-r cells near random points: cell centres +- half a cell, many resolutions
    lon, lat = _sphere_points(rng, 50_000)
    for res in (5, 9, 12, 15):
        # snap onto an exactly representable grid to create ties in the projection
        step = 10.0 ** (-(res // 2 + 1))
        lo = np.round(lon / step) * step
        la = np.round(lat / step) * step
        got = h3ctx.grid_longlatascellid(lo, la, res)
        want = oracle.h3_point_to_index(lo, la, res)
        assert np.array_equal(got, want), res


def test_h3_jdk_toggle(h3ctx):
    rng = np.random.default_rng(9)
    lon, lat = _sphere_points(rng, 100_000)
    h3ctx.set_option("jdk", 11)
    try:
        got = h3ctx.grid_longlatascellid(lon, lat, 12)
    finally:
        h3ctx.set_option("jdk", 8)
    assert np.array_equal(got, oracle.h3_point_to_index(lon, lat, 12, jdk=11))


def test_h3_nonfinite_and_resolution_errors(h3ctx):
    got = h3ctx.grid_longlatascellid(np.array([np.nan, 1.0, np.inf]), np.array([1.0, np.nan, 2.0]), 9)
    assert list(got) == [0, 0, 0]
    with pytest.raises(IllegalStateException, match="H3 resolution has to be between 0 and 15; found 16"):
        h3ctx.grid_longlatascellid(np.array([1.0]), np.array([1.0]), 16)
    with pytest.raises(IllegalStateException, match="found -1"):
        h3ctx.grid_longlatascellid(np.array([1.0]), np.array([1.0]), -1)
    assert h3ctx.index_system.get_resolution("9") == 9


def test_h3_empty_input(h3ctx):
    assert len(h3ctx.grid_longlatascellid(np.zeros(0), np.zeros(0), 9)) == 0


def test_grid_pointascellid_wkt(h3ctx):
    pts = ["POINT (30 10)", "POINT (-74.044444 40.689167)"]
    got = h3ctx.grid_pointascellid(pts, 10)
    assert int(got[0]) == 623385352048508927
    assert int(got[1]) == 0x8A2A1072B59FFFF


def test_h3_device_tensors(h3ctx):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(3)
    lon, lat = _sphere_points(rng, 100_000)
    got = h3ctx.grid_longlatascellid(torch.tensor(lon, device="cuda"), torch.tensor(lat, device="cuda"), 9)
    assert got.is_cuda
    assert np.array_equal(got.cpu().numpy(), oracle.h3_point_to_index(lon, lat, 9))


def test_bng_golden_gpu(bngctx):
    for c in GOLD["bng_point_to_index"]:
        got = bngctx.grid_longlatascellid(np.array([float(c["e"])]), np.array([float(c["n"])]), c["res"])
        assert got == [c["fmt"]]
        raw = bngctx.grid_longlatascellid(np.array([float(c["e"])]), np.array([float(c["n"])]), c["res"], raw=True)
        assert int(raw[0]) == c["id"]
        assert bngctx.index_system.parse(c["fmt"]) == c["id"]


@pytest.mark.parametrize("res", [1, 2, 3, 4, 5, 6, -1, -2, -3, -4, -5, -6])
def test_bng_matches_oracle(bngctx, res):
    rng = np.random.default_rng(200 + res)
    e = rng.uniform(-1e5, 8e5, 200_000)
    n = rng.uniform(-1e5, 1.4e6, 200_000)
    e[:1000] = np.round(e[:1000])  # integral coordinates exercise the bin edges
    n[:1000] = np.round(n[:1000])
    got = bngctx.grid_longlatascellid(e, n, res, raw=True)
    want, err = oracle.bng_point_to_index_batch(e, n, res)
    assert not err.any()
    assert np.array_equal(got, want)


def test_bng_errors(bngctx):
    with pytest.raises(IllegalStateException, match="NaN coordinates are not supported."):
        bngctx.grid_longlatascellid(np.array([np.nan]), np.array([100.0]), 5)
    with pytest.raises(IllegalStateException, match="BNG resolution not supported"):
        bngctx.grid_longlatascellid(np.array([1.0]), np.array([1.0]), 7)
    assert bngctx.index_system.get_resolution("100m") == 4
    assert bngctx.index_system.get_resolution("500m") == -4


# ---------------- (c) st_contains ----------------
def test_st_contains_golden_gpu(h3ctx):
    poly = GOLD["contains"]["polygon"]
    pts = [p for p, _ in GOLD["contains"]["cases"]]
    got = h3ctx.st_contains(poly, pts)
    assert list(got) == [e for _, e in GOLD["contains"]["cases"]]


def test_st_contains_matches_oracle(h3ctx, zones):
    rng = np.random.default_rng(11)
    ids = list(range(0, 263, 7))
    bx, by = boundary_points(zones, ids, rng)
    geoms, xs, ys = [], [], []
    for i in range(len(bx)):
        g = ids[i % len(ids)]
        geoms.append(zones.wkb(g))
        xs.append(bx[i])
        ys.append(by[i])
    for g in ids:  # random interior/exterior points per zone
        x0, y0, x1, y1 = zones.geom_bbox(g)
        for _ in range(200):
            geoms.append(zones.wkb(g, big_endian=False))
            xs.append(rng.uniform(x0, x1))
            ys.append(rng.uniform(y0, y1))
    got = h3ctx.st_contains(geoms, (np.array(xs), np.array(ys)))
    want = np.array([oracle.wkb_contains(w, x, y) for w, x, y in zip(geoms, xs, ys)])
    assert np.array_equal(got, want)
    assert want.sum() > 0 and (~want).sum() > 0


# ---------------- (b)+(c) the chip join ----------------
def _join_case(ctx, zones, res, n_points, seed, grid=oracle.GRID_H3):
    rng = np.random.default_rng(seed)
    ids = list(rng.choice(len(zones), 40, replace=False))
    chips = synthetic_chips(zones, ids, res, lambda x, y, r: oracle.h3_point_to_index(x, y, r), rng)
    table = ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], res,
                           n_polygons=len(ids))
    sub = zones.subset(ids)
    x, y = quickstart_points(sub, n_points, seed=seed)
    bx, by = boundary_points(zones, ids, rng, n_per=20)
    x = np.concatenate([x, bx])
    y = np.concatenate([y, by])
    return chips, table, x, y, len(ids)


@pytest.mark.parametrize("res", [8, 9, 10])
def test_join_counts_match_oracle(h3ctx, zones, res):
    chips, table, x, y, npoly = _join_case(h3ctx, zones, res, 300_000, seed=res)
    got = h3ctx.pip_join_count(table, x, y)
    want, total = oracle.pip_join(chips_to_oracle(chips), oracle.GRID_H3, res, x, y, npoly, threads=8)
    assert np.array_equal(got, want)
    assert total > 1000
    assert int(got.sum()) == total
    assert h3ctx.last_stats()["contains_tests"] > 0
    # the tile path and the generic path (no tile directory) give the same counts
    try:
        for tiles, praster in ((1, 0), (0, 0)):
            h3ctx.set_option("tiles", tiles)
            h3ctx.set_option("point_raster", praster)
            assert np.array_equal(h3ctx.pip_join_count(table, x, y), want), (tiles, praster)
    finally:
        h3ctx.set_option("tiles", 1)
        h3ctx.set_option("point_raster", 1)


def _chip_boundary_points(chips, rng, limit=4000):
    """Vertices of border chips, points on their segments, and both 1-3 ulp nudges of each."""
    from mosaic_amd.wkb import read_wkb

    offs, data = chips["wkb"]
    xs, ys = [], []
    border = np.nonzero(chips["is_core"] == 0)[0]
    for i in rng.choice(border, min(limit, len(border)), replace=False):
        _, parts = read_wkb(data[offs[i]:offs[i + 1]])
        ring = np.asarray(parts[0][0])
        k = int(rng.integers(1, len(ring)))
        t = rng.uniform()
        for px, py in (ring[k], ring[k - 1] + t * (ring[k] - ring[k - 1])):
            for d in (0, 1, -1, 3):
                xs.append(np.nextafter(px, np.inf) if d == 1 else (np.nextafter(px, -np.inf) if d == -1 else px))
                ys.append(py if d != 3 else np.nextafter(np.nextafter(py, np.inf), np.inf))
    return np.array(xs), np.array(ys)


def test_join_tessellated_chips_every_strategy(h3ctx):
    """Real grid_tessellateexplode chips (35 NYC zones, res 9) with points on / next to the chips'
    own vertices and segments: every join path and raster size gives the oracle's pairs.

    Chip vertices include H3 cell corners, where H3's answer hangs on the last bit of libm: the
    exact path's glibc restatement makes every row's cell equal the oracle's."""
    from mosaic_amd.context import tessellate

    zones35 = PolygonSet.load("nyc_taxi_zones_35")
    chips = tessellate("H3", zones35, 9)
    rng = np.random.default_rng(5)
    x0, y0, x1, y1 = zones35.bbox()
    bx, by = _chip_boundary_points(chips, rng)
    x = np.concatenate([rng.uniform(x0, x1, 400_000), bx])
    y = np.concatenate([rng.uniform(y0, y1, 400_000), by])
    cells = h3ctx.grid_longlatascellid(x, y, 9, raw=True)
    differ = np.nonzero(cells != oracle.h3_point_to_index(x, y, 9))[0]
    assert len(differ) == 0, [(x[i], y[i]) for i in differ[:5]]
    offs, data = chips["wkb"]
    oc = dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
              wkb_offsets=offs, wkb=data)
    _, total, orow, okey = oracle.pip_join(oc, oracle.GRID_H3, 9, x, y, len(zones35), pairs=True)
    assert total > 10_000
    want = set(zip(orow.tolist(), okey.tolist()))
    try:
        for raster, lane_edges in ((16, 8), (1, 8), (5, 0), (32, 32), (2, 0)):
            h3ctx.set_option("raster", raster)
            h3ctx.set_option("lane_edges", lane_edges)
            table = h3ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 9,
                                     n_polygons=len(zones35))
            assert table.tiles()["built"] == 1
            # (stream_pipe 2: k_join_stream_cpt, the default -- the boundary points fill whole groups
            # with pending rows, so its > 64-row overflow path runs too; 1: k_join_stream_pipe; 0:
            # k_join_stream, the unpipelined float-coordinate stream kernel)
            for tiles, praster, pipe in ((1, 1, 2), (1, 1, 1), (1, 1, 0), (1, 0, 1), (0, 0, 1)):
                h3ctx.set_option("tiles", tiles)
                h3ctx.set_option("point_raster", praster)
                h3ctx.set_option("stream_pipe", pipe)
                rows, keys = h3ctx.pip_join_pairs(table, x, y)
                got = set(zip(rows.tolist(), keys.tolist()))
                assert got == want, (raster, lane_edges, tiles, praster, pipe, len(got ^ want))
                counts = h3ctx.pip_join_count(table, x, y)
                assert np.array_equal(counts, np.bincount(okey, minlength=len(zones35))), (raster, tiles, praster, pipe)
            h3ctx.set_option("tiles", 1)
            h3ctx.set_option("point_raster", 1)
            h3ctx.set_option("stream_pipe", 2)
            table.close()
    finally:
        h3ctx.set_option("raster", 16)
        h3ctx.set_option("lane_edges", 0)
        h3ctx.set_option("tiles", 1)
        h3ctx.set_option("point_raster", 1)
        h3ctx.set_option("stream_pipe", 2)


def _tile_edge_points(t, rng, n):
    """Points on and 1 ulp either side of the tile directory's row / column lines."""
    nx, ny, x0, y0, sx, sy = t["nx"], t["ny"], t["x0"], t["y0"], t["sx"], t["sy"]
    xs = x0 + rng.integers(0, nx + 1, n) / sx
    ys = y0 + rng.uniform(0, ny / sy, n)
    ys2 = y0 + rng.integers(0, ny + 1, n) / sy
    xs2 = x0 + rng.uniform(0, nx / sx, n)
    x = np.concatenate([xs, np.nextafter(xs, np.inf), np.nextafter(xs, -np.inf), xs2, xs2])
    y = np.concatenate([ys, ys, ys, ys2, np.nextafter(ys2, -np.inf)])
    return x, y


def test_join_tiled_nyc_zones_match_oracle(h3ctx, zones):
    """The bench workload's build side (all 263 zones, grid_tessellateexplode at res 9) with the
    tile directory: uniform points over and beyond the zones' bbox, clustered points, points on
    tile lines and on chip boundaries -- counts equal the oracle's and the untiled kernel's."""
    from mosaic_amd.context import tessellate

    chips = tessellate("H3", zones, 9)
    table = h3ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 9,
                             n_polygons=len(zones))
    t = table.tiles()
    assert t["built"] == 1 and t["records"] > 100, t
    rng = np.random.default_rng(11)
    x0, y0, x1, y1 = zones.bbox()
    wx, wy = x1 - x0, y1 - y0
    ux = rng.uniform(x0 - 0.2 * wx, x1 + 0.2 * wx, 600_000)
    uy = rng.uniform(y0 - 0.2 * wy, y1 + 0.2 * wy, 600_000)
    qx, qy = quickstart_points(zones, 200_000, seed=12)
    bx, by = _chip_boundary_points(chips, rng, limit=3000)
    tx, ty = _tile_edge_points(t, rng, 40_000)
    x = np.concatenate([ux, qx, tx, bx, [np.nan, np.inf, x0]])
    y = np.concatenate([uy, qy, ty, by, [y0, 0.0, np.nan]])
    cells = h3ctx.grid_longlatascellid(x, y, 9, raw=True)
    ocells = oracle.h3_point_to_index(x, y, 9)
    assert np.array_equal(cells, ocells)
    keep = np.ones(len(x), bool)
    offs, data = chips["wkb"]
    oc = dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
              wkb_offsets=offs, wkb=data)
    want, total = oracle.pip_join(oc, oracle.GRID_H3, 9, x[keep], y[keep], len(zones), threads=8)
    assert total > 100_000
    assert t["raster"] == 1 and t["pure_sub_blocks"] > 1000, t
    got = h3ctx.pip_join_count(table, x[keep], y[keep])
    assert np.array_equal(got, want)
    rows, keys = h3ctx.pip_join_pairs(table, x[keep], y[keep])
    assert len(rows) == total and np.array_equal(np.bincount(keys, minlength=len(zones)), want)
    try:
        # other workgroup sizes of the stream kernel
        for block in (256, 512, 64):
            h3ctx.set_option("stream_block", block)
            assert np.array_equal(h3ctx.pip_join_count(table, x[keep], y[keep]), want), block
            rows2, keys2 = h3ctx.pip_join_pairs(table, x[keep], y[keep])
            assert np.array_equal(np.sort(rows2), np.sort(rows)), block
        h3ctx.set_option("stream_block", 1024)
        # row counts that are not multiples of 256 (the wave's tail iteration), misaligned columns
        # (the scalar-load variant) and the tiled kernel agree with the oracle on every prefix
        import torch

        xs, ys = x[keep], y[keep]
        xt, yt = torch.from_numpy(xs).cuda(), torch.from_numpy(ys).cuda()
        for cut in (1, 2, 3, 255, 257, len(xs) - 5):
            ref, _ = oracle.pip_join(oc, oracle.GRID_H3, 9, xs[:-cut], ys[:-cut], len(zones), threads=8)
            assert np.array_equal(h3ctx.pip_join_count(table, xs[:-cut], ys[:-cut]), ref), cut
            # device columns starting 8 bytes past a 16-byte boundary
            ref1, _ = oracle.pip_join(oc, oracle.GRID_H3, 9, xs[1:-cut], ys[1:-cut], len(zones), threads=8)
            got1 = h3ctx.pip_join_count(table, xt[1:-cut], yt[1:-cut]).cpu().numpy()
            assert np.array_equal(got1, ref1), cut
        for tiles, praster in ((1, 0), (0, 0)):
            h3ctx.set_option("tiles", tiles)
            h3ctx.set_option("point_raster", praster)
            assert np.array_equal(h3ctx.pip_join_count(table, x[keep], y[keep]), want), (tiles, praster)
    finally:
        h3ctx.set_option("stream_block", 1024)
        h3ctx.set_option("tiles", 1)
        h3ctx.set_option("point_raster", 1)
    table.close()


@pytest.mark.parametrize("sub,cell", [(4, 2), (16, 8), (64, 4)])
def test_join_point_raster_sizes(h3ctx, zones, sub, cell):
    """Other point-raster shapes (coarse: most points take the tile path; fine; many sub-blocks)
    give the oracle's counts on clustered points (the C3 mixture) at res 10."""
    from mosaic_amd.context import tessellate

    ids = list(range(0, 263, 3))
    sub_zones = zones.subset(ids)
    chips = tessellate("H3", sub_zones, 10)
    h3ctx.set_option("raster_sub", sub)
    h3ctx.set_option("raster_cell", cell)
    try:
        table = h3ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 10,
                                 n_polygons=len(ids))
    finally:
        h3ctx.set_option("raster_sub", 64)
        h3ctx.set_option("raster_cell", 16)
    t = table.tiles()
    assert t["raster"] == 1 and t["raster_sub"] == sub and t["raster_cell"] == cell, t
    x, y = quickstart_points(sub_zones, 400_000, sigma=0.002, seed=31)
    offs, data = chips["wkb"]
    oc = dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
              wkb_offsets=offs, wkb=data)
    want, total = oracle.pip_join(oc, oracle.GRID_H3, 10, x, y, len(ids), threads=8)
    assert total > 100_000
    assert np.array_equal(h3ctx.pip_join_count(table, x, y), want)
    table.close()


def test_join_pairs_match_oracle(h3ctx, zones):
    chips, table, x, y, npoly = _join_case(h3ctx, zones, 9, 100_000, seed=21)
    rows, keys = h3ctx.pip_join_pairs(table, x, y, capacity=16)  # forces the capacity retry
    _, total, orow, okey = oracle.pip_join(chips_to_oracle(chips), oracle.GRID_H3, 9, x, y, npoly, pairs=True)
    order = np.lexsort((okey, orow))
    assert len(rows) == total
    assert np.array_equal(rows, orow[order]) and np.array_equal(keys, okey[order])


def test_join_many_polygons_global_counts(h3ctx, zones):
    """More polygon keys than the LDS histogram holds: the global-atomic count path."""
    rng = np.random.default_rng(4)
    ids = list(range(263))
    chips = synthetic_chips(zones, ids, 9, lambda x, y, r: oracle.h3_point_to_index(x, y, r), rng, pts_per_zone=50)
    # spread keys over a large key space
    chips["polygon_key"] = chips["polygon_key"] * 40
    n_poly = 263 * 40
    table = h3ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 9, n_poly)
    x, y = quickstart_points(zones, 200_000, seed=4)
    got = h3ctx.pip_join_count(table, x, y)
    want, _ = oracle.pip_join(chips_to_oracle(chips), oracle.GRID_H3, 9, x, y, n_poly, threads=8)
    assert np.array_equal(got, want)


def test_join_empty_and_edge_inputs(h3ctx, zones):
    chips, table, x, y, npoly = _join_case(h3ctx, zones, 9, 1000, seed=2)
    assert not h3ctx.pip_join_count(table, np.zeros(0), np.zeros(0)).any()
    got = h3ctx.pip_join_count(table, np.array([np.nan, 0.0]), np.array([0.0, np.nan]))
    assert not got.any()
    empty = h3ctx.chip_table(np.zeros(0, np.uint8), np.zeros(0, np.int64), [], np.zeros(0, np.int32), 9, 0)
    assert len(h3ctx.pip_join_count(empty, x, y)) == 0


def test_join_device_tensors(h3ctx, zones):
    torch = pytest.importorskip("torch")
    chips, table, x, y, npoly = _join_case(h3ctx, zones, 9, 200_000, seed=8)
    got = h3ctx.pip_join_count(table, torch.tensor(x, device="cuda"), torch.tensor(y, device="cuda"))
    want, _ = oracle.pip_join(chips_to_oracle(chips), oracle.GRID_H3, 9, x, y, npoly, threads=8)
    assert np.array_equal(got.cpu().numpy(), want)


@pytest.mark.parametrize("res,every", [(3, 3), (4, 3), (5, 25)])
def test_join_bng_dense_table(bngctx, res, every):
    """BNG dense cell table (k_join_stream_bng): tessellated chips of the London postcode zones in
    EPSG:27700 metres (tests/golden/make_bng_fixture.py), uniform points, points on and 1 ulp around
    cell lines, negative and >= 1e7 coordinates (outside the one-to-one range: generic path) --
    counts equal the oracle's and the generic kernel's, with and without the LDS cell level (res 5:
    the level holds blocks of cells, block shift > 0)."""
    from mosaic_amd.context import tessellate

    ids = list(range(0, 177, every))
    proj = PolygonSet.load("london_postcodes_bng").subset(ids)
    chips = tessellate("BNG", proj, res)
    table = bngctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], res,
                              n_polygons=len(ids))
    ti = table.tiles()
    assert ti["built"] == 1 and ti["records"] > 0  # LDS cell level bytes
    lds_budget = 160 * 1024 - (len(ids) + 64) * 4 - 16 * 320 * 4
    assert (ti["entries"] > 0) == (ti["nx"] * ti["ny"] > lds_budget)  # block shift
    assert ti["rings"] > 0  # border-cell sub-cells split by one straight edge (line records)
    rng = np.random.default_rng(40 + res)
    x0, y0, x1, y1 = proj.bbox()
    x = rng.uniform(x0 - 2000, x1 + 2000, 400_000)
    y = rng.uniform(y0 - 2000, y1 + 2000, 400_000)
    step = 10.0 ** (6 - res)
    lx = np.floor(rng.uniform(x0, x1, 20_000) / step) * step  # on vertical cell lines
    ly = np.floor(rng.uniform(y0, y1, 20_000) / step) * step  # on horizontal cell lines
    ux, uy = rng.uniform(x0, x1, 20_000), rng.uniform(y0, y1, 20_000)
    lines_x = np.concatenate([lx, np.nextafter(lx, -np.inf), np.nextafter(lx, np.inf), ux, ux])
    lines_y = np.concatenate([uy, uy, uy, ly, np.nextafter(ly, -np.inf)])
    odd_x = np.array([-0.5, -1.5, -150000.0, 1e7, 2.5e9, x0 + 10.0, 5e6])
    odd_y = np.array([y0 + 10.0, y0 + 20.0, y0, y0 + 30.0, y0 + 40.0, -0.25, 1.2e7])
    x = np.concatenate([x, lines_x, odd_x])
    y = np.concatenate([y, lines_y, odd_y])
    offs, data = chips["wkb"]
    oc = dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
              wkb_offsets=offs, wkb=data)
    want, total = oracle.pip_join(oc, oracle.GRID_BNG, res, x, y, len(ids), threads=8)
    assert total > 10_000
    assert np.array_equal(bngctx.pip_join_count(table, x, y), want)
    rows, keys = bngctx.pip_join_pairs(table, x, y)
    assert len(rows) == total and np.array_equal(np.bincount(keys, minlength=len(ids)), want)
    bngctx.set_option("tiles", 0)
    try:
        assert np.array_equal(bngctx.pip_join_count(table, x, y), want)
    finally:
        bngctx.set_option("tiles", 1)
    bngctx.set_option("bng_cpt", 0)  # the uncompacted BNG stream kernel (not the default)
    try:
        assert np.array_equal(bngctx.pip_join_count(table, x, y), want)
        assert bngctx.last_kernel() == "k_join_stream_bng"
        r1, k1 = bngctx.pip_join_pairs(table, x, y)
        assert np.array_equal(np.sort(r1 * len(ids) + k1), np.sort(rows * len(ids) + keys))
    finally:
        bngctx.set_option("bng_cpt", 1)
    bngctx.set_option("point_raster", 0)  # dense cell table without the border-cell leaf blocks
    try:
        t2 = bngctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], res,
                               n_polygons=len(ids))
    finally:
        bngctx.set_option("point_raster", 1)
    assert np.array_equal(bngctx.pip_join_count(t2, x, y), want)
    t2.close()
    # dense cell table without the LDS cell level and line records, 8 x 8 sub-cells
    for k, v in (("bng_lds", 0), ("raster_lines", 0), ("bng_cell", 8)):
        bngctx.set_option(k, v)
    try:
        t3 = bngctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], res,
                               n_polygons=len(ids))
    finally:
        for k, v in (("bng_lds", 1), ("raster_lines", 1), ("bng_cell", 32)):
            bngctx.set_option(k, v)
    assert t3.tiles()["records"] == 0 and t3.tiles()["rings"] == 0
    assert np.array_equal(bngctx.pip_join_count(t3, x, y), want)
    r3, k3 = bngctx.pip_join_pairs(t3, x, y)
    assert np.array_equal(np.sort(r3 * len(ids) + k3), np.sort(rows * len(ids) + keys))
    t3.close()
    with pytest.raises(IllegalStateException, match="NaN"):
        bngctx.pip_join_count(table, np.array([x0 + 5.0, np.nan]), np.array([y0 + 5.0, y0]))
    table.close()


def test_join_bng(bngctx):
    # the London postcode zones in EPSG:27700 metres; chips from BNG cells of random points
    proj = PolygonSet.load("london_postcodes_bng")
    rng = np.random.default_rng(6)
    ids = list(range(0, 177, 5))
    res = 4

    def cell_fn(xs, ys, r):
        out, err = oracle.bng_point_to_index_batch(xs, ys, r)
        return out

    chips = synthetic_chips(proj, ids, res, cell_fn, rng, pts_per_zone=300)
    table = bngctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], res,
                              n_polygons=len(ids))
    x0, y0, x1, y1 = proj.bbox()
    x = rng.uniform(x0, x1, 300_000)
    y = rng.uniform(y0, y1, 300_000)
    got = bngctx.pip_join_count(table, x, y)
    want, total = oracle.pip_join(chips_to_oracle(chips), oracle.GRID_BNG, res, x, y, len(ids), threads=8)
    assert np.array_equal(got, want) and total > 0
    with pytest.raises(IllegalStateException, match="NaN"):
        bngctx.pip_join_count(table, np.array([np.nan]), np.array([1.0]))


@pytest.mark.parametrize("n_buildings", [20_000, 40_000])
def test_join_c4_buildings(h3ctx, n_buildings):
    """C4 shape: OSM-style building footprints (rectangles and L-shapes, 8-40 m sides) chipped at
    res 11 -- nearly all chips are border chips, polygon keys beyond the LDS histogram (global
    counts) and, at 40k buildings, beyond the point raster's 16-bit codes (tile path).  Points 70 %
    near buildings, 30 % uniform, plus chip vertices and edge points: counts and pairs equal the
    oracle's."""
    import torch

    from mosaic_amd.context import tessellate
    from mosaic_amd.data import building_points_device, synthetic_buildings

    b = synthetic_buildings(n_buildings, bbox=(-74.02, 40.70, -73.93, 40.80), n_centres=16, sigma=0.005)
    chips = tessellate("H3", b, 11)
    assert chips["is_core"].sum() < 0.05 * len(chips["is_core"])
    table = h3ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 11,
                             n_polygons=n_buildings)
    t = table.tiles()
    assert t["built"] == 1
    assert t["raster"] == (1 if n_buildings < 32765 else 0), t
    xd, yd = building_points_device(b, 1_500_000, seed=77)
    x, y = xd.cpu().numpy(), yd.cpu().numpy()
    del xd, yd
    torch.cuda.empty_cache()
    rng = np.random.default_rng(78)
    bx, by = _chip_boundary_points(chips, rng, limit=3000)
    x = np.concatenate([x, bx])
    y = np.concatenate([y, by])
    cells = h3ctx.grid_longlatascellid(x, y, 11, raw=True)
    assert np.array_equal(cells, oracle.h3_point_to_index(x, y, 11))
    offs, data = chips["wkb"]
    oc = dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
              wkb_offsets=offs, wkb=data)
    want, total = oracle.pip_join(oc, oracle.GRID_H3, 11, x, y, n_buildings, threads=8)
    assert total > 200_000
    assert np.array_equal(h3ctx.pip_join_count(table, x, y), want)
    rows, keys = h3ctx.pip_join_pairs(table, x, y)
    assert len(rows) == total and np.array_equal(np.bincount(keys, minlength=n_buildings), want)
    table.close()


# ---------------- point geometry column decode ----------------
def _column(rows):
    lens = np.array([len(r) for r in rows], np.int64)
    offs = np.zeros(len(rows) + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    return offs, np.frombuffer(b"".join(rows) or b"\0", np.uint8).copy()


@pytest.mark.parametrize("offsets32", [False, True])
def test_point_decode_corpus(h3ctx, offsets32):
    """Device decoder vs the oracle restatement (oracle/point_decode.py) on the adversarial corpus:
    identical decode / row-path split, bit-identical coordinates; null rows stay null."""
    import ctypes
    import struct

    from mosaic_amd import _native as N
    from oracle import point_decode as PD
    from tests.helpers import point_rows

    rows = point_rows(np.random.default_rng(41))
    for fmt in (0, 1, 2):
        sel = [r for f, r in rows if f == fmt]
        sel = sel + [b""]  # a null row (validity 0) with an empty value
        offs, data = _column(sel)
        if offsets32:
            offs = offs.astype(np.int32)
        valid = np.ones(len(sel), np.uint8)
        valid[-1] = 0
        n = len(sel)
        x, y, st = np.empty(n), np.empty(n), np.empty(n, np.uint8)
        n_rp = ctypes.c_int64(0)
        f = fmt | (N.GEOM_OFFSETS32 if offsets32 else 0)
        N.check(N.lib().mosaic_point_geom_decode(h3ctx.handle, f, N.ptr(offs), N.ptr(data), N.ptr(valid), n, N.ptr(x),
                                                 N.ptr(y), N.ptr(st), ctypes.byref(n_rp)))
        assert st[-1] == N.ROW_NULL
        n_path = 0
        for k, r in enumerate(sel[:-1]):
            want = PD.decode(fmt, r)
            if want[0] == "ok":
                assert st[k] == N.ROW_OK, (fmt, r)
                assert struct.pack("<dd", x[k], y[k]) == struct.pack("<dd", want[1], want[2]), (fmt, r, x[k], y[k])
            else:
                assert st[k] == N.ROW_PATH, (fmt, r)
                n_path += 1
        assert n_rp.value == n_path > 0


def test_grid_pointascellid_geometry_columns(h3ctx, bngctx):
    """grid_pointascellid over WKT / WKB / hex columns == grid_longlatascellid of the decoded
    coordinates == the oracle; rows the engine leaves to the row path are reported, not guessed."""
    from mosaic_amd import RowPathRequired
    from mosaic_amd.wkb import point_wkb

    rng = np.random.default_rng(43)
    x = np.round(rng.uniform(-74.3, -73.7, 50_000), 6)
    y = np.round(rng.uniform(40.5, 40.9, 50_000), 6)
    want = oracle.h3_point_to_index(x, y, 9)
    wkt = ["POINT (%r %r)" % (float(a), float(b)) for a, b in zip(x, y)]
    assert np.array_equal(h3ctx.grid_pointascellid(wkt, 9), want)
    wkb = [point_wkb(a, b, big_endian=bool(k % 2)) for k, (a, b) in enumerate(zip(x, y))]
    assert np.array_equal(h3ctx.grid_pointascellid(wkb, 9), want)
    hexrows = [w.hex() for w in wkb[:5000]]
    assert np.array_equal(h3ctx.grid_pointascellid(hexrows, 9, fmt="hex"), want[:5000])
    # nulls and row-path rows
    mixed = [wkt[0], None, "POLYGON ((0 0, 1 0, 1 1, 0 0))", "POINT EMPTY", wkt[1]]
    cells, st = h3ctx.grid_pointascellid(mixed, 9, return_status=True)
    assert list(st) == [1, 0, 2, 2, 1] and cells[0] == want[0] and cells[4] == want[1] and cells[1] == 0
    with pytest.raises(RowPathRequired) as ei:
        h3ctx.grid_pointascellid(mixed, 9)
    assert list(ei.value.rows) == [2, 3]
    # BNG: metres, string ids; NaN coordinates still raise the reference's exception
    e = np.round(rng.uniform(0, 700_000, 20_000), 1)
    nn = np.round(rng.uniform(0, 1_300_000, 20_000), 1)
    got = bngctx.grid_pointascellid(["POINT (%r %r)" % (float(a), float(b)) for a, b in zip(e, nn)], "100m", raw=True)
    assert np.array_equal(got, oracle.bng_point_to_index_batch(e, nn, 4)[0])
    with pytest.raises(IllegalStateException, match="NaN"):
        bngctx.grid_pointascellid(["POINT (NaN 5)"], 4)


def test_point_decode_device_buffers_at_scale(h3ctx):
    """C1 shape: 10M taxi-GPS WKT rows (1e-6 degree rounding) resident on the device, int32
    offsets (Spark's Arrow utf8): cells equal the direct lon/lat path on the same doubles."""
    torch = pytest.importorskip("torch")
    from mosaic_amd.data import quickstart_points

    zones = PolygonSet.load("nyc_taxi_zones")
    x, y = quickstart_points(zones, 2_000_000, seed=44)
    x, y = np.round(x, 6), np.round(y, 6)
    rows = [("POINT (%.6f %.6f)" % (a, b)).encode() for a, b in zip(x, y)] * 5
    offs, data = _column(rows)
    offs32 = torch.tensor(offs.astype(np.int32), device="cuda")
    dd = torch.tensor(data, device="cuda")
    cells, st = h3ctx.grid_pointascellid((offs32, dd, None), 9, raw=True, fmt="wkt", return_status=True)
    assert cells.is_cuda and int((st != 1).sum()) == 0
    direct = h3ctx.grid_longlatascellid(np.tile(x, 5), np.tile(y, 5), 9, raw=True)
    assert np.array_equal(cells.cpu().numpy(), direct)
    assert np.array_equal(direct[:2_000_000], oracle.h3_point_to_index(x, y, 9))
