"""grid_tessellateexplode (BNG) with the cell classification on the GPU: parity with the host producer.

mosaic_tessellate_gpu classifies every candidate cell (border / core / dropped) with
k_bng_tess_classify and clips border cells on the host; mosaic_tessellate does all of it on the
host.  The chip sets must agree row for row and byte for byte (is_core, index_id, polygon key,
WKB).  The host producer itself is pinned against the reference's chip-join == brute-force
invariant (MosaicFrameBehaviors.scala:136-223) in test_tessellate.py, and the chip join over the
GPU-produced chips is checked against the brute-force oracle here as well.
"""
import time

import numpy as np
import pytest

import oracle
from mosaic_amd import MosaicContext
from mosaic_amd.context import tessellate
from mosaic_amd.data import PolygonSet

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = MosaicContext.build("BNG", "JTS")
    yield c
    c.close()


@pytest.fixture(scope="module")
def london_m():
    # the London postcode zones in EPSG:27700 metres (tests/golden/make_bng_fixture.py)
    return PolygonSet.load("london_postcodes_bng")


def _same(a, b):
    assert len(a["index_id"]) == len(b["index_id"])
    for k in ("is_core", "index_id", "polygon_key"):
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(a["wkb"][0], b["wkb"][0])
    assert np.array_equal(a["wkb"][1], b["wkb"][1])


@pytest.mark.parametrize("res", [3, -3, 4])
def test_bng_gpu_tessellation_equals_host(ctx, london_m, res):
    polys = london_m if res != 4 else london_m.subset(range(0, 177, 4))
    t0 = time.perf_counter()
    host = tessellate("BNG", polys, res)
    t1 = time.perf_counter()
    gpu = tessellate("BNG", polys, res, ctx=ctx)
    t2 = time.perf_counter()
    _same(host, gpu)
    assert len(host["index_id"]) > 100 and (host["is_core"] == 0).sum() > 0
    if res == 4:  # 100 m cells: postcode interiors hold core cells
        assert host["is_core"].sum() > 0
    from mosaic_amd import _native as N

    ms = N.lib().mosaic_tess_last_classify_ms(ctx.handle)
    print(f"res {res}: {len(host['index_id'])} chips, host {t1 - t0:.3f} s, gpu path {t2 - t1:.3f} s "
          f"(classify kernel {ms:.3f} ms)")


def test_bng_gpu_tessellation_join_invariant(ctx, london_m):
    polys = london_m.subset(range(0, 177, 5))
    chips = tessellate("BNG", polys, 3, ctx=ctx)
    rng = np.random.default_rng(7)
    x0, y0, x1, y1 = polys.bbox()
    x = rng.uniform(x0, x1, 40_000)
    y = rng.uniform(y0, y1, 40_000)
    want, total_bf = oracle.brute_force_count(polys, x, y)
    offs, data = chips["wkb"]
    o = dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
             wkb_offsets=offs, wkb=data)
    got, _ = oracle.pip_join(o, oracle.GRID_BNG, 3, x, y, len(polys), threads=8)
    assert np.array_equal(got, want) and total_bf > 1000


def test_bng_gpu_tessellation_holes_multipart_empty(ctx):
    # geometry 0: 3.5 km square with a 1.2 km hole; geometry 1: empty; geometry 2: two parts
    sq = lambda x0, y0, s: [(x0, y0), (x0 + s, y0), (x0 + s, y0 + s), (x0, y0 + s), (x0, y0)]
    rings = [sq(530250.0, 180250.0, 3500.0), sq(531100.0, 181100.0, 1200.0)[::-1],
             sq(540000.0, 170000.0, 900.0), sq(542500.0, 171500.0, 2100.0)]
    xy = np.array([p for r in rings for p in r], np.float64)
    ring_offsets = np.cumsum([0] + [len(r) for r in rings]).astype(np.int64)
    part_rings = np.array([0, 2, 3, 4], np.int64)
    geom_parts = np.array([0, 1, 1, 3], np.int64)
    polys = PolygonSet(xy, ring_offsets, part_rings, geom_parts)
    for res in (3, 4, -4):
        for keep in (True, False):
            _same(tessellate("BNG", polys, res, keep_core_geom=keep),
                  tessellate("BNG", polys, res, keep_core_geom=keep, ctx=ctx))
    chips = tessellate("BNG", polys, 3, ctx=ctx)
    assert set(chips["polygon_key"].tolist()) == {0, 2}


@pytest.mark.parametrize("res,densify", [(8, 1), (9, 1), (9, 4), (10, 1)])
def test_h3_gpu_tessellation_equals_host(ctx, res, densify):
    zones = PolygonSet.load("nyc_taxi_zones")
    polys = zones if res < 10 else zones.subset(range(0, 263, 3))
    t0 = time.perf_counter()
    host = tessellate("H3", polys, res, densify=densify)
    t1 = time.perf_counter()
    gpu = tessellate("H3", polys, res, densify=densify, ctx=ctx)
    t2 = time.perf_counter()
    _same(host, gpu)
    assert host["is_core"].sum() > 0 and (host["is_core"] == 0).sum() > 0
    from mosaic_amd import _native as N

    ms = N.lib().mosaic_tess_last_classify_ms(ctx.handle)
    print(f"H3 res {res} densify {densify}: {len(host['index_id'])} chips, host {t1 - t0:.3f} s, "
          f"gpu path {t2 - t1:.3f} s (classify kernel {ms:.3f} ms)")


def test_h3_gpu_tessellation_join_invariant():
    # MosaicFrameBehaviors.scala:136-223 shape: 98 trips x 35 zones, H3 res 8, through the
    # MosaicContext mirror (grid_tessellateexplode) and the GPU chip join
    z35 = PolygonSet.load("nyc_taxi_zones_35")
    trips = np.load("tests/golden/nyctaxi_yellow_trips_pickups.npy")
    h3 = MosaicContext.build("H3", "JTS")
    chips = h3.grid_tessellateexplode(z35, 8)
    table = h3.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 8,
                          n_polygons=len(z35))
    gpu_counts = h3.pip_join_count(table, trips[:, 0], trips[:, 1])
    table.close()
    h3.close()
    want, total_bf = oracle.brute_force_count(z35, trips[:, 0], trips[:, 1])
    offs, data = chips["wkb"]
    o = dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
             wkb_offsets=offs, wkb=data)
    got, _ = oracle.pip_join(o, oracle.GRID_H3, 8, trips[:, 0], trips[:, 1], len(z35))
    assert np.array_equal(got, want) and total_bf > 0
    assert np.array_equal(np.asarray(gpu_counts), want)


def test_gpu_tessellation_errors(ctx):
    from mosaic_amd import IllegalStateException

    z = PolygonSet.load("nyc_taxi_zones_35").subset([0])
    with pytest.raises(IllegalStateException, match="found 16"):
        tessellate("H3", z, 16, ctx=ctx)
    with pytest.raises(IllegalStateException, match="BNG resolution not supported"):
        tessellate("BNG", z, 0, ctx=ctx)


def test_h3_gpu_reference_tessellation_fixtures():
    # the reference's regression polygons (issue #243 at res 7: 10 distinct chips; issue #260 at res
    # 3: > 0 chips) through the GPU producer, equal to the host producer
    from .test_tessellate import REF_243, REF_260, _one_polygon

    h3 = MosaicContext.build("H3", "JTS")
    for coords, res in ((REF_243, 7), (REF_260, 3)):
        p = _one_polygon(coords)
        host = tessellate("H3", p, res)
        gpu = h3.grid_tessellateexplode(p, res)
        _same(host, gpu)
    assert len(set(gpu["index_id"].tolist())) >= 1
    h3.close()


@pytest.mark.parametrize("res,densify", [(9, 1), (9, 16), (10, 64)])
def test_h3_gpu_tessellation_holes_multipart_duplicates(ctx, res, densify):
    # H3 chips of a holed, two-part geometry whose rings repeat consecutive vertices (zero-length
    # segments), an empty geometry and a plain square, at large densify: GPU producer == host producer
    def sq(x0, y0, s, dup=False):
        r = [(x0, y0), (x0 + s, y0), (x0 + s, y0 + s), (x0, y0 + s), (x0, y0)]
        return r[:2] + [r[1]] + r[2:] if dup else r

    rings = [sq(-73.99, 40.70, 0.045, dup=True), sq(-73.975, 40.715, 0.012)[::-1],
             sq(-73.93, 40.76, 0.02), sq(-73.90, 40.78, 0.015, dup=True), sq(-74.02, 40.62, 0.01)]
    xy = np.array([p for r in rings for p in r], np.float64)
    ring_offsets = np.cumsum([0] + [len(r) for r in rings]).astype(np.int64)
    part_rings = np.array([0, 2, 3, 4, 5], np.int64)
    geom_parts = np.array([0, 2, 2, 3], np.int64)  # geometry 0: holed part + part; 1: empty; 2: square
    polys = PolygonSet(xy, ring_offsets, part_rings, geom_parts)
    h3 = MosaicContext.build("H3", "JTS")
    for keep in (True, False):
        host = tessellate("H3", polys, res, densify=densify, keep_core_geom=keep)
        gpu = tessellate("H3", polys, res, densify=densify, keep_core_geom=keep, ctx=h3)
        _same(host, gpu)
    assert set(gpu["polygon_key"].tolist()) == {0, 2}
    assert gpu["is_core"].sum() > 0 and (gpu["is_core"] == 0).sum() > 0
    h3.close()


def test_gpu_tessellation_small_rings_lane_kernel(ctx):
    """Building-scale inputs go to k_tess_clip_lane (one lane per border cell: every ring <= 24
    vertices, clip polygon <= 12 vertices); rings beyond that, or a densified hexagon of 18 sides,
    to the wave kernel -- both must give the host producer's chip set byte for byte."""
    from mosaic_amd.data import synthetic_buildings

    bld = synthetic_buildings(20_000)
    for res, densify in ((11, 1), (12, 2), (11, 3)):
        host = tessellate("H3", bld, res, densify=densify)
        gpu = tessellate("H3", bld, res, densify=densify, ctx=ctx)
        _same(host, gpu)
        assert (host["is_core"] == 0).sum() > 10_000
    # BNG (clip squares, mode 1): small random polygons in London metres at 10 m cells, some with
    # more than 24 vertices (wave kernel) beside the small ones
    rng = np.random.default_rng(11)
    rings = []
    for i in range(3000):
        cx, cy = rng.uniform(525000, 535000), rng.uniform(175000, 185000)
        nvx = int(rng.integers(3, 40))
        ang = np.sort(rng.uniform(0, 2 * np.pi, nvx))
        rad = rng.uniform(8.0, 40.0, nvx)
        ring = [(cx + r * np.cos(a), cy + r * np.sin(a)) for a, r in zip(ang, rad)]
        rings.append(ring + ring[:1])
    xy = np.array([p for r in rings for p in r], np.float64)
    ring_offsets = np.cumsum([0] + [len(r) for r in rings]).astype(np.int64)
    part_rings = np.arange(len(rings) + 1, dtype=np.int64)
    geom_parts = np.arange(len(rings) + 1, dtype=np.int64)
    polys = PolygonSet(xy, ring_offsets, part_rings, geom_parts)
    host = tessellate("BNG", polys, 5)
    gpu = tessellate("BNG", polys, 5, ctx=ctx)
    _same(host, gpu)
    assert (host["is_core"] == 0).sum() > 10_000
