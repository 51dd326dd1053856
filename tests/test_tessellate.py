"""Chip production (host) against the reference's invariant, CPU only.

MosaicFrameBehaviors.scala:136-223 asserts: chip-join row count == brute-force st_contains join
row count (99 taxi trips x 35 zones, H3 res 8 / BNG res 3).  Here the chip join and the brute force
are both evaluated by the CPU oracle; the chips come from the product's tessellator.
"""
import numpy as np
import pytest

import oracle
from mosaic_amd import wkb as W
from mosaic_amd.context import tessellate
from mosaic_amd.data import PolygonSet, quickstart_points


def _as_oracle(chips):
    offs, data = chips["wkb"]
    return dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
                wkb_offsets=offs, wkb=data)


@pytest.fixture(scope="module")
def zones35():
    return PolygonSet.load("nyc_taxi_zones_35")


def test_reference_join_invariant_h3_res8(zones35):
    trips = np.load("tests/golden/nyctaxi_yellow_trips_pickups.npy")
    chips = tessellate("H3", zones35, 8)
    want, total_bf = oracle.brute_force_count(zones35, trips[:, 0], trips[:, 1])
    got, total = oracle.pip_join(_as_oracle(chips), oracle.GRID_H3, 8, trips[:, 0], trips[:, 1], len(zones35))
    assert total == total_bf
    assert np.array_equal(got, want)


@pytest.mark.parametrize("res,densify", [(8, 8), (9, 8), (9, 1)])
def test_chip_join_equals_brute_force_random(zones35, res, densify):
    chips = tessellate("H3", zones35, res, densify=densify)
    x, y = quickstart_points(zones35, 100_000, seed=res)
    want, total_bf = oracle.brute_force_count(zones35, x, y)
    got, total = oracle.pip_join(_as_oracle(chips), oracle.GRID_H3, res, x, y, len(zones35), threads=8)
    # every mismatch would be a point within ~1e-8 degrees of a cell edge (the chip boundary follows
    # straight lon/lat chords while H3 cell edges are great-circle arcs); none on this sample
    assert np.abs(got - want).sum() <= (0 if densify > 1 else 2)
    assert total_bf > 10_000


def test_chip_structure(zones35):
    chips = tessellate("H3", zones35, 9)
    offs, data = chips["wkb"]
    n = len(chips["index_id"])
    assert n > 1000
    # every index id is a res-9 H3 cell
    assert np.all((chips["index_id"] >> 52 & 15) == 9)
    # core chips are whole cells: the cell of the core chip's own centroid is that chip's id
    core = np.nonzero(chips["is_core"])[0][:200]
    for i in core:
        kind, parts = W.read_wkb(data[offs[i]:offs[i + 1]].tobytes())
        ring = np.array(parts[0][0][:-1])
        cx, cy = ring.mean(0)
        assert int(oracle.h3_point_to_index([cx], [cy], 9)[0]) == chips["index_id"][i]
    # one chip per (zone, cell)
    pairs = set(zip(chips["polygon_key"].tolist(), chips["index_id"].tolist()))
    assert len(pairs) == n


def test_keep_core_geom_false(zones35):
    chips = tessellate("H3", zones35, 9, keep_core_geom=False)
    offs, _ = chips["wkb"]
    lens = np.diff(offs)
    assert np.all(lens[chips["is_core"] == 1] == 0)
    assert np.all(lens[chips["is_core"] == 0] > 0)


def test_bng_tessellation_invariant():
    # the London postcode zones in EPSG:27700 metres (tests/golden/make_bng_fixture.py)
    proj = PolygonSet.load("london_postcodes_bng").subset(range(0, 177, 6))
    chips = tessellate("BNG", proj, 3)
    rng = np.random.default_rng(0)
    x0, y0, x1, y1 = proj.bbox()
    x = rng.uniform(x0, x1, 50_000)
    y = rng.uniform(y0, y1, 50_000)
    want, total_bf = oracle.brute_force_count(proj, x, y)
    got, total = oracle.pip_join(_as_oracle(chips), oracle.GRID_BNG, 3, x, y, len(proj), threads=8)
    assert np.array_equal(got, want) and total_bf > 1000


def test_tessellate_errors():
    from mosaic_amd import IllegalStateException

    z = PolygonSet.load("nyc_taxi_zones_35").subset([0])
    with pytest.raises(IllegalStateException, match="found 16"):
        tessellate("H3", z, 16)
    with pytest.raises(IllegalStateException, match="BNG resolution not supported"):
        tessellate("BNG", z, 0)


def _one_polygon(coords):
    xy = np.array(coords, np.float64)
    return PolygonSet(xy, [0, len(xy)], [0, 1], [0, 1])


# The reference's own tessellation regression fixtures (WKT coordinates copied as data):
# issue #243, core/TestMosaic.scala:9-16 -- mosaicFill at H3 res 7 gives 10 chips, all distinct
REF_243 = [(4.42, 51.78), (4.38, 51.78), (4.39, 51.83), (4.40, 51.83), (4.41, 51.8303), (4.417, 51.8295),
           (4.42, 51.83), (4.44, 51.81), (4.42, 51.78)]
# issue #260, expressions/index/MosaicFillBehaviors.scala:177-195 -- grid_tessellate at res 3 has > 0 chips
REF_260 = [(5.26, 52.72), (5.20, 52.71), (5.21, 52.75), (5.26, 52.75), (5.26, 52.72)]


def test_reference_tessellation_fixtures():
    c = tessellate("H3", _one_polygon(REF_243), 7)
    assert len(c["index_id"]) == 10 and len(set(c["index_id"].tolist())) == 10
    c = tessellate("H3", _one_polygon(REF_260), 3)
    assert len(c["index_id"]) > 0
    # every chip's polygon key is the input geometry and its cell holds part of the polygon
    assert set(c["polygon_key"].tolist()) == {0}


def test_chip_set_zero_copy_lifetime():
    """tessellate()'s arrays view the chip set's own columns (mosaic_chip_set_columns): the set lives
    until the last array is collected, and the views equal a copying export of the same set."""
    import gc

    from mosaic_amd.data import PolygonSet

    zones = PolygonSet.load("nyc_taxi_zones_35")
    a = tessellate("H3", zones, 8)
    b = tessellate("H3", zones, 8)
    wkb_offs, wkb = a["wkb"]
    ids = a["index_id"].copy()
    del a
    gc.collect()
    _ = [np.zeros(1 << 16) for _ in range(64)]  # reuse freed memory, if any were freed
    assert np.array_equal(wkb_offs, b["wkb"][0]) and np.array_equal(wkb, b["wkb"][1])
    assert np.array_equal(ids, b["index_id"])
    assert wkb_offs[-1] == len(wkb) and wkb_offs[0] == 0
