"""st_intersects_aggregate (§8(f) row 4): the chip-join aggregate of two chip sets.

Reference: ST_IntersectsAggregate.update (expressions/geometry/ST_IntersectsAggregate.scala:28-39)
folds ``left.is_core || right.is_core || left.wkb intersects right.wkb`` with OR over the equi-join
of two mosaic_explode outputs on index_id, grouped by (left id, right id)
(ST_IntersectsBehaviors.scala:34-47).  Pinned by the reference's own tests:
  * intersectsAggBehaviour (ST_IntersectsBehaviors.scala:85-134): five chip rows -> flags
    [true, true, true, true, false];
  * intersectsBehaviour (:13-61): the aggregate equals flat st_intersects of the original polygons
    for every joined (left, right) group (boroughs vs randomly translated boroughs);
and the oracle's segment predicate against exact rational arithmetic (oracle/exact.py).
CPU tests check the oracle; the GPU tests (marked gpu) run mosaic_intersects_aggregate through
the C ABI against it."""
import struct

import numpy as np
import pytest

import oracle
from oracle import exact
from mosaic_amd.context import tessellate
from mosaic_amd.data import PolygonSet


def _poly_wkb(rings):
    out = struct.pack("<BII", 1, 3, len(rings))
    for r in rings:
        out += struct.pack("<I", len(r)) + b"".join(struct.pack("<dd", x, y) for x, y in r)
    return out


def _square(x0, y0, s):
    return [(x0, y0), (x0 + s, y0), (x0 + s, y0 + s), (x0, y0 + s), (x0, y0)]


def _agg_rows():
    """ST_IntersectsBehaviors.scala:85-134 with BNG-like square cells: chip = the cell's shell
    without vertex 2 (a triangle).  Row k: (left core, left cell, left geometry, right core, right
    cell, right geometry); expected flags [true, true, true, true, false]."""
    cell1, cell2 = 1001, 1002
    sq1, sq2 = _square(0.0, 0.0, 100.0), _square(300.0, 0.0, 100.0)
    tri1 = [p for i, p in enumerate(sq1) if i != 2]
    tri2 = [p for i, p in enumerate(sq2) if i != 2]
    P1, P2, C1, C2 = _poly_wkb([sq1]), _poly_wkb([sq2]), _poly_wkb([tri1]), _poly_wkb([tri2])
    rows = [(True, cell1, P1, True, cell1, P1), (False, cell1, C1, True, cell1, P1),
            (True, cell2, P2, False, cell2, C2), (False, cell2, C2, False, cell2, C2),
            (False, cell2, C1, False, cell2, C2)]
    return rows, [True, True, True, True, False]


def _side(rows, which):
    o = 0 if which == "left" else 3
    wkbs = [r[o + 2] for r in rows]
    offs = np.zeros(len(wkbs) + 1, np.int64)
    np.cumsum([len(w) for w in wkbs], out=offs[1:])
    return dict(index_id=np.array([r[o + 1] for r in rows], np.int64),
                is_core=np.array([r[o] for r in rows], np.uint8),
                polygon_key=np.arange(len(rows), dtype=np.int32),
                wkb=(offs, np.frombuffer(b"".join(wkbs), np.uint8)))


def test_oracle_agg_rows_match_reference_flags(oracle_lib):
    rows, expect = _agg_rows()
    got = oracle.intersects_aggregate(_side(rows, "left"), _side(rows, "right"))
    assert [got[(k, k)] for k in range(len(rows))] == expect


def test_oracle_segments_match_exact_rationals(oracle_lib):
    rng = np.random.default_rng(11)
    cases = 0
    for _ in range(3000):
        # integer-grid segments (many exact touches / collinear overlaps) and near-degenerate ones
        if rng.random() < 0.5:
            pts = [tuple(float(v) for v in rng.integers(0, 6, 2)) for _ in range(4)]
        else:
            a = rng.random(2)
            b = rng.random(2)
            t = rng.random()
            m = a + t * (b - a)  # a point on (or within rounding of) segment ab
            d = rng.random(2) - 0.5
            pts = [tuple(a), tuple(b), tuple(m), tuple(m + d)]
        p1, p2, q1, q2 = pts
        assert oracle.segments_intersect(p1, p2, q1, q2) == exact.segments_intersect(p1, p2, q1, q2), pts
        cases += 1
    assert cases == 3000


def _chips_dict(chips):
    return dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
                wkb=chips["wkb"])


def _translated(zones, dx, dy):
    return PolygonSet(zones.xy + np.array([dx, dy]), zones.ring_offsets, zones.part_rings, zones.geom_parts,
                      zones.names)


def test_oracle_agg_equals_flat_intersects(oracle_lib):
    """intersectsBehaviour's invariant on the reference's 35 NYC zones (H3 res 8 chips) against
    a translated copy: every joined group's aggregate equals flat intersects of the polygons."""
    zones = PolygonSet.load("nyc_taxi_zones_35")
    moved = _translated(zones, 0.0031, 0.0017)
    left = tessellate("H3", zones, 8)
    right = tessellate("H3", moved, 8)
    agg = oracle.intersects_aggregate(_chips_dict(left), _chips_dict(right))
    assert len(agg) > 35
    n_true = 0
    for (ka, kb), flag in agg.items():
        assert flag == oracle.wkb_intersects(zones.wkb(ka), moved.wkb(kb)), (ka, kb)
        n_true += flag
    assert 0 < n_true < len(agg)


# ---- GPU: mosaic_intersects_aggregate through the C ABI ----

@pytest.fixture(scope="module")
def ctx():
    from mosaic_amd import MosaicContext

    c = MosaicContext.build("H3")
    yield c
    c.close()


def _table(ctx, chips, res):
    return ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], res)


@pytest.mark.gpu
def test_gpu_agg_rows_match_reference_flags(ctx):
    rows, expect = _agg_rows()
    # real res-5 H3 cells stand in for the reference's two index ids (the aggregate never decodes them)
    cells = oracle.h3_point_to_index(np.array([0.0, 10.0]), np.array([0.0, 10.0]), 5)
    rows = [(a, int(cells[0] if c1 == 1001 else cells[1]), g1, b, int(cells[0] if c2 == 1001 else cells[1]), g2)
            for a, c1, g1, b, c2, g2 in rows]
    left, right = _side(rows, "left"), _side(rows, "right")
    lk, rk, fl = ctx.st_intersects_aggregate(_table(ctx, left, 5), _table(ctx, right, 5))
    got = {(int(a), int(b)): bool(f) for a, b, f in zip(lk, rk, fl)}
    assert got == oracle.intersects_aggregate(left, right)
    assert [got[(k, k)] for k in range(len(rows))] == expect


@pytest.mark.gpu
@pytest.mark.parametrize("name,res,shift", [("nyc_taxi_zones_35", 8, (0.0031, 0.0017)),
                                            ("nyc_taxi_zones", 9, (0.0007, -0.0011)),
                                            ("nyc_taxi_zones", 9, (0.0, 0.0))])
def test_gpu_agg_matches_oracle(ctx, name, res, shift):
    """GPU groups == the oracle's groups and flags, bit for bit; shift (0, 0) joins the zones with
    themselves (every chip pair of a cell shares boundary: touching and collinear segments)."""
    zones = PolygonSet.load(name)
    moved = _translated(zones, *shift)
    left, right = tessellate("H3", zones, res), tessellate("H3", moved, res)
    lk, rk, fl = ctx.st_intersects_aggregate(_table(ctx, left, res), _table(ctx, right, res))
    got = {(int(a), int(b)): bool(f) for a, b, f in zip(lk, rk, fl)}
    want = oracle.intersects_aggregate(_chips_dict(left), _chips_dict(right))
    assert got == want
    assert list(zip(lk, rk)) == sorted(zip(lk, rk))


def test_quickstart_points_small_zone_sets():
    """__graft_entry__.smoke() draws its points from 21 zones: fewer than the 32 mixture centres."""
    from mosaic_amd.data import quickstart_points

    zones = PolygonSet.load("nyc_taxi_zones")
    x, y = quickstart_points(zones.subset(list(range(0, 263, 13))), 20000, seed=1)
    assert len(x) == len(y) == 20000 and np.isfinite(x).all()
    a = quickstart_points(zones, 1000, seed=3)
    b = quickstart_points(zones, 1000, seed=3)
    assert np.array_equal(a[0], b[0])
