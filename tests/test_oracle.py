"""Pins the CPU oracle against the reference's golden vectors (CPU only, no GPU)."""
import json
import math
import os
import random

import numpy as np
import pytest

from mosaic_amd import wkb as W

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_vectors.json")))


# ---------------- H3 ----------------
@pytest.mark.parametrize("case", GOLD["h3_point_to_cell"], ids=lambda c: f"{c['lon']},{c['lat']},r{c['res']}")
@pytest.mark.parametrize("jdk", [8, 11])
def test_h3_known_answers(oracle_lib, case, jdk):
    got = oracle_lib.h3_point_to_index([case["lon"]], [case["lat"]], case["res"], jdk=jdk)[0]
    assert int(got) == case["cell"], (hex(int(got)), hex(case["cell"]), case["source"])


def _base_cell(h):
    return (h >> 45) & 127


def test_h3_res0_base_cells_cover_globe(oracle_lib):
    lat = np.repeat(np.arange(-89.5, 90, 1.0), 360)
    lon = np.tile(np.arange(-179.5, 180, 1.0), 180)
    cells = oracle_lib.h3_point_to_index(lon, lat, 0)
    assert set(_base_cell(int(c)) for c in cells) == set(range(122))
    # res-0 ids: mode 1, res 0, all 15 digits unused (7)
    assert all((int(c) & ((1 << 45) - 1)) == (1 << 45) - 1 for c in cells[:100])


def test_h3_res0_docs_polyfill_and_tessellate(oracle_lib):
    """The docs' res-0 polyfill cells are exactly the base cells whose centres fall inside the
    multipolygon, and every tessellated cell is touched by it (spatial-indexing.rst:213-221, 546-556)."""
    parts = W.read_wkt("MULTIPOLYGON (((30 20, 45 40, 10 40, 30 20)), ((15 5, 40 10, 10 20, 5 10, 15 5)))")[1]
    from oracle import exact

    # sample the multipolygon densely; every sampled point's res-0 cell must be in the tessellation
    rng = np.random.default_rng(1)
    pts = []
    while len(pts) < 4000:
        x, y = rng.uniform(5, 45), rng.uniform(5, 40)
        if exact.contains(parts, (x, y)):
            pts.append((x, y))
    pts = np.array(pts)
    cells = set(int(c) for c in oracle_lib.h3_point_to_index(pts[:, 0], pts[:, 1], 0))
    assert cells <= set(GOLD["h3_res0_tessellate"])
    assert set(GOLD["h3_res0_polyfill"]) <= cells


def test_h3_nonfinite_is_null(oracle_lib):
    out = oracle_lib.h3_point_to_index([float("nan"), 1.0, float("inf")], [1.0, float("nan"), 2.0], 9)
    assert list(out) == [0, 0, 0]
    assert oracle_lib.h3_geo_to_h3(0.1, 0.1, 16) == 0
    assert oracle_lib.h3_geo_to_h3(0.1, 0.1, -1) == 0


def test_h3_parent_child_consistency(oracle_lib):
    """Structural invariant: the res r cell of a point is the parent (digit truncation) of its
    res r+1 cell, away from cell edges -- checked on points at cell centres' neighbourhood."""
    rng = np.random.default_rng(7)
    lon = rng.uniform(-180, 180, 2000)
    lat = np.degrees(np.arcsin(rng.uniform(-1, 1, 2000)))
    for res in (3, 6, 9):
        fine = oracle_lib.h3_point_to_index(lon, lat, res + 1)
        coarse = oracle_lib.h3_point_to_index(lon, lat, res)
        # H3 parents are not geometric containers (aperture 7): only compare the base cell, which is
        # stable away from base-cell edges, and the 'unused digit' padding.
        assert np.all((coarse >> 52 & 15) == res)
        agree = np.mean([_base_cell(int(a)) == _base_cell(int(b)) for a, b in zip(fine, coarse)])
        assert agree > 0.99


# ---------------- BNG ----------------
@pytest.mark.parametrize("case", GOLD["bng_point_to_index"], ids=lambda c: f"r{c['res']}")
def test_bng_golden(oracle_lib, case):
    got = oracle_lib.bng_point_to_index(case["e"], case["n"], case["res"])
    assert got == case["id"]
    assert oracle_lib.bng_format(got) == case["fmt"]


def test_bng_nan_and_bad_res(oracle_lib):
    with pytest.raises(ValueError, match="NaN coordinates are not supported."):
        oracle_lib.bng_point_to_index(float("nan"), 100.0, 5)
    with pytest.raises(ValueError, match="NaN coordinates are not supported."):
        oracle_lib.bng_point_to_index(100.0, float("nan"), 5)
    with pytest.raises(ValueError, match="BNG resolution not supported"):
        oracle_lib.bng_point_to_index(100.0, 100.0, 0)


def test_bng_out_of_range_still_encodes(oracle_lib):
    # TestBNGIndexSystem.scala:156-161 / SURVEY a7: (-50000, 50, 3) -> 999950000
    assert oracle_lib.bng_point_to_index(-50000.0, 50.0, 3) == 999950000
    assert oracle_lib.bng_point_to_index(50.0, 500000000.0, 4) > 0


# ---------------- JTS contains ----------------
def test_contains_golden(oracle_lib):
    poly = W.read_wkt(GOLD["contains"]["polygon"])[1]
    wkb = W.geometry_wkb(poly)
    for pt, expected in GOLD["contains"]["cases"]:
        x, y = W.read_wkt(pt)[1]
        assert oracle_lib.wkb_contains(wkb, x, y) == expected
        assert oracle_lib.wkb_contains(W.geometry_wkb(poly, big_endian=False), x, y) == expected


def test_contains_boundary_semantics(oracle_lib):
    sq = [[(0.0, 0.0), (10.0, 0.0), (10.0, 10.0), (0.0, 10.0), (0.0, 0.0)]]
    wkb = W.geometry_wkb([sq])
    assert oracle_lib.wkb_contains(wkb, 5, 5)
    for p in [(0, 0), (5, 0), (10, 5), (0, 10), (10, 10), (0, 5)]:
        assert not oracle_lib.wkb_contains(wkb, *p), p  # boundary -> false
    assert not oracle_lib.wkb_contains(wkb, 11, 5)
    # MultiPolygon: two squares touching at a vertex: Mod-2 rule -> the shared vertex is interior
    sq2 = [[(10.0, 10.0), (20.0, 10.0), (20.0, 20.0), (10.0, 20.0), (10.0, 10.0)]]
    mp = W.geometry_wkb([sq, sq2])
    assert oracle_lib.wkb_contains(mp, 10, 10)
    assert not oracle_lib.wkb_contains(mp, 10, 5)
    # empty polygon
    assert not oracle_lib.wkb_contains(W.geometry_wkb([[]]), 0, 0)


def test_contains_matches_exact_rationals(oracle_lib):
    """Random rings, points snapped onto edges/vertices and near them: the C oracle (FP filter +
    JTS double-double) agrees with exact rational arithmetic."""
    from oracle import exact

    rng = random.Random(3)
    for trial in range(150):
        n = rng.randint(3, 12)
        cx, cy = rng.uniform(-75, -73), rng.uniform(40, 41)
        angs = sorted(rng.uniform(0, 2 * math.pi) for _ in range(n))
        ring = [(cx + rng.uniform(0.001, 0.01) * math.cos(a), cy + rng.uniform(0.001, 0.01) * math.sin(a))
                for a in angs]
        ring.append(ring[0])
        parts = [[ring]]
        wkb = W.geometry_wkb(parts)
        pts = []
        for _ in range(30):
            i = rng.randrange(n)
            (x1, y1), (x2, y2) = ring[i], ring[i + 1]
            t = rng.random()
            kind = rng.random()
            if kind < 0.3:
                pts.append(ring[i])
            elif kind < 0.6:
                pts.append((x1 + t * (x2 - x1), y1 + t * (y2 - y1)))  # near/on an edge (rounded)
            elif kind < 0.7:
                pts.append((x1, rng.uniform(cy - 0.01, cy + 0.01)))  # same x as a vertex
            elif kind < 0.8:
                pts.append((rng.uniform(cx - 0.01, cx + 0.01), y1))  # same y as a vertex
            else:
                pts.append((rng.uniform(cx - 0.012, cx + 0.012), rng.uniform(cy - 0.012, cy + 0.012)))
        for p in pts:
            assert oracle_lib.wkb_contains(wkb, *p) == exact.contains(parts, p), (trial, p)


def test_orientation_filter_and_dd(oracle_lib):
    assert oracle_lib.orientation_index((0, 0), (1, 1), (2, 2)) == 0
    assert oracle_lib.orientation_index((0, 0), (1, 0), (0, 1)) == 1
    assert oracle_lib.orientation_index((0, 0), (1, 0), (0, -1)) == -1
    # nearly collinear: forces the double-double path
    p1, p2 = (-74.18445299999996, 40.694995999999904), (-74.18448899999999, 40.69509499999987)
    t = 0.3
    q = (p1[0] + t * (p2[0] - p1[0]), p1[1] + t * (p2[1] - p1[1]))
    from oracle import exact

    assert oracle_lib.orientation_index(p1, p2, q) == exact.orientation(p1, p2, q)
