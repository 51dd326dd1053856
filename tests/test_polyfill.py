"""grid_polyfill (expressions/index/Polyfill.scala -> IndexSystem.polyfill) on the GPU
(mosaic_amd/csrc/polyfill.hip, h3_polyfill.h) against the CPU oracle (oracle/polyfill.c).

H3 (H3IndexSystem.polyfill, core/index/H3IndexSystem.scala:113-126 -> h3-java 3.7.0 polyfill per
polygon part -> H3 C v3.7 _polyfillInternal).  Pins:
  * the reference docs' example (docs/source/api/spatial-indexing.rst:213-221): res 0 of
    MULTIPOLYGON (((30 20, 45 40, 10 40, 30 20)), ((15 5, 40 10, 10 20, 5 10, 15 5))) is the set
    {577586652210266111, 578360708396220415, 577269992861466623}.  The docs list them as
    [A, B, C]; the reference's code path concatenates per-part lists (H3IndexSystem.scala:118-124)
    and B's centre lies in the second part, A's and C's in the first, so that listing cannot come
    from it -- the set is the pin, the order within each part is H3's output-table order;
  * the oracle's independent construction: kRing(1) from the cell geometry (checked against the
    sphere-search k-ring below), so its set and -- when no cell was displaced by probing -- its order
    check the kernel's ring walk, claim order and table emulation;
  * properties: every returned centre is inside (H3's ray cast), every cell whose centre lies
    clearly inside a convex part is returned.
BNG (BNGIndexSystem.polyfill, core/index/BNGIndexSystem.scala:185-204): same set as the oracle's
breadth-first restatement, cells in the Scala 2.12 HashSet order (hash-trie order, restated in
test_scala_set_order)."""
import ctypes
import math
import os
import subprocess

import numpy as np
import pytest

import oracle
from mosaic_amd.data import PolygonSet

DOCS_PARTS = [[[(30, 20), (45, 40), (10, 40), (30, 20)]], [[(15, 5), (40, 10), (10, 20), (5, 10), (15, 5)]]]
DOCS_CELLS = {577586652210266111, 578360708396220415, 577269992861466623}


def polygon_set(geoms):
    """geoms: list of geometries, each a list of parts (lists of rings of (x, y)) -> PolygonSet"""
    xy, ro, pr, gp = [], [0], [0], [0]
    for parts in geoms:
        for rings in parts:
            for r in rings:
                xy.extend(r)
                ro.append(len(xy))
            pr.append(len(ro) - 1)
        gp.append(len(pr) - 1)
    return PolygonSet(np.array(xy, np.float64).reshape(-1, 2), ro, pr, gp)


def oracle_h3(ps, g, res):
    return oracle.h3_polyfill(ps.parts(g), res)


def scala_order_key(v):
    v = int(v)
    iv = ((v & 0xFFFFFFFF) ^ 0x80000000) - 0x80000000
    h = iv if iv == v else (((v ^ (v >> 32)) & 0xFFFFFFFF) ^ 0x80000000) - 0x80000000
    h &= 0xFFFFFFFF
    h = (h + (~(h << 9) & 0xFFFFFFFF)) & 0xFFFFFFFF
    h ^= h >> 14
    h = (h + (h << 4)) & 0xFFFFFFFF
    h ^= h >> 10
    return tuple((h >> (5 * lv)) & 31 for lv in range(7))


# ---- CPU: the oracle ----
def test_oracle_docs_example_res0():
    cells, _ = oracle.h3_polyfill(DOCS_PARTS, 0)
    assert set(cells.tolist()) == DOCS_CELLS and len(cells) == 3
    a, _ = oracle.h3_polyfill_part(DOCS_PARTS[0][0:1], 0)
    b, _ = oracle.h3_polyfill_part(DOCS_PARTS[1][0:1], 0)
    assert set(a.tolist()) == {577586652210266111, 577269992861466623}
    assert b.tolist() == [578360708396220415]


PENTAGON_BASE_CELLS = (4, 14, 24, 38, 49, 58, 63, 72, 83, 97, 107, 117)


def pentagon_cell(bc, res):
    h = (1 << 59) | (res << 52) | (bc << 45)
    for r in range(res + 1, 16):
        h |= 7 << (3 * (15 - r))
    return h


def test_oracle_ring1_matches_sphere_kring():
    rng = np.random.default_rng(7)
    cells = []
    for _ in range(120):
        lat, lon = math.degrees(math.asin(rng.uniform(-1, 1))), rng.uniform(-180, 180)
        res = int(rng.integers(0, 13))
        cells.append(int(oracle.h3_point_to_index(np.array([lon]), np.array([lat]), res)[0]))
    for bc in PENTAGON_BASE_CELLS:
        for res in (0, 2, 5):
            cells += sorted(oracle.h3_kring_set(pentagon_cell(bc, res), 1))
    for c in cells:
        assert set(oracle.h3_ring1(c).tolist()) == set(int(k) for k in oracle.h3_kring_set(c, 1)), c


def pentagon_polygons(radius_deg):
    """an octagon around each pentagon's centre (degrees; lon spread by 1 / cos(lat))"""
    out = []
    for bc in PENTAGON_BASE_CELLS:
        la, lo = (math.degrees(v) for v in oracle.h3_to_geo(pentagon_cell(bc, 0)))
        ring = []
        for i in range(8):
            a = 2 * math.pi * (i + 0.3) / 8
            x = lo + radius_deg * math.cos(a) / math.cos(math.radians(la))
            ring.append((x if x <= 180 else x - 360, la + radius_deg * math.sin(a)))
        ring.append(ring[0])
        out.append((bc, ring))
    return out


def h3_inside(parts, lon, lat):
    """H3 pointInsidePolygon in degrees (no transmeridian), for the property tests"""
    def loop(r):
        inside = False
        n = len(r)
        for i in range(n):
            (ax, ay), (bx, by) = r[i], r[(i + 1) % n]
            if ay > by:
                ax, ay, bx, by = bx, by, ax, ay
            if lat < ay or lat > by or ay == by:
                continue
            if ax + (bx - ax) * (lat - ay) / (by - ay) > lon:
                inside = not inside
        return inside
    return loop(parts[0]) and not any(loop(h) for h in parts[1:])


@pytest.mark.parametrize("res", [8, 9])
def test_oracle_nyc_zone_properties(res):
    zones = PolygonSet.load("nyc_taxi_zones")
    rng = np.random.default_rng(res)
    for g in rng.choice(len(zones), 6, replace=False):
        for rings in zones.parts(int(g)):
            cells, _ = oracle.h3_polyfill_part(rings, res)
            assert len(set(cells.tolist())) == len(cells)
            for c in cells[:200]:
                la, lo = oracle.h3_to_geo(int(c))
                assert h3_inside(rings, math.degrees(lo), math.degrees(la))


def test_oracle_convex_part_complete():
    """every cell whose centre is clearly inside a convex polygon is found"""
    ring = [(-74.0, 40.70), (-73.95, 40.69), (-73.93, 40.74), (-73.97, 40.77), (-74.01, 40.75), (-74.0, 40.70)]
    res = 9
    cells, _ = oracle.h3_polyfill_part([ring], res)
    got = set(cells.tolist())
    xs, ys = np.meshgrid(np.linspace(-74.02, -73.92, 300), np.linspace(40.68, 40.78, 300))
    sample = set(oracle.h3_point_to_index(xs.ravel(), ys.ravel(), res).tolist())
    for c in sample:
        la, lo = oracle.h3_to_geo(c)
        la, lo = math.degrees(la), math.degrees(lo)
        inside = h3_inside([ring], lo, la)
        if inside:
            assert c in got
        elif c in got:
            pytest.fail("outside centre returned")


def test_oracle_bng_polyfill_brute_force():
    """BNG: the breadth-first set equals every cell (of the bbox) whose centre a convex polygon holds"""
    ring = [(530000.0, 180000.0), (534500.0, 179000.0), (536000.0, 183500.0), (531000.0, 185000.0),
            (530000.0, 180000.0)]
    res = 3
    got = oracle.bng_polyfill([[ring]], res)
    e = 1000
    want = []
    wkb = polygon_set([[[ring]]]).wkb(0)
    for x in range(529000, 537000, e):
        for y in range(178000, 186000, e):
            if oracle.wkb_contains(wkb, x + e / 2, y + e / 2):
                want.append(oracle.bng_point_to_index(x + 1, y + 1, res))
    assert sorted(got.tolist()) == sorted(want) and len(want) > 10


def test_scala_set_order_key():
    # hash of a Long that fits in an Int is the Int itself; improve() then 5-bit groups from the low end
    assert scala_order_key(0) == scala_order_key(0)
    keys = [scala_order_key(v) for v in (1, 2, 3, 2 ** 40 + 7)]
    assert len(set(keys)) == 4


@pytest.fixture(scope="module")
def host_polyfill(tmp_path_factory):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = tmp_path_factory.mktemp("h3pf") / "libh3pf.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-Wno-unknown-pragmas", "-shared", "-fPIC",
                    "-I", os.path.join(root, "mosaic_amd", "csrc"), "-o", str(so),
                    os.path.join(root, "tests", "native", "h3_polyfill_host.cpp")], check=True)
    lib = ctypes.CDLL(str(so))
    lib.h3_polyfill_host.restype = ctypes.c_int64
    vp = ctypes.c_void_p
    lib.h3_polyfill_host.argtypes = [vp, vp, vp, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int64]

    def run(rings, res):
        lat = np.concatenate([[oracle.to_radians(v[1]) for v in r] for r in rings]).astype(np.float64)
        lon = np.concatenate([[oracle.to_radians(v[0]) for v in r] for r in rings]).astype(np.float64)
        ro = np.zeros(len(rings) + 1, np.int64)
        np.cumsum([len(r) for r in rings], out=ro[1:])
        out = np.zeros(1 << 20, np.int64)
        n = lib.h3_polyfill_host(lat.ctypes.data, lon.ctypes.data, ro.ctypes.data, len(rings), res, out.ctypes.data,
                                 len(out))
        assert n >= 0
        return out[:n].copy()
    return run


@pytest.mark.parametrize("res", [0, 2, 8, 9])
def test_kernel_code_on_host_matches_oracle(host_polyfill, res):
    """the kernel's device code (h3_polyfill.h, the ring walk, h3_exact, h3ToGeo) compiled for the
    host and run in H3's sequential loop: same cells as the oracle, same order when collision-free"""
    if res <= 2:
        cases = DOCS_PARTS
    else:
        zones = PolygonSet.load("nyc_taxi_zones")
        cases = [p for g in range(0, len(zones), 9) for p in zones.parts(g)]
    n_ordered = 0
    for rings in cases:
        got = host_polyfill(rings, res)
        want, cf = oracle.h3_polyfill_part(rings, res)
        assert sorted(got.tolist()) == sorted(want.tolist())
        if cf:
            assert got.tolist() == want.tolist()
            n_ordered += 1
    assert n_ordered >= len(cases) // 4


@pytest.mark.parametrize("res", [1, 2, 3, 4])
def test_kernel_code_on_host_pentagons(host_polyfill, res):
    """searches through the 12 pentagon base cells (H3's kRing falls back to _kRingInternal there):
    the kernel's code on the host gives the oracle's set, and its order when collision-free"""
    n_ordered = 0
    for bc, ring in pentagon_polygons((12.0, 6.0, 3.0, 1.5)[res - 1]):
        got = host_polyfill([ring], res)
        want, cf = oracle.h3_polyfill_part([ring], res)
        assert len(want) > 5 and pentagon_cell(bc, res) in set(want.tolist()), (bc, res)
        assert sorted(got.tolist()) == sorted(want.tolist()), (bc, res)
        if cf:
            assert got.tolist() == want.tolist(), (bc, res)
            n_ordered += 1


# ---- GPU ----
@pytest.fixture(scope="module")
def h3ctx():
    from mosaic_amd import MosaicContext
    c = MosaicContext.build("H3", "JTS")
    yield c
    c.close()


@pytest.fixture(scope="module")
def bngctx():
    from mosaic_amd import MosaicContext
    c = MosaicContext.build("BNG", "JTS")
    yield c
    c.close()


def _check_h3(gpu_rows, ps, res):
    n_ordered = 0
    for g in range(len(ps)):
        want_parts = [oracle.h3_polyfill_part(r, res) for r in ps.parts(g) if r and len(r[0])]
        want = np.concatenate([w for w, _ in want_parts]) if want_parts else np.zeros(0, np.int64)
        got = gpu_rows[g]
        assert sorted(got.tolist()) == sorted(want.tolist()), g
        if all(cf for _, cf in want_parts):
            assert got.tolist() == want.tolist(), g
            n_ordered += 1
    return n_ordered


@pytest.mark.gpu
def test_gpu_docs_example(h3ctx):
    ps = polygon_set([DOCS_PARTS])
    for res in range(0, 4):
        rows = h3ctx.grid_polyfill(ps, res)
        _check_h3(rows, ps, res)
    assert set(h3ctx.grid_polyfill(ps, 0)[0].tolist()) == DOCS_CELLS


@pytest.mark.gpu
@pytest.mark.parametrize("res", [7, 8, 9, 10])
def test_gpu_nyc_zones_match_oracle(h3ctx, res):
    zones = PolygonSet.load("nyc_taxi_zones")
    if res == 10:
        zones = zones.subset(list(range(0, len(zones), 3)))
    rows = h3ctx.grid_polyfill(zones, res)
    assert len(rows) == len(zones)
    n_ordered = _check_h3(rows, zones, res)
    assert n_ordered > len(zones) // 4
    assert sum(len(r) for r in rows) > 0


@pytest.mark.gpu
def test_gpu_holes_multipart_repeated_vertices(h3ctx):
    shell = [(-74.02, 40.70), (-73.94, 40.70), (-73.94, 40.78), (-74.02, 40.78), (-74.02, 40.70)]
    hole = [(-74.0, 40.72), (-73.98, 40.76), (-73.96, 40.72), (-73.96, 40.72), (-74.0, 40.72)]
    tri = [(-73.90, 40.60), (-73.80, 40.62), (-73.86, 40.70), (-73.86, 40.70), (-73.90, 40.60)]
    empty_part = []
    ps = polygon_set([[[shell, hole], [tri]], [[tri]], [], [[shell]]])
    for res in (8, 9, 10):
        rows = h3ctx.grid_polyfill(ps, res)
        _check_h3(rows, ps, res)
        assert len(rows[2]) == 0
        assert set(rows[0].tolist()) < set(rows[3].tolist()) | set(rows[1].tolist())


@pytest.mark.gpu
def test_gpu_large_res_and_global(h3ctx):
    """coarse cells over a continent (face edges inside the search) and a fine-resolution zone"""
    asia = [(55.0, 30.0), (95.0, 30.0), (100.0, 50.0), (65.0, 55.0), (55.0, 30.0)]
    ps = polygon_set([[[asia]]])
    for res in (0, 1, 2, 3, 4):
        rows = h3ctx.grid_polyfill(ps, res)
        _check_h3(rows, ps, res)
    zones = PolygonSet.load("nyc_taxi_zones").subset([1, 7, 42])
    rows = h3ctx.grid_polyfill(zones, 11)
    _check_h3(rows, zones, 11)


@pytest.mark.gpu
def test_gpu_pentagon_searches(h3ctx):
    """searches entering pentagon base cells (africa at res 0-3, an octagon around each of the 12
    pentagons at res 1-4): the oracle's sets, its order when collision-free"""
    africa = [(-17.0, 14.0), (10.0, 35.0), (32.0, 30.0), (51.0, 11.0), (40.0, -15.0), (20.0, -35.0),
              (12.0, -5.0), (-17.0, 14.0)]
    ps = polygon_set([[[africa]]])
    for res in (0, 1, 2, 3):
        _check_h3(h3ctx.grid_polyfill(ps, res), ps, res)
    for res in (1, 2, 3, 4):
        rings = pentagon_polygons((12.0, 6.0, 3.0, 1.5)[res - 1])
        ps = polygon_set([[[r]] for _, r in rings])
        rows = h3ctx.grid_polyfill(ps, res)
        _check_h3(rows, ps, res)
        for (bc, _), row in zip(rings, rows):
            assert pentagon_cell(bc, res) in set(row.tolist())


@pytest.mark.gpu
@pytest.mark.parametrize("res", [3, 4])
def test_gpu_bng_london(bngctx, res):
    london = PolygonSet.load("london_postcodes_bng")
    sub = london.subset(list(range(0, len(london), 5 if res == 4 else 1)))
    rows = bngctx.grid_polyfill(sub, res, raw=True)
    for g in range(len(sub)):
        want = oracle.bng_polyfill(sub.parts(g), res)
        got = rows[g]
        assert sorted(got.tolist()) == want.tolist(), g
        keys = [scala_order_key(v) for v in got]
        assert keys == sorted(keys)
    s = bngctx.grid_polyfill(sub.subset([0]), res)
    assert all(isinstance(v, str) for v in s[0])


# ---- getBufferRadius (H3IndexSystem.scala:73-80, BNGIndexSystem.scala:146-149) ----
def test_oracle_jts_centroid_cases():
    """JTS 1.19 Centroid (area-weighted triangle fan, shells reset the base point, holes subtract).
    The docs' st_centroid2D example (docs/source/api/spatial-functions.rst:258-262) shows
    {25.454545454545453, 26.96969696969697}; JTS 1.19's cg3.y / 3 / areasum2 rounds y one ulp higher
    (the docs were rendered with another geometry API), so only x is compared with it."""
    cx, cy = oracle.jts_centroid([[[(30, 10), (40, 40), (20, 40), (10, 20), (30, 10)]]])
    assert cx == 25.454545454545453 and abs(cy - 26.96969696969697) <= 4e-15
    assert oracle.jts_centroid([[[(0, 0), (4, 0), (4, 4), (0, 4), (0, 0)]]]) == (2.0, 2.0)
    # a hole removes its area: square 0..4 minus square 0..2 -> centroid (7/3, 7/3)
    cx, cy = oracle.jts_centroid([[[(0, 0), (4, 0), (4, 4), (0, 4), (0, 0)], [(0, 0), (0, 2), (2, 2), (2, 0), (0, 0)]]])
    assert abs(cx - 7 / 3) < 1e-12 and abs(cy - 7 / 3) < 1e-12
    assert oracle.jts_centroid([[[(0, 0), (1, 1), (2, 2), (0, 0)]]]) is None


def test_oracle_buffer_radius_scale():
    zones = PolygonSet.load("nyc_taxi_zones")
    r9 = oracle.h3_buffer_radius(zones.parts(0), 9)
    r10 = oracle.h3_buffer_radius(zones.parts(0), 10)
    assert 0.0015 < r9 < 0.003 and abs(r9 / r10 - math.sqrt(7)) < 0.2


@pytest.mark.gpu
def test_gpu_buffer_radius_matches_oracle(h3ctx, bngctx):
    zones = PolygonSet.load("nyc_taxi_zones")
    for res in (0, 5, 9, 11, 13):
        got = h3ctx.buffer_radius(zones, res)
        want = np.array([oracle.h3_buffer_radius(zones.parts(g), res) for g in range(len(zones))])
        assert np.array_equal(got, want), res
    london = PolygonSet.load("london_postcodes_bng")
    assert np.all(bngctx.buffer_radius(london, 4) == 100 * math.sqrt(2) / 2)
