"""st_intersection_aggregate (§8(f) row 4): the union the reference's ST_IntersectionAggregate.update /
merge builds per (left id, right id) group of the chip join (expressions/geometry/
ST_IntersectionAggregate.scala:40-72) -- its area, the quantity the reference's tests check within 1e-8
(ST_IntersectionBehaviors.scala:22-71 intersectionBehaviour, :73-135 intersectionAggBehaviour), and
its geometry as WKB.  The geometry's vertex order cannot be pinned (the reference's depends on Spark's
aggregation order), so it is pinned as a set: the symmetric difference between the engine's polygons
and the exact per-cell union (oracle/exact.py symdiff_area, float slabs) must be ~0, and pieces of
adjacent cells must be dissolved into one polygon.

The engine computes per (group, cell) the piece of the union -- the cell for a (core, core) pair, else
(the group's left chips there, or the cell when one is core) n (its right chips, likewise) -- by an
arrangement overlay (overlay.h, one GPU lane per cell) whose boundary edges the host stitches across
cells (isect_geom.cpp); the area is the sum of the pieces' areas.  The checkers are different
algorithms: exact rational vertical slabs (oracle/exact.py intersection_area) and float slabs of the
symmetric difference (symdiff_area), between all vertex and crossing abscissae, where section lengths
are linear and the midpoint rule exact.  Pins: intersectionAggBehaviour's chip rows (H3 cells with vertex 2 dropped)
must give the union area of the four geometries, and intersectionBehaviour's invariant -- the
aggregate over the chips of two polygons equals the area of the polygons' flat intersection --
on NYC zones against a translated copy."""
import ctypes
import math
import os
import struct
import subprocess

import numpy as np
import pytest

import oracle
from oracle import exact
from mosaic_amd.context import tessellate
from mosaic_amd.data import PolygonSet
from mosaic_amd.wkb import read_wkb


def _poly_wkb(rings):
    out = struct.pack("<BII", 1, 3, len(rings))
    for r in rings:
        out += struct.pack("<I", len(r)) + b"".join(struct.pack("<dd", x, y) for x, y in r)
    return out


def _tri(x0, y0, s):
    return [(x0, y0), (x0 + s, y0), (x0, y0 + s), (x0, y0)]


def test_exact_area_cases():
    sq = lambda x0, y0, s: [(x0, y0), (x0 + s, y0), (x0 + s, y0 + s), (x0, y0 + s), (x0, y0)]
    assert exact.intersection_area([[sq(0, 0, 2)]], [[sq(1, 1, 2)]]) == 1
    assert exact.intersection_area([[sq(0, 0, 2)]], [[sq(2, 0, 2)]]) == 0  # shared edge only
    assert exact.intersection_area([[sq(0, 0, 4), sq(1, 1, 1)]], [[sq(0, 0, 4)]]) == 15  # hole
    assert exact.intersection_area([[_tri(0, 0, 2)]], [[sq(0, 0, 1)]]) == 1
    # an L-shape against a square straddling its notch
    ell = [(0, 0), (3, 0), (3, 1), (1, 1), (1, 3), (0, 3), (0, 0)]
    assert exact.intersection_area([[ell]], [[sq(0.5, 0.5, 2)]]) == 1.75


def _parts_arrays(parts):
    rings = [r for p in parts for r in p]
    xy = np.ascontiguousarray(np.concatenate([np.asarray(r, float) for r in rings]))
    ro = np.zeros(len(rings) + 1, np.int64)
    np.cumsum([len(r) for r in rings], out=ro[1:])
    pr = np.zeros(len(parts) + 1, np.int64)
    np.cumsum([len(p) for p in parts], out=pr[1:])
    return xy, ro, pr


def _chip_index(chips):
    """(key, cell) -> [(is_core, parts)] in row order"""
    offs, data = chips["wkb"]
    d = {}
    for i in range(len(chips["index_id"])):
        w = bytes(data[offs[i]:offs[i + 1]])
        parts = read_wkb(w)[1] if len(w) else []
        d.setdefault((int(chips["polygon_key"][i]), int(chips["index_id"][i])), []).append((int(chips["is_core"][i]), parts))
    return d


def oracle_aggregate(left, right):
    """{(left key, right key): area} of the union of the cells' increments: exact rationals for cells
    with one pair, the float slab area of the union for cells with several"""
    out = {}
    for g, units in _units(_chip_index(left), _chip_index(right)).items():
        area = 0
        for cell, lv, rv in units:
            a, b, need = _increments(lv, rv, cell)
            if len(lv) * len(rv) > 1 and need == 3:
                area += exact.symdiff_area([], [(a, b)])[1]
            elif need == 3:
                area += float(exact.intersection_area(a, b))
            else:
                area += float(exact.polygon_area(a if need == 1 else b))
        out[g] = area
    return out


def _translated(ps, f=0.1):
    """st_translate(wkt, sqrt(st_area(wkt) * 0.1), ...) per geometry (ST_IntersectionBehaviors.scala:39-41)"""
    xy = ps.xy.copy()
    for g in range(len(ps)):
        d = math.sqrt(float(exact.polygon_area(ps.parts(g))) * f)
        a = ps.ring_offsets[ps.part_rings[ps.geom_parts[g]]]
        b = ps.ring_offsets[ps.part_rings[ps.geom_parts[g + 1]]]
        xy[a:b] += d
    return PolygonSet(xy, ps.ring_offsets, ps.part_rings, ps.geom_parts)


@pytest.fixture(scope="module")
def h3ctx():
    from mosaic_amd import MosaicContext
    c = MosaicContext.build("H3", "JTS")
    yield c
    c.close()


@pytest.mark.gpu
def test_gpu_intersection_agg_reference_rows(h3ctx):
    """intersectionAggBehaviour: two H3 cells, each as a core chip (its polygon) and as a border chip
    (its shell without vertex 2); all rows one group -> the union area of the four geometries"""
    ids = [608726199203528703, 608726199220305919]
    res = (ids[0] >> 52) & 15
    polys, chips = [], []
    for c in ids:
        b = oracle.h3_to_geo_boundary(c)
        ring = [(math.degrees(lo), math.degrees(la)) for la, lo in b]
        ring.append(ring[0])
        polys.append(ring)
        chips.append([p for i, p in enumerate(ring) if i != 2])
    rows_core = [1, 1, 0, 0]
    rows_id = [ids[0], ids[1], ids[0], ids[1]]
    rows_wkb = [_poly_wkb([polys[0]]), _poly_wkb([polys[1]]), _poly_wkb([chips[0]]), _poly_wkb([chips[1]])]
    left = h3ctx.chip_table(rows_core, rows_id, rows_wkb, [0, 0, 0, 0], res, n_polygons=1)
    right = h3ctx.chip_table(rows_core, rows_id, rows_wkb, [0, 0, 0, 0], res, n_polygons=1)
    lk, rk, area, st = h3ctx.st_intersection_aggregate_area(left, right)
    assert list(lk) == [0] and list(rk) == [0] and list(st) == [0]
    union = float(exact.polygon_area([[polys[0]]]) + exact.polygon_area([[polys[1]]]))
    assert abs(area[0] - union) < 1e-7  # the reference's bound (10e-8)
    # a cell holding two border-chip pairs of one group and no (core, core) pair: the union of the
    # two (identical) pieces, through the cell overlay (round 4 refused it)
    left2 = h3ctx.chip_table([0, 0], [ids[0], ids[0]], [rows_wkb[2], rows_wkb[2]], [0, 0], res, n_polygons=1)
    right2 = h3ctx.chip_table([0], [ids[0]], [rows_wkb[2]], [0], res, n_polygons=1)
    _, _, a2, s2 = h3ctx.st_intersection_aggregate_area(left2, right2)
    assert list(s2) == [0] and abs(a2[0] - float(exact.polygon_area([[chips[0]]]))) < 1e-12
    lk, rk, area, st, wkb = h3ctx.st_intersection_aggregate(left, right)
    assert list(st) == [0] and abs(area[0] - union) < 1e-7
    kind, parts = read_wkb(wkb[0])
    assert len(parts) == 1 and abs(float(exact.polygon_area(parts)) - union) < 1e-7  # the two cells, dissolved
    for t in (left, right, left2, right2):
        t.close()


@pytest.mark.gpu
def test_gpu_intersection_agg_nyc_zones(h3ctx):
    """intersectionBehaviour on NYC zones at res 8: engine == exact per-cell aggregate for every
    group; aggregate == the flat intersection area of the original polygons (the reference's
    invariant, 1e-8) for the groups of a polygon with its own translated copy"""
    # valid single-polygon zones (the flat-intersection invariant below needs JTS-valid input)
    zones = PolygonSet.load("nyc_taxi_zones").subset([3, 7, 9, 11, 15, 23, 24, 40])
    moved = _translated(zones)
    res = 8
    lc = tessellate("H3", zones, res, ctx=h3ctx)
    rc = tessellate("H3", moved, res, ctx=h3ctx)
    left = h3ctx.chip_table(lc["is_core"], lc["index_id"], list(_wkb_list(lc)), lc["polygon_key"], res,
                            n_polygons=len(zones))
    right = h3ctx.chip_table(rc["is_core"], rc["index_id"], list(_wkb_list(rc)), rc["polygon_key"], res,
                             n_polygons=len(zones))
    lk, rk, area, st = h3ctx.st_intersection_aggregate_area(left, right)
    want = oracle_aggregate(lc, rc)
    assert set(zip(lk.tolist(), rk.tolist())) == set(want)
    assert len(want) > 0 and not st.any()
    for a, b, v in zip(lk, rk, area):
        w = want[(int(a), int(b))]
        assert abs(v - w) <= 1e-13 + 1e-9 * abs(w), (a, b, v, w)
    checked = 0
    for a, b, v, s in zip(lk, rk, area, st):
        if a == b and not s:
            flat = exact.intersection_area(zones.parts(int(a)), moved.parts(int(b)))
            assert abs(v - float(flat)) <= 1e-8, (a, v, float(flat))
            checked += 1
    assert checked >= 4
    # each group's pieces are summed on the host in cell order: the same bits on every call
    for _ in range(3):
        lk2, rk2, area2, st2 = h3ctx.st_intersection_aggregate_area(left, right)
        assert np.array_equal(lk2, lk) and np.array_equal(rk2, rk) and np.array_equal(st2, st)
        assert np.array_equal(area2.view(np.uint64), area.view(np.uint64))
    left.close()
    right.close()


def _wkb_list(chips):
    offs, data = chips["wkb"]
    return [bytes(data[offs[i]:offs[i + 1]]) for i in range(len(offs) - 1)]


# ---- the union's geometry (overlay.h per cell, isect_geom.cpp across cells) ----

def _build_so(tmp_path_factory, name, sources):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = tmp_path_factory.mktemp(name) / f"lib{name}.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-shared", "-fPIC", "-I",
                    os.path.join(root, "mosaic_amd", "csrc"), "-o", str(so)] + [os.path.join(root, s) for s in sources],
                   check=True)
    return ctypes.CDLL(str(so))


def _flat(parts):
    if not parts:
        return np.zeros(2), np.zeros(1, np.int64), np.zeros(1, np.int64)
    return _parts_arrays(parts)


@pytest.fixture(scope="module")
def host_overlay(tmp_path_factory):
    """overlay.h compiled for the host: (A parts, B parts, need) -> (directed edges, area)"""
    lib = _build_so(tmp_path_factory, "ov", ["tests/native/overlay_host.cpp"])
    vp, i = ctypes.c_void_p, ctypes.c_int
    lib.overlay_host.restype = ctypes.c_int
    lib.overlay_host.argtypes = [vp, vp, i, vp, i, vp, vp, i, vp, i, i, vp, i, vp]

    def run(a, b, need):
        xa, ra, pa = _flat(a)
        xb, rb, pb = _flat(b)
        out = np.zeros(4 * 65536)
        ar = ctypes.c_double()
        n = lib.overlay_host(xa.ctypes.data, ra.ctypes.data, len(ra) - 1, pa.ctypes.data, len(pa) - 1, xb.ctypes.data,
                             rb.ctypes.data, len(rb) - 1, pb.ctypes.data, len(pb) - 1, need, out.ctypes.data, 65536,
                             ctypes.byref(ar))
        assert n >= 0
        return out[:4 * n].reshape(-1, 4).tolist(), ar.value
    return run


@pytest.fixture(scope="module")
def host_stitch(tmp_path_factory):
    """isect_geom.cpp: edges -> WKB (None when the edges do not close)"""
    lib = _build_so(tmp_path_factory, "st", ["tests/native/stitch_host.cpp", "mosaic_amd/csrc/isect_geom.cpp"])
    lib.stitch_host.restype = ctypes.c_long
    lib.stitch_host.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_double, ctypes.c_void_p, ctypes.c_long,
                                ctypes.c_void_p]

    def run(edges, snap):
        e = np.ascontiguousarray(np.array(edges, float).reshape(-1, 4))
        buf = np.zeros(1 << 22, np.uint8)
        ar = ctypes.c_double()
        n = lib.stitch_host(e.ctypes.data, len(e), snap, buf.ctypes.data, len(buf), ctypes.byref(ar))
        return (bytes(buf[:n]) if n >= 0 else None), ar.value
    return run


def h3_snap(res):
    """isect_geom's node tolerance for H3 (mosaic_hip.hip stitch_snap): since the chips are the
    reference's planar clips, adjacent cells' chips meet exactly and the tolerance is the overlay's
    own node scale, 180 x 2^-40 degrees at every resolution"""
    return 180.0 * 2.0 ** -40


def _sq(x0, y0, s):
    return [(x0, y0), (x0 + s, y0), (x0 + s, y0 + s), (x0, y0 + s), (x0, y0)]


def test_overlay_unit_cases(host_overlay):
    """one cell's overlay against the exact set: squares, holes, L-shapes, shared edges, overlapping
    parts on one side (the union before the intersection), identical and ulp-shifted edges"""
    ell = [(0, 0), (3, 0), (3, 1), (1, 1), (1, 3), (0, 3), (0, 0)]
    sq = _sq
    cases = [([[sq(0, 0, 2)]], [[sq(1, 1, 2)]]), ([[sq(0, 0, 2)]], [[sq(2, 0, 2)]]),
             ([[sq(0, 0, 4), sq(1, 1, 1)]], [[sq(0, 0, 4)]]), ([[ell]], [[sq(0.5, 0.5, 2)]]), ([[ell]], [[ell[::-1]]]),
             ([[sq(0, 0, 1)], [sq(2, 0, 1)]], [[sq(0.5, 0, 2)]]), ([[sq(0, 0, 2)], [sq(1, 1, 2)]], [[sq(0.5, 0.5, 2)]]),
             ([[sq(0, 0, 2)], [sq(1, 0, 2)]], [[sq(0, 0, 3)], [sq(2, -1, 1)]]), ([[sq(0, 0, 2)]], [[sq(0, 0, 2)]]),
             ([[sq(0, 0, 2)], [sq(0, 0, 2)]], [[sq(1, 0, 2)]]), ([[sq(0, 0, 1)], [sq(1, 0, 1)]], [[sq(0, 0, 2)]])]
    for a, b in cases:
        e, ar = host_overlay(a, b, 3)
        d, ax, aw = exact.symdiff_area(e, [(a, b)])
        assert d < 1e-12 and abs(ar - ax) < 1e-12, (a, b, d, ar, ax)
    e, ar = host_overlay([[sq(0, 0, 2)], [sq(1, 1, 2)]], [], 1)  # B core: the union of A
    assert abs(ar - 7) < 1e-12 and exact.symdiff_area(e, [([[sq(0, 0, 2)], [sq(1, 1, 2)]], None)])[0] < 1e-12
    a = [[sq(-74.0, 40.7, 0.01)]]
    b = [[[(x + math.ulp(x), y) for x, y in sq(-74.0, 40.7, 0.01)]]]
    e, ar = host_overlay(a, b, 3)
    assert len(e) == 4 and exact.symdiff_area(e, [(a, b)])[0] < 1e-18


def _units(li, ri):
    """(left key, right key) -> [(cell, left chips, right chips)] of the chip join"""
    by_cell = {}
    for (k, cell), v in ri.items():
        by_cell.setdefault(cell, []).append((k, v))
    groups = {}
    for (lk, cell), lv in li.items():
        for rk, rv in by_cell.get(cell, []):
            groups.setdefault((lk, rk), []).append((cell, lv, rv))
    return groups


def _increments(lv, rv, cell, bng_res=None):
    """the reference's increments of one cell as an overlay unit (A parts | None, B parts | None, need)"""
    acore, bcore = any(c for c, _ in lv), any(c for c, _ in rv)
    A = [p for _, ps in lv for p in ps]
    B = [p for _, ps in rv for p in ps]
    if acore and bcore:
        if bng_res is None:
            ring = [(math.degrees(lo), math.degrees(la)) for la, lo in oracle.h3_to_geo_boundary(cell)]
            return [[ring + ring[:1]]], None, 1
        return [read_wkb(oracle.bng_cell_wkb(cell))[1][0]], None, 1
    if acore:
        return None, B, 2
    if bcore:
        return A, None, 1
    return A, B, 3


def _wkb_edges(w):
    """edges of the engine's WKB, interior on the left (its shells are clockwise)"""
    _, parts = read_wkb(w)
    out = []
    for p in parts:
        for r in p:
            out += [(r[i + 1][0], r[i + 1][1], r[i][0], r[i][1]) for i in range(len(r) - 1)]
    return parts, out


def _shares_edge(parts):
    """two polygons of a MultiPolygon with a common edge (not dissolved)"""
    def keys(p):
        return {tuple(sorted([(round(r[i][0], 9), round(r[i][1], 9)), (round(r[i + 1][0], 9), round(r[i + 1][1], 9))]))
                for r in p for i in range(len(r) - 1)}
    ks = [keys(p) for p in parts]
    return any(ks[i] & ks[j] for i in range(len(ks)) for j in range(i + 1, len(ks)))


def _check_group(units, wkb, area, snap):
    """the group's WKB against the exact union of its cells' increments.  Chips of adjacent cells
    meet along their shared side exactly (the reference's planar clips against cell polygons that
    share their vertices), up to the overlay's node scale `snap`: the symmetric difference is bounded
    by snap x the polygons' perimeter, and is ~0 for a group within one cell.  The area (the sum of
    the cells' pieces) is X's within the same bound."""
    us = [(a, b) for a, b, _ in units]
    parts, e = _wkb_edges(wkb)
    d, ax, aw = exact.symdiff_area(e, us)
    per = sum(math.hypot(x1 - x0, y1 - y0) for x0, y0, x1, y1 in e)
    # (the overlay's node tolerance, 2^-40 of the coordinates, moves vertices by <= 7e-11 degrees:
    # 1e-13 of absolute slack; the float slab checker's own precision: 1e-8 relative)
    bound = (snap * per if len(units) > 1 else 0.0) + 1e-9 * ax + 1e-13
    assert d <= bound, (d, bound, ax)
    # (the area sums the cells' pieces, so a sliver where two cells' chips overlap counts twice there)
    assert abs(area - ax) <= bound + 1e-8 * ax, (area, ax)
    assert not _shares_edge(parts)
    return len(parts)


@pytest.mark.parametrize("res", [8, 9])
def test_overlay_stitch_nyc_groups(host_overlay, host_stitch, res):
    """zones against a translated copy: per cell the overlay (host build of the device code), across
    cells the stitching; every group's polygons equal the exact union (symmetric difference ~0) and
    pieces of adjacent cells are dissolved (no polygon shares an edge with another)"""
    zones = PolygonSet.load("nyc_taxi_zones").subset([3, 7, 9, 11, 15, 23, 24, 40])
    moved = _translated(zones)
    groups = _units(_chip_index(tessellate("H3", zones, res)), _chip_index(tessellate("H3", moved, res)))
    assert len(groups) >= 10
    multi_cell = 0
    for g, units in sorted(groups.items()):
        edges, area, us = [], 0.0, []
        for cell, lv, rv in units:
            a, b, need = _increments(lv, rv, cell)
            e, ar = host_overlay(a or [], b or [], need)
            edges += e
            area += ar
            us.append((a, b, need))
        w, _ = host_stitch(edges, h3_snap(res))
        assert w is not None, g
        _check_group(us, w, area, h3_snap(res))
        multi_cell += len(units) > 1
    assert multi_cell >= 5


def _overlapping_left(zones, k, res):
    """a chip set whose key 0 holds zone k and a copy shifted by a fraction of a cell: overlapping
    chips of one key in one cell (the case the union exists for)"""
    a = zones.subset([k])
    xy = a.xy.copy()
    xy[:, 0] += 0.0013
    xy[:, 1] += 0.0007
    b = PolygonSet(xy, a.ring_offsets, a.part_rings, a.geom_parts)
    ca, cb = tessellate("H3", a, res), tessellate("H3", b, res)
    out = {}
    for c in (ca, cb):
        offs, data = c["wkb"]
        out.setdefault("is_core", []).extend(c["is_core"].tolist())
        out.setdefault("index_id", []).extend(c["index_id"].tolist())
        out.setdefault("wkb", []).extend(bytes(data[offs[i]:offs[i + 1]]) for i in range(len(offs) - 1))
    out["polygon_key"] = [0] * len(out["index_id"])
    return out


def _index_rows(rows):
    d = {}
    for core, cid, w, k in zip(rows["is_core"], rows["index_id"], rows["wkb"], rows["polygon_key"]):
        d.setdefault((int(k), int(cid)), []).append((int(core), read_wkb(w)[1] if len(w) else []))
    return d


def test_overlay_overlapping_chips(host_overlay, host_stitch):
    """a key whose chips overlap within cells (two overlapping polygons under one key) against a
    translated zone: the union of the overlapping pieces, exact, dissolved"""
    zones = PolygonSet.load("nyc_taxi_zones")
    res = 9
    left = _overlapping_left(zones, 3, res)
    moved = _translated(zones.subset([3]))
    groups = _units(_index_rows(left), _chip_index(tessellate("H3", moved, res)))
    (g, units), = groups.items()
    assert sum(len(lv) > 1 for _, lv, _ in units) >= 5
    edges, area, us = [], 0.0, []
    for cell, lv, rv in units:
        a, b, need = _increments(lv, rv, cell)
        e, ar = host_overlay(a or [], b or [], need)
        edges += e
        area += ar
        us.append((a, b, need))
    w, _ = host_stitch(edges, h3_snap(res))
    assert w is not None
    _check_group(us, w, area, h3_snap(res))


def _table(ctx, rows, res, n):
    return ctx.chip_table(rows["is_core"], rows["index_id"], list(rows["wkb"]), rows["polygon_key"], res, n_polygons=n)


def _rows(chips):
    return dict(is_core=chips["is_core"], index_id=chips["index_id"], wkb=_wkb_list(chips), polygon_key=chips["polygon_key"])


@pytest.mark.gpu
@pytest.mark.parametrize("res", [5, 7, 8, 9, 10])
def test_gpu_intersection_agg_geometry_nyc(h3ctx, res):
    """all 263 NYC zones against a translated copy (res 7 the reference's test resolution,
    res 5 a coarse one where the stitch tolerance must stay bounded): no group refused; the area API and
    the geometry API agree; sampled groups' polygons equal the exact union of their cells' increments
    (symmetric difference ~0), dissolved across cells"""
    zones = PolygonSet.load("nyc_taxi_zones")
    moved = _translated(zones)
    lc, rc = tessellate("H3", zones, res, ctx=h3ctx), tessellate("H3", moved, res, ctx=h3ctx)
    left, right = _table(h3ctx, _rows(lc), res, len(zones)), _table(h3ctx, _rows(rc), res, len(zones))
    lk, rk, area, st, wkb = h3ctx.st_intersection_aggregate(left, right)
    lk2, rk2, area2, st2 = h3ctx.st_intersection_aggregate_area(left, right)
    assert len(lk) > 500 and np.array_equal(st, st2)
    if res >= 7:
        assert not st.any()
    else:
        # coarse cells hold whole zones: a unit past the overlay's per-unit edge limit, or a stitch
        # whose area disagrees with the units', is refused (status 1, area NaN), never returned
        # distorted; the rest are exact
        assert st.mean() < 0.05 and np.isnan(area[st != 0]).all(), (int(st.sum()), len(st))
    assert np.array_equal(lk, lk2) and np.array_equal(rk, rk2)
    assert np.array_equal(area.view(np.uint64), area2.view(np.uint64))  # (one unit pipeline)
    groups = _units(_chip_index(lc), _chip_index(rc))
    assert set(zip(lk.tolist(), rk.tolist())) == set(groups)
    idx = {(int(a), int(b)): i for i, (a, b) in enumerate(zip(lk, rk))}
    rng = np.random.default_rng(res)
    sample = [k for k in sorted(groups) if len(groups[k]) > 1 and len(groups[k]) <= 40 and st[idx[k]] == 0]
    for g in [sample[i] for i in rng.choice(len(sample), min(12, len(sample)), replace=False)]:
        us = [_increments(lv, rv, cell) for cell, lv, rv in groups[g]]
        _check_group(us, wkb[idx[g]], area[idx[g]], h3_snap(res))
    left.close()
    right.close()


@pytest.mark.gpu
def test_gpu_intersection_agg_overlapping_chips(h3ctx):
    """the overlapping chip set on the GPU: no refusal, geometry exact and dissolved, the area API
    equal to the geometry API"""
    zones = PolygonSet.load("nyc_taxi_zones")
    res = 9
    rows = _overlapping_left(zones, 3, res)
    moved = _translated(zones.subset([3]))
    rc = tessellate("H3", moved, res)
    left, right = _table(h3ctx, rows, res, 1), _table(h3ctx, _rows(rc), res, 1)
    lk, rk, area, st, wkb = h3ctx.st_intersection_aggregate(left, right)
    _, _, area2, st2 = h3ctx.st_intersection_aggregate_area(left, right)
    assert list(st) == [0] and list(st2) == [0] and abs(area[0] - area2[0]) <= 1e-12 * area[0]
    (g, units), = _units(_index_rows(rows), _chip_index(rc)).items()
    _check_group([_increments(lv, rv, cell) for cell, lv, rv in units], wkb[0], area[0], h3_snap(res))
    left.close()
    right.close()


def _bng_zones(n=4, size=300.0):
    """London postcode zones (EPSG:27700) scaled about their vertex mean to ~`size` metres across:
    small enough for the reference's BNG resolutions 5 (10 m) and 6 (1 m)"""
    z = PolygonSet.load("london_postcodes_bng")
    xy = []
    ro, pr, gp = [0], [0], [0]
    for g in range(n):
        parts = z.parts(g * 7)
        allv = np.array([v for p in parts for r in p for v in r])
        c = allv.mean(axis=0)
        f = size / max(np.ptp(allv[:, 0]), np.ptp(allv[:, 1]))
        for p in parts:
            for r in p:
                xy += [tuple(c + (np.asarray(v) - c) * f + np.array([450.0 * g, 0.0])) for v in r]
                ro.append(len(xy))
            pr.append(len(ro) - 1)
        gp.append(len(pr) - 1)
    return PolygonSet(np.array(xy), ro, pr, gp)


@pytest.mark.gpu
@pytest.mark.parametrize("res", [5, 6])
def test_gpu_intersection_agg_bng(res):
    """st_intersection_aggregate on BNG at the reference's resolutions (intersectionBehaviour
    on BNG res 5, selfIntersectionBehaviour on BNG res 6, ST_IntersectionTest.scala:27-32): zones
    against a translated copy and against themselves -- no group refused, the area API equal to the
    geometry API, sampled groups' polygons equal to the exact union of their cells' increments
    (symmetric difference within the node scale), dissolved across cells."""
    from mosaic_amd import MosaicContext

    ctx = MosaicContext.build("BNG", "JTS")
    zones = _bng_zones(size={5: 300.0, 6: 30.0}[res])  # (~900 cells a zone)
    snap = 1e6 * 2.0 ** -40
    for other in (_translated(zones), zones):
        lc, rc = tessellate("BNG", zones, res, ctx=ctx), tessellate("BNG", other, res, ctx=ctx)
        left, right = _table(ctx, _rows(lc), res, len(zones)), _table(ctx, _rows(rc), res, len(other))
        lk, rk, area, st, wkb = ctx.st_intersection_aggregate(left, right)
        lk2, rk2, area2, st2 = ctx.st_intersection_aggregate_area(left, right)
        assert len(lk) >= len(zones) and not st.any() and not st2.any()
        assert np.array_equal(lk, lk2) and np.array_equal(rk, rk2)
        assert np.array_equal(area.view(np.uint64), area2.view(np.uint64))
        groups = _units(_chip_index(lc), _chip_index(rc))
        assert set(zip(lk.tolist(), rk.tolist())) == set(groups)
        idx = {(int(a), int(b)): i for i, (a, b) in enumerate(zip(lk, rk))}
        for g in sorted(groups)[:3]:
            us = [_increments(lv, rv, cell, bng_res=res) for cell, lv, rv in groups[g]]
            _check_group(us, wkb[idx[g]], area[idx[g]], snap)
        left.close()
        right.close()
    ctx.close()
