"""st_intersection_aggregate (§8(f) row 4) as its area: st_area of the union the reference's
ST_IntersectionAggregate.update / merge builds per (left id, right id) group of the chip join
(expressions/geometry/ST_IntersectionAggregate.scala) -- the quantity its tests check within 1e-8
(ST_IntersectionBehaviors.scala:22-71 intersectionBehaviour, :73-135 intersectionAggBehaviour).

The engine (mosaic_intersection_aggregate, isect_area.h) sums per cell: the cell for a (core, core)
pair, the other chip for one core side, and area(left n right) otherwise as the signed sum of the
overlaps of the two chips' edge triangles fanned from a common origin.
The checker (oracle/exact.py intersection_area) is a different algorithm in exact rationals:
vertical slabs between all vertex and crossing abscissae, where the section length is linear and the
midpoint rule exact.  Pins: intersectionAggBehaviour's chip rows (H3 cells with vertex 2 dropped)
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


@pytest.fixture(scope="module")
def host_area(tmp_path_factory):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = tmp_path_factory.mktemp("ia") / "libia.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-shared", "-fPIC", "-I",
                    os.path.join(root, "mosaic_amd", "csrc"), "-o", str(so),
                    os.path.join(root, "tests", "native", "isect_area_host.cpp")], check=True)
    lib = ctypes.CDLL(str(so))
    lib.isect_area_host.restype = ctypes.c_double
    vp, i = ctypes.c_void_p, ctypes.c_int
    lib.isect_area_host.argtypes = [vp, vp, i, vp, i, vp, vp, i, vp, i]

    def run(a, b):
        xa, ra, pa = _parts_arrays(a)
        xb, rb, pb = _parts_arrays(b)
        return lib.isect_area_host(xa.ctypes.data, ra.ctypes.data, len(ra) - 1, pa.ctypes.data, len(pa) - 1,
                                   xb.ctypes.data, rb.ctypes.data, len(rb) - 1, pb.ctypes.data, len(pb) - 1)
    return run


def test_kernel_code_on_host_matches_exact(host_area):
    """the device area code compiled for the host against the exact slab oracle: squares, holes,
    L-shapes, shared edges, opposite orientations, and tessellated chip pairs of valid NYC zones
    against a translated copy"""
    sq = lambda x0, y0, s: [(x0, y0), (x0 + s, y0), (x0 + s, y0 + s), (x0, y0 + s), (x0, y0)]
    ell = [(0, 0), (3, 0), (3, 1), (1, 1), (1, 3), (0, 3), (0, 0)]
    cases = [([[sq(0, 0, 2)]], [[sq(1, 1, 2)]]), ([[sq(0, 0, 2)]], [[sq(2, 0, 2)]]),
             ([[sq(0, 0, 4), sq(1, 1, 1)]], [[sq(0, 0, 4)]]), ([[ell]], [[sq(0.5, 0.5, 2)]]),
             ([[ell]], [[ell[::-1]]]), ([[sq(0, 0, 1)], [sq(2, 0, 1)]], [[sq(0.5, 0, 2)]])]
    for a, b in cases:
        assert abs(host_area(a, b) - float(exact.intersection_area(a, b))) < 1e-12
    zones = PolygonSet.load("nyc_taxi_zones").subset([3, 7, 9, 11])
    moved = _translated(zones)
    li, ri = _chip_index(tessellate("H3", zones, 8)), _chip_index(tessellate("H3", moved, 8))
    n = 0
    for (k, cell), lv in li.items():
        rv = ri.get((k, cell))
        if not rv or lv[0][0] or rv[0][0]:
            continue
        got, want = host_area(lv[0][1], rv[0][1]), float(exact.intersection_area(lv[0][1], rv[0][1]))
        assert abs(got - want) <= 1e-13 + 1e-9 * want, (cell, got, want)
        n += 1
    assert n >= 5


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
    """{(left key, right key): (area, supported)} with the engine's per-cell rules, areas exact"""
    li, ri = _chip_index(left), _chip_index(right)
    by_cell_r = {}
    for (k, cell), v in ri.items():
        by_cell_r.setdefault(cell, []).append((k, v))
    out = {}
    for (lk, cell), lv in li.items():
        for rk, rv in by_cell_r.get(cell, []):
            pairs = [(a, b) for a in lv for b in rv]
            area, ok = out.get((lk, rk), (0, True))
            cc = [a for a, b in pairs if a[0] and b[0]]
            if cc:
                area += exact.polygon_area(cc[0][1])
            elif len(pairs) > 1:
                ok = False
            else:
                a, b = pairs[0]
                if a[0]:
                    area += exact.polygon_area(b[1])
                elif b[0]:
                    area += exact.polygon_area(a[1])
                else:
                    area += exact.intersection_area(a[1], b[1])
            out[(lk, rk)] = (area, ok)
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
    # a cell holding two border-chip pairs of one group and no (core, core) pair is refused
    left2 = h3ctx.chip_table([0, 0], [ids[0], ids[0]], [rows_wkb[2], rows_wkb[2]], [0, 0], res, n_polygons=1)
    right2 = h3ctx.chip_table([0], [ids[0]], [rows_wkb[2]], [0], res, n_polygons=1)
    assert list(h3ctx.st_intersection_aggregate_area(left2, right2)[3]) == [1]
    for t in (left, right, left2, right2):
        t.close()


@pytest.mark.gpu
def test_gpu_intersection_agg_nyc_zones(h3ctx):
    """intersectionBehaviour on NYC zones at res 8: engine == exact per-cell aggregate for every
    group; aggregate == the flat intersection area of the original polygons (the reference's
    invariant, 1e-8) for the groups of a polygon with its own translated copy"""
    # valid single-polygon zones (no self-crossing ring: on invalid rings JTS's union and the
    # winding-number area of the engine are not defined the same way)
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
    assert len(want) > 0
    for a, b, v, s in zip(lk, rk, area, st):
        w, ok = want[(int(a), int(b))]
        assert bool(s) == (not ok)
        if ok:
            assert abs(v - float(w)) <= 1e-12 + 1e-9 * abs(float(w)), (a, b, v, float(w))
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
