"""TEST INFRASTRUCTURE ONLY: ctypes bindings to the CPU oracle (oracle/liboracle.so).

Only tests/, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
package, and only as the checker (or the timed CPU baseline).  The product
(``mosaic_amd`` / ``libmosaic_hip.so``) never imports it.  See ``oracle/oracle.h`` for the
reference file:line each restated function follows and how each is pinned.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

GRID_H3 = 0
GRID_BNG = 1


def build():
    """Compile liboracle.so with gcc (oracle/Makefile)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        i64, f64, i32, vp = ctypes.c_int64, ctypes.c_double, ctypes.c_int, ctypes.c_void_p
        L.oracle_h3_geo_to_h3.restype = i64
        L.oracle_h3_geo_to_h3.argtypes = [f64, f64, i32]
        L.oracle_to_radians.restype = f64
        L.oracle_to_radians.argtypes = [f64, i32]
        L.oracle_h3_point_to_index.restype = None
        L.oracle_h3_point_to_index.argtypes = [vp, vp, i64, i32, i32, vp]
        L.oracle_libm_eval.restype = None
        L.oracle_libm_eval.argtypes = [i32, vp, vp, i64, vp]
        L.oracle_h3_debug.restype = None
        L.oracle_h3_debug.argtypes = [f64, f64, i32, vp, vp, vp, vp]
        L.oracle_bng_point_to_index.restype = i64
        L.oracle_bng_point_to_index.argtypes = [f64, f64, i32, ctypes.POINTER(ctypes.c_int)]
        L.oracle_bng_point_to_index_batch.restype = None
        L.oracle_bng_point_to_index_batch.argtypes = [vp, vp, i64, i32, vp, vp]
        L.oracle_bng_format.restype = i32
        L.oracle_bng_format.argtypes = [i64, ctypes.c_char_p, i32]
        L.oracle_bng_parse.restype = i32
        L.oracle_bng_parse.argtypes = [ctypes.c_char_p, i32, ctypes.POINTER(i64)]
        L.oracle_orientation_index.restype = i32
        L.oracle_orientation_index.argtypes = [f64] * 6
        L.oracle_wkb_contains.restype = i32
        L.oracle_wkb_contains.argtypes = [ctypes.c_char_p, i64, f64, f64]
        L.oracle_pip_join.restype = i64
        L.oracle_pip_join.argtypes = [vp, i32, i32, i32, vp, vp, i64, vp, i64, vp, vp, i64, i32]
        L.oracle_brute_force_count.restype = i64
        L.oracle_brute_force_count.argtypes = [vp, vp, vp, i64, vp, i64]
        L.oracle_segments_intersect.restype = i32
        L.oracle_segments_intersect.argtypes = [f64] * 8
        L.oracle_wkb_intersects.restype = i32
        L.oracle_wkb_intersects.argtypes = [ctypes.c_char_p, i64, ctypes.c_char_p, i64]
        for fn in ("oracle_bng_kloop", "oracle_bng_kring"):
            getattr(L, fn).restype = i32
            getattr(L, fn).argtypes = [i64, i32, vp]
        L.oracle_bng_is_valid.restype = i32
        L.oracle_bng_is_valid.argtypes = [i64]
        L.oracle_bng_cell_origin.restype = i32
        L.oracle_bng_cell_origin.argtypes = [i64, vp]
        L.oracle_h3_to_geo.restype = None
        L.oracle_h3_to_geo.argtypes = [i64, vp, vp]
        L.oracle_h3_kring_set.restype = i64
        L.oracle_h3_kring_set.argtypes = [i64, i32, vp, vp, i64]
        L.oracle_h3_to_geo_boundary.restype = i32
        L.oracle_h3_to_geo_boundary.argtypes = [i64, vp]
        L.oracle_h3_is_pentagon.restype = i32
        L.oracle_h3_is_pentagon.argtypes = [i64]
        L.oracle_h3_polyfill.restype = i64
        L.oracle_h3_polyfill.argtypes = [vp, vp, vp, i32, i32, vp, i64, ctypes.POINTER(ctypes.c_int)]
        L.oracle_h3_ring1.restype = i32
        L.oracle_h3_ring1.argtypes = [i64, vp]
        L.oracle_jts_centroid.restype = i32
        L.oracle_jts_centroid.argtypes = [vp, vp, vp]
        L.oracle_h3_buffer_radius.restype = f64
        L.oracle_h3_buffer_radius.argtypes = [vp, i32, i32]
        L.oracle_bng_polyfill.restype = i64
        L.oracle_bng_polyfill.argtypes = [vp, i32, vp, i64]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def h3_point_to_index(lon, lat, res, jdk=8):
    """H3IndexSystem.pointToIndex(lon, lat, res) for arrays (degrees)."""
    lon = np.ascontiguousarray(lon, dtype=np.float64)
    lat = np.ascontiguousarray(lat, dtype=np.float64)
    out = np.empty(lon.shape[0], dtype=np.int64)
    lib().oracle_h3_point_to_index(_ptr(lon), _ptr(lat), lon.shape[0], res, jdk, _ptr(out))
    return out


def h3_to_geo(cell):
    """h3ToGeo: the cell centre (lat, lng) in radians (H3 C v3.7 _faceIjkToGeo)."""
    lat = np.zeros(1)
    lon = np.zeros(1)
    lib().oracle_h3_to_geo(int(cell), _ptr(lat), _ptr(lon))
    return float(lat[0]), float(lon[0])


def h3_kring_set(cell, k):
    """kRing(cell, k) as {cell: ring distance}, found on the sphere (oracle/h3.c)."""
    cap = 1 + 3 * k * (k + 1) + 64
    out = np.zeros(cap, np.int64)
    dist = np.zeros(cap, np.int32)
    n = lib().oracle_h3_kring_set(int(cell), k, _ptr(out), _ptr(dist), cap)
    assert n >= 0
    return dict(zip(out[:n].tolist(), dist[:n].tolist()))


def h3_to_geo_boundary(cell):
    """h3ToGeoBoundary: [(lat, lng)] radians, 5..10 vertices (H3 C v3.7 _faceIjkToGeoBoundary)."""
    out = np.zeros(20)
    n = lib().oracle_h3_to_geo_boundary(int(cell), _ptr(out))
    return [(float(out[2 * i]), float(out[2 * i + 1])) for i in range(n)]


def h3_is_pentagon(cell):
    return bool(lib().oracle_h3_is_pentagon(int(cell)))


def h3_geo_to_h3(lat_rad, lng_rad, res):
    return lib().oracle_h3_geo_to_h3(lat_rad, lng_rad, res)


def to_radians(deg, jdk=8):
    return lib().oracle_to_radians(deg, jdk)


def libm_eval(fn, a, b=None):
    """The host glibc functions H3 C calls: fn 0 sin, 1 cos (sincos), 2 tan, 3 acos, 4 atan2(a, b)."""
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(a if b is None else b, dtype=np.float64)
    out = np.empty_like(a)
    lib().oracle_libm_eval(fn, _ptr(a), _ptr(b), a.shape[0], _ptr(out))
    return out


def h3_debug(lat_rad, lng_rad, res):
    face = np.zeros(1, np.int32)
    x = np.zeros(1)
    y = np.zeros(1)
    ijk = np.zeros(3, np.int32)
    lib().oracle_h3_debug(lat_rad, lng_rad, res, _ptr(face), _ptr(x), _ptr(y), _ptr(ijk))
    return int(face[0]), float(x[0]), float(y[0]), tuple(int(v) for v in ijk)


def bng_point_to_index(e, n, res):
    """BNGIndexSystem.pointToIndex; raises ValueError for NaN like the reference's IllegalStateException."""
    err = ctypes.c_int(0)
    v = lib().oracle_bng_point_to_index(e, n, res, ctypes.byref(err))
    if err.value == 1:
        raise ValueError("NaN coordinates are not supported.")
    if err.value == 2:
        raise ValueError(f"BNG resolution not supported; found {res}")
    return v


def bng_point_to_index_batch(e, n, res):
    e = np.ascontiguousarray(e, dtype=np.float64)
    n = np.ascontiguousarray(n, dtype=np.float64)
    out = np.empty(e.shape[0], dtype=np.int64)
    err = np.empty(e.shape[0], dtype=np.uint8)
    lib().oracle_bng_point_to_index_batch(_ptr(e), _ptr(n), e.shape[0], res, _ptr(out), _ptr(err))
    return out, err


def bng_parse(text):
    """BNGIndexSystem.parse; None where the reference throws."""
    b = text.encode()
    out = ctypes.c_int64(0)
    return out.value if lib().oracle_bng_parse(b, len(b), ctypes.byref(out)) else None


def bng_format(cell_id):
    buf = ctypes.create_string_buffer(64)
    n = lib().oracle_bng_format(cell_id, buf, 64)
    if n < 0:
        raise ValueError(f"cannot format {cell_id}")
    return buf.value.decode()


def orientation_index(p1, p2, q):
    return lib().oracle_orientation_index(p1[0], p1[1], p2[0], p2[1], q[0], q[1])


def wkb_contains(wkb: bytes, x, y):
    r = lib().oracle_wkb_contains(wkb, len(wkb), x, y)
    if r < 0:
        raise ValueError("unparseable WKB")
    return bool(r)


def bng_kloop(cell, k):
    out = np.zeros(max(8 * k, 1), np.int64)
    m = lib().oracle_bng_kloop(int(cell), int(k), _ptr(out))
    if m < 0:
        raise ValueError("undecodable BNG id")
    return out[:m]


def bng_kring(cell, k):
    out = np.zeros(1 + 4 * k * (k + 1), np.int64)
    m = lib().oracle_bng_kring(int(cell), int(k), _ptr(out))
    if m < 0:
        raise ValueError("undecodable BNG id")
    return out[:m]


def bng_is_valid(cell):
    return bool(lib().oracle_bng_is_valid(int(cell)))


def bng_cell_wkb(cell):
    """grid_boundaryaswkb for a BNG cell: BNGIndexSystem.indexToGeometry's square (x, y), (x + e, y),
    (x + e, y + e), (x, y + e), (x, y) as JTS WKBWriter's default big-endian 2D Polygon."""
    import struct

    o = np.zeros(4, np.int32)
    if not lib().oracle_bng_cell_origin(int(cell), _ptr(o)):
        raise ValueError("undecodable BNG id")
    _, e, x, y = (int(v) for v in o)
    x1 = int(np.int32(np.uint32((x + e) & 0xffffffff)))
    y1 = int(np.int32(np.uint32((y + e) & 0xffffffff)))
    pts = [(x, y), (x1, y), (x1, y1), (x, y1), (x, y)]
    return struct.pack(">BIII", 0, 3, 1, 5) + b"".join(struct.pack(">dd", float(a), float(b)) for a, b in pts)


def segments_intersect(p1, p2, q1, q2):
    return bool(lib().oracle_segments_intersect(p1[0], p1[1], p2[0], p2[1], q1[0], q1[1], q2[0], q2[1]))


def wkb_intersects(wa: bytes, wb: bytes):
    r = lib().oracle_wkb_intersects(wa, len(wa), wb, len(wb))
    if r < 0:
        raise ValueError("unparseable WKB")
    return bool(r)


def intersects_aggregate(left, right):
    """Reference semantics of left.join(right, index_id).groupBy(left key, right key)
    .agg(st_intersects_aggregate) (ST_IntersectsAggregate.scala:28-39) over two chip dicts
    (index_id, is_core, polygon_key, wkb=(offsets, data)): {(left key, right key): flag}."""
    from collections import defaultdict

    by_cell = defaultdict(list)
    lo, ld = left["wkb"]
    for i, c in enumerate(left["index_id"]):
        by_cell[int(c)].append(i)
    ro, rd = right["wkb"]
    out = {}
    for j, c in enumerate(right["index_id"]):
        for i in by_cell.get(int(c), ()):
            g = (int(left["polygon_key"][i]), int(right["polygon_key"][j]))
            if out.get(g):
                continue
            hit = bool(left["is_core"][i]) or bool(right["is_core"][j])
            if not hit:
                hit = wkb_intersects(bytes(ld[lo[i]:lo[i + 1]]), bytes(rd[ro[j]:ro[j + 1]]))
            out[g] = out.get(g, False) or hit
    return out


class _Chips(ctypes.Structure):
    _fields_ = [("n_chips", ctypes.c_int64), ("index_id", ctypes.c_void_p), ("is_core", ctypes.c_void_p),
                ("polygon_key", ctypes.c_void_p), ("wkb_offsets", ctypes.c_void_p), ("wkb", ctypes.c_void_p)]


def brute_force_count(polygons, x, y):
    """Brute-force st_contains counts of a PolygonSet (one key per geometry)."""
    wkbs = [polygons.wkb(g) for g in range(len(polygons))]
    lens = np.array([len(w) for w in wkbs], np.int64)
    offs = np.zeros(len(wkbs) + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    data = np.frombuffer(b"".join(wkbs), np.uint8).copy()
    keys = np.arange(len(wkbs), dtype=np.int32)
    core = np.zeros(len(wkbs), np.uint8)
    ids = np.zeros(len(wkbs), np.int64)
    c = _Chips(len(wkbs), _ptr(ids).value, _ptr(core).value, _ptr(keys).value, _ptr(offs).value, _ptr(data).value)
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    counts = np.zeros(max(len(wkbs), 1), np.int64)
    total = lib().oracle_brute_force_count(ctypes.byref(c), _ptr(x), _ptr(y), len(x), _ptr(counts), len(wkbs))
    return counts[:len(wkbs)], total


def pip_join(chips, grid, res, x, y, n_polygons, jdk=8, pairs=False, threads=1):
    """Chip join oracle.  ``chips`` is a dict of numpy arrays: index_id (int64), is_core (uint8),
    polygon_key (int32), wkb_offsets (int64, n+1), wkb (uint8).  Returns (counts, n_pairs[, rows, keys])."""
    keep = {k: np.ascontiguousarray(v) for k, v in chips.items()}
    c = _Chips(len(keep["index_id"]), _ptr(keep["index_id"]).value, _ptr(keep["is_core"]).value,
               _ptr(keep["polygon_key"]).value, _ptr(keep["wkb_offsets"]).value,
               _ptr(keep["wkb"]).value if len(keep["wkb"]) else None)
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    counts = np.zeros(max(n_polygons, 1), dtype=np.int64)
    if pairs:
        # first pass to size the output
        total = lib().oracle_pip_join(ctypes.byref(c), grid, res, jdk, _ptr(x), _ptr(y), len(x), _ptr(counts),
                                      n_polygons, None, None, 0, 1)
        rows = np.empty(max(total, 1), np.int64)
        keys = np.empty(max(total, 1), np.int32)
        counts[:] = 0
        lib().oracle_pip_join(ctypes.byref(c), grid, res, jdk, _ptr(x), _ptr(y), len(x), _ptr(counts), n_polygons,
                              _ptr(rows), _ptr(keys), total, 1)
        return counts[:n_polygons], total, rows[:total], keys[:total]
    total = lib().oracle_pip_join(ctypes.byref(c), grid, res, jdk, _ptr(x), _ptr(y), len(x), _ptr(counts),
                                  n_polygons, None, None, 0, threads)
    return counts[:n_polygons], total


class _Geom(ctypes.Structure):
    _fields_ = [("xy", ctypes.c_void_p), ("ring_offsets", ctypes.c_void_p), ("part_rings", ctypes.c_void_p),
                ("n_parts", ctypes.c_int64)]


def _geom_arrays(parts):
    """parts: list of parts, each a list of rings of (x, y) -> (xy, ring_offsets, part_rings)."""
    rings = [np.asarray(r, np.float64).reshape(-1, 2) for part in parts for r in part]
    xy = np.ascontiguousarray(np.concatenate(rings) if rings else np.zeros((0, 2)), np.float64)
    ro = np.zeros(len(rings) + 1, np.int64)
    np.cumsum([len(r) for r in rings], out=ro[1:])
    pr = np.zeros(len(parts) + 1, np.int64)
    np.cumsum([len(p) for p in parts], out=pr[1:])
    return xy, ro, pr


def h3_polyfill_part(rings, res, jdk=8, cap=1 << 22):
    """H3 polyfill of one polygon part (rings of (lon, lat) degrees, shell first): (cells in H3's
    output order, collision_free)."""
    lat = np.ascontiguousarray(np.concatenate([[to_radians(v[1], jdk) for v in r] for r in rings]), np.float64)
    lon = np.ascontiguousarray(np.concatenate([[to_radians(v[0], jdk) for v in r] for r in rings]), np.float64)
    ro = np.zeros(len(rings) + 1, np.int64)
    np.cumsum([len(r) for r in rings], out=ro[1:])
    out = np.zeros(cap, np.int64)
    cf = ctypes.c_int(0)
    n = lib().oracle_h3_polyfill(_ptr(lat), _ptr(lon), _ptr(ro), len(rings), res, _ptr(out), cap, ctypes.byref(cf))
    if n < 0:
        raise RuntimeError("oracle_h3_polyfill failed")
    return out[:n].copy(), bool(cf.value)


def h3_polyfill(parts, res, jdk=8):
    """grid_polyfill (H3) of a geometry given as parts: the parts' cells concatenated, plus whether
    every part's order is certain (collision-free)."""
    cells, ok = [], True
    for rings in parts:
        if not rings or len(rings[0]) == 0:
            continue
        c, cf = h3_polyfill_part(rings, res, jdk)
        cells.append(c)
        ok &= cf
    return (np.concatenate(cells) if cells else np.zeros(0, np.int64)), ok


def h3_ring1(cell):
    out = np.zeros(16, np.int64)
    n = lib().oracle_h3_ring1(int(cell), _ptr(out))
    return out[:n].copy()


def jts_centroid(parts):
    xy, ro, pr = _geom_arrays(parts)
    g = _Geom(_ptr(xy).value, _ptr(ro).value, _ptr(pr).value, len(parts))
    c = np.zeros(2, np.float64)
    if not lib().oracle_jts_centroid(ctypes.byref(g), _ptr(c), _ptr(c[1:])):
        return None
    return float(c[0]), float(c[1])


def bng_polyfill(parts, res, cap=1 << 22):
    """grid_polyfill (BNG) of a geometry given as parts (eastings / northings): the cell set, as a
    sorted array."""
    xy, ro, pr = _geom_arrays(parts)
    g = _Geom(_ptr(xy).value, _ptr(ro).value, _ptr(pr).value, len(parts))
    out = np.zeros(cap, np.int64)
    n = lib().oracle_bng_polyfill(ctypes.byref(g), res, _ptr(out), cap)
    if n < 0:
        raise RuntimeError("oracle_bng_polyfill failed")
    return np.sort(out[:n])


def h3_buffer_radius(parts, res, jdk=8):
    """H3IndexSystem.getBufferRadius of a geometry given as parts of (lon, lat) rings."""
    xy, ro, pr = _geom_arrays(parts)
    g = _Geom(_ptr(xy).value, _ptr(ro).value, _ptr(pr).value, len(parts))
    return lib().oracle_h3_buffer_radius(ctypes.byref(g), res, jdk)
