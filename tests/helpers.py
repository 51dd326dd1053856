"""Test helpers: synthetic chip tables and adversarial points (host side)."""
import numpy as np

from mosaic_amd import wkb as W


def synthetic_chips(zones, geom_ids, res, cell_fn, rng, pts_per_zone=400, core_frac=0.3, clip=False):
    """A chip table whose cells are the cells of random points inside each zone's bbox.

    The join's semantics are defined for any chip table, so parity tests do not need real
    tessellation output: every chip gets the zone's full geometry as its wkb (or none when core).
    Returns dict(is_core, index_id, wkb list, polygon_key) with zone position as the key.
    """
    is_core, ids, wkbs, keys = [], [], [], []
    for k, g in enumerate(geom_ids):
        x0, y0, x1, y1 = zones.geom_bbox(g)
        xs = rng.uniform(x0, x1, pts_per_zone)
        ys = rng.uniform(y0, y1, pts_per_zone)
        cells = np.unique(cell_fn(xs, ys, res))
        blob = zones.wkb(g, big_endian=bool(k % 2))
        for c in cells:
            core = rng.random() < core_frac
            is_core.append(1 if core else 0)
            ids.append(int(c))
            wkbs.append(None if core and rng.random() < 0.5 else blob)
            keys.append(k)
    return dict(is_core=np.array(is_core, np.uint8), index_id=np.array(ids, np.int64), wkb=wkbs,
                polygon_key=np.array(keys, np.int32))


def chips_to_oracle(chips):
    lens = np.array([0 if w is None else len(w) for w in chips["wkb"]], np.int64)
    offs = np.zeros(len(lens) + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    data = np.frombuffer(b"".join(b"" if w is None else w for w in chips["wkb"]) or b"\0", np.uint8).copy()
    return dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
                wkb_offsets=offs, wkb=data)


def boundary_points(zones, geom_ids, rng, n_per=40):
    """Points exactly on zone vertices, on exactly representable edge points, and just off them."""
    xs, ys = [], []
    for g in geom_ids:
        for rings in zones.parts(g):
            ring = rings[0]
            for _ in range(n_per):
                i = int(rng.integers(0, len(ring) - 1))
                (ax, ay), (bx, by) = ring[i], ring[i + 1]
                kind = rng.random()
                if kind < 0.4:
                    xs.append(ax)
                    ys.append(ay)
                elif kind < 0.7:
                    t = 0.5
                    xs.append(ax + t * (bx - ax))
                    ys.append(ay + t * (by - ay))
                else:
                    xs.append(np.nextafter(ax, ax + 1))
                    ys.append(ay)
    return np.array(xs), np.array(ys)


def _halfway_strings(rng, n):
    """Decimal strings exactly halfway between two adjacent doubles (and one digit off either
    side): the cases where correct rounding needs more than the first 17 digits."""
    from decimal import Decimal, getcontext

    getcontext().prec = 1200
    out = []
    for _ in range(n):
        e = int(rng.integers(-40, 40))
        v = float(rng.uniform(1, 2)) * 2.0 ** e * (1 if rng.random() < 0.5 else -1)
        nx = np.nextafter(v, np.inf)
        mid = (Decimal(v) + Decimal(float(nx))) / 2
        s = format(mid, "f")
        out.append(s)
        out.append(s + "0000000000000000000001")  # just above halfway: sticky digit far out
        out.append(format(mid, ".25e"))
        out.append(format(mid, ".18e"))  # 19 digits: the double-double path must still round right
        out.append(format(mid, ".16e"))
    return out


def point_rows(rng, n=3000):
    """(format, row bytes) corpus for the point decoder: valid points in every syntax the decoder
    accepts, numbers that stress correct rounding, and rows that must take the row path (other
    geometry types, EMPTY, malformed text / WKB).  Formats: 0 WKB, 1 WKT, 2 hex WKB."""
    import struct

    rows = []
    # the reference's own WKT point fixtures (test/package.scala:70, 91)
    rows += [(1, b"POINT (-75.78033 35.18937)"), (1, b"POINT (75780 35189)")]
    nums = []
    for _ in range(n):
        v = float(rng.uniform(-180, 180))
        r = rng.random()
        if r < 0.2:
            nums.append(repr(v))
        elif r < 0.4:
            nums.append("%.6f" % v)
        elif r < 0.5:
            nums.append("%.16f" % v)
        elif r < 0.6:
            nums.append("%.20e" % (v * 10.0 ** int(rng.integers(-300, 300))))
        elif r < 0.7:
            nums.append(repr(float(rng.uniform(-1, 1)) * 10.0 ** int(rng.integers(-320, 308))))
        elif r < 0.8:
            nums.append("%d" % int(v * 1e6))
        elif r < 0.9:
            nums.append("%.40g" % v)
        else:
            nums.append("".join(str(int(d)) for d in rng.integers(0, 10, int(rng.integers(18, 60)))) + "e-" +
                        str(int(rng.integers(0, 60))))
    nums += _halfway_strings(rng, 200)
    nums += ["4.9e-324", "2.4703282292062327e-324", "2.4703282292062328e-324", "1.7976931348623157e308",
             "1.7976931348623158e308", "1.7976931348623159e308", "1e309", "2.2250738585072012e-308",
             "2.2250738585072011e-308", "0.0", "-0.0", "1.", ".5", "+3.25", "-.125e+2", "7d", "7.5F", "1e-400",
             "9007199254740993", "9007199254740993.0000000000000000000000001", "1" + "0" * 400, "0." + "0" * 330 + "5",
             "1" * 900 + "e-880", "Infinity", "-Infinity", "NaN", "nan", "-NaN"]
    rng.shuffle(nums)
    fmts = ["POINT ({} {})", "POINT({} {})", "point ( {}  {} )", "  POINT\t(\n{} {})\r\n", "POINT Z ({} {} 1.5)",
            "POINTZ ({} {} 3)", "POINT M ({} {} 2)", "POINT ZM ({} {} 1 2)", "Point ({} {} 9)", "POINT zm({} {} 1 2)"]
    for k in range(0, len(nums) - 1, 2):
        f = fmts[int(rng.integers(0, len(fmts)))]
        rows.append((1, f.format(nums[k], nums[k + 1]).encode()))
    # row path: other types, empty, malformed
    rows += [(1, s.encode()) for s in [
        "POINT EMPTY", "point empty", "POINT Z EMPTY", "POLYGON EMPTY", "MULTIPOINT ((10 40), (40 30))",
        "LINESTRING (0 0, 1 1)", "POLYGON ((0 0, 1 0, 1 1, 0 0))", "GEOMETRYCOLLECTION (POINT (1 2))",
        "POINT (1)", "POINT (1 2 3 4)", "POINT Z (1 2)", "POINT ZM (1 2 3)", "POINT (1 2) x", "POINT (1, 2)",
        "POINT (1 2", "POINT 1 2", "POINT (0x1p3 2)", "POINT (1e 2)", "POINT (1.2.3 4)", "POINT (-nan 1)",
        "POINT (Inf 1)", "POINTQ (1 2)", "", "   ", "POINT (1 2) # c", "POINT (1-2 3)", "POINT (--1 2)"]]
    # WKB: little / big endian, EWKB Z / M / SRID, ISO Z / M / ZM, other types, truncated, NaN
    for k in range(600):
        x, y = float(rng.uniform(-180, 180)), float(rng.uniform(-90, 90))
        le = k % 2 == 0
        e = "<" if le else ">"
        bo = b"\x01" if le else b"\x00"
        kind = k % 8
        if kind == 0:
            b = bo + struct.pack(e + "Idd", 1, x, y)
        elif kind == 1:
            b = bo + struct.pack(e + "Iddd", 0x80000001, x, y, 5.0)
        elif kind == 2:
            b = bo + struct.pack(e + "IIdd", 0x20000001, 4326, x, y)
        elif kind == 3:
            b = bo + struct.pack(e + "Idddd", 3001, x, y, 1.0, 2.0)
        elif kind == 4:
            b = bo + struct.pack(e + "Iddd", 2001, x, y, 7.0)
        elif kind == 5:
            b = bo + struct.pack(e + "IIddd", 0xE0000001 & 0xA0000001, 27700, x, y, 1.0)
        elif kind == 6:
            b = bo + struct.pack(e + "Idd", 1, x, y) + b"\x00" * 7  # trailing bytes are ignored
        else:
            b = b"\x07" + struct.pack(">Idd", 1, x, y)  # any other byte order byte: big endian
        rows.append((0, b))
        rows.append((2, (b.hex().upper() if k % 3 else b.hex()).encode()))
    rows += [(0, b) for b in [b"", b"\x01", b"\x01\x01\x00\x00\x00" + b"\x00" * 15,
                              b"\x01" + struct.pack("<Idd", 1, float("nan"), 1.0),
                              b"\x01" + struct.pack("<Idd", 1, 1.0, float("nan")),
                              b"\x01" + struct.pack("<I", 3) + b"\x00" * 8, b"\x01" + struct.pack("<I", 9) + b"\x00" * 16,
                              b"\x00" + struct.pack(">Iddd", 1001, 1.0, 2.0, 3.0)[:-1]]]
    rows += [(2, s) for s in [b"0101000000000000000000F03F00000000000000400", b"01010000000000000000000F03G000000000000000040",
                              b"", b"0"]]
    return rows


def h3_cell_boundary_points(rng, n, res, lon_range=(-180.0, 180.0), lat_range=(-90.0, 90.0), iters=60):
    """Points within an ulp of H3 cell boundaries at `res`, by bisection on the oracle's cells.

    Pairs (p, p + d) with |d| about one cell edge that land in different cells are bisected until
    the two ends are adjacent doubles (or `iters` halvings): both ends are returned, so every pair
    straddles a boundary of the reference's own cells (edges, vertices where three cells meet, the
    fold axes and face edges at coarse resolutions).  Returns (lon, lat) arrays (degrees)."""
    import oracle

    edge_deg = 0.0019 * 7 ** ((9 - res) / 2.0)  # ~ res-r hexagon edge in degrees of latitude
    lon = rng.uniform(*lon_range, n)
    lat = rng.uniform(*lat_range, n)
    ang = rng.uniform(0, 2 * np.pi, n)
    span = edge_deg * rng.uniform(0.3, 1.5, n)
    lon2 = lon + span * np.cos(ang) / np.maximum(np.cos(np.radians(lat)), 0.05)
    lat2 = np.clip(lat + span * np.sin(ang), -90.0, 90.0)
    c0 = oracle.h3_point_to_index(lon, lat, res)
    c1 = oracle.h3_point_to_index(lon2, lat2, res)
    k = c0 != c1
    ax, ay, bx, by, ca = lon[k], lat[k], lon2[k], lat2[k], c0[k]
    for _ in range(iters):
        mx, my = 0.5 * (ax + bx), 0.5 * (ay + by)
        cm = oracle.h3_point_to_index(mx, my, res)
        same = cm == ca
        ax, ay = np.where(same, mx, ax), np.where(same, my, ay)
        bx, by = np.where(same, bx, mx), np.where(same, by, my)
    return np.concatenate([ax, bx]), np.concatenate([ay, by])
