"""Host-side geometry encoding helpers: WKB and WKT for (Multi)Polygons and Points.

These mirror what the reference's JTS IO produces and consumes for the chip join's data contract:
chip ``wkb`` is JTS ``WKBWriter`` output (2D, big-endian by default --
MosaicGeometryJTS.scala:147 ``new WKBWriter().write``), and points arrive as WKT text in the
Quickstart (``MosaicGeometryIOCodeGenJTS.scala:16-29``).  Not on the hot path: the device reads
decoded rings from the chip table built by ``libmosaic_hip.so``.

Geometry model used throughout the package: a polygonal geometry is a list of parts; each part is
a list of rings; each ring is a list of (x, y) tuples, closed (first == last); ring 0 is the shell.
"""
import re
import struct

WKB_POINT = 1
WKB_POLYGON = 3
WKB_MULTIPOLYGON = 6


def polygon_wkb(rings, big_endian=True):
    bo = ">" if big_endian else "<"
    out = [struct.pack(bo + "BI", 0 if big_endian else 1, WKB_POLYGON), struct.pack(bo + "I", len(rings))]
    for ring in rings:
        out.append(struct.pack(bo + "I", len(ring)))
        out.append(b"".join(struct.pack(bo + "dd", x, y) for x, y in ring))
    return b"".join(out)


def geometry_wkb(parts, big_endian=True):
    """Polygon when there is one part, MultiPolygon otherwise (JTS WKBWriter layout)."""
    if len(parts) == 1:
        return polygon_wkb(parts[0], big_endian)
    bo = ">" if big_endian else "<"
    head = struct.pack(bo + "BII", 0 if big_endian else 1, WKB_MULTIPOLYGON, len(parts))
    return head + b"".join(polygon_wkb(p, big_endian) for p in parts)


def point_wkb(x, y, big_endian=True):
    bo = ">" if big_endian else "<"
    return struct.pack(bo + "BIdd", 0 if big_endian else 1, WKB_POINT, x, y)


def _read_geom(buf, pos):
    le = buf[pos] == 1
    bo = "<" if le else ">"
    (t,) = struct.unpack_from(bo + "I", buf, pos + 1)
    pos += 5
    if t & 0x20000000:
        pos += 4
    flags_z = bool(t & 0x80000000)
    flags_m = bool(t & 0x40000000)
    t &= 0x0FFFFFFF
    dims = 2 + (t // 1000 in (1, 3)) + (t // 1000 in (2, 3)) + flags_z + flags_m
    t %= 1000
    if t == WKB_POINT:
        vals = struct.unpack_from(bo + "d" * dims, buf, pos)
        return ("point", (vals[0], vals[1])), pos + 8 * dims
    if t == WKB_POLYGON:
        (nr,) = struct.unpack_from(bo + "I", buf, pos)
        pos += 4
        rings = []
        for _ in range(nr):
            (npts,) = struct.unpack_from(bo + "I", buf, pos)
            pos += 4
            vals = struct.unpack_from(bo + "d" * (dims * npts), buf, pos)
            pos += 8 * dims * npts
            rings.append([(vals[dims * k], vals[dims * k + 1]) for k in range(npts)])
        return ("polygon", [rings]), pos
    if t == WKB_MULTIPOLYGON:
        (np_,) = struct.unpack_from(bo + "I", buf, pos)
        pos += 4
        parts = []
        for _ in range(np_):
            (kind, g), pos = _read_geom(buf, pos)
            if kind != "polygon":
                raise ValueError("MultiPolygon member is not a Polygon")
            parts.extend(g)
        return ("polygon", parts), pos
    raise ValueError(f"unsupported WKB geometry type {t}")


def read_wkb(buf):
    """Returns ('point', (x, y)) or ('polygon', parts)."""
    g, _ = _read_geom(bytes(buf), 0)
    return g


_NUM = r"[-+]?(?:\d+\.?\d*|\.\d+)(?:[eE][-+]?\d+)?"


def _parse_ring_list(txt):
    rings = []
    for ring_txt in re.findall(r"\(([^()]*)\)", txt):
        pts = []
        for pair in ring_txt.split(","):
            nums = re.findall(_NUM, pair)
            pts.append((float(nums[0]), float(nums[1])))
        rings.append(pts)
    return rings


def read_wkt(text):
    """Minimal WKT reader for POINT / POLYGON / MULTIPOLYGON (JTS WKTReader subset)."""
    t = text.strip()
    head = t.split("(", 1)[0].strip().upper()
    if head.endswith("EMPTY") or t.upper().endswith("EMPTY"):
        kind = head.split()[0]
        return ("point", None) if kind == "POINT" else ("polygon", [])
    if head == "POINT":
        nums = re.findall(_NUM, t)
        return ("point", (float(nums[0]), float(nums[1])))
    if head == "POLYGON":
        return ("polygon", [_parse_ring_list(t)])
    if head == "MULTIPOLYGON":
        inner = t[t.index("(") + 1:t.rindex(")")]
        parts = []
        depth, start = 0, None
        for i, ch in enumerate(inner):
            if ch == "(":
                if depth == 0:
                    start = i
                depth += 1
            elif ch == ")":
                depth -= 1
                if depth == 0:
                    parts.append(_parse_ring_list(inner[start + 1:i]))
        return ("polygon", parts)
    raise ValueError(f"unsupported WKT: {text[:40]}")


def point_wkt(x, y):
    """JTS WKTWriter-style point text (repr keeps the exact double)."""
    return f"POINT ({x!r} {y!r})"
