"""TEST INFRASTRUCTURE ONLY: pure-Python restatement of the point-geometry decode in front of
grid_pointascellid (PointIndexGeom.scala:32-40 -> GeometryAPI.geometry, GeometryAPI.scala:64-72 ->
MosaicGeometryJTS.fromWKB / fromWKT / fromHEX, MosaicGeometryJTS.scala:164, 195-200 -> getCentroid
:49-53 -> MosaicPointJTS.getX / getY :23-25).  The arithmetic lives in JTS 1.19 (jts-core, pom.xml
:98-102, absent here [3P]); restated from its published WKTReader / WKBReader behaviour:

* WKT: java.io.StreamTokenizer (whitespace bytes 0..32, word chars [A-Za-z0-9+-.] and >= 160);
  "POINT" with an optional Z / M / ZM suffix or following word; "EMPTY"; "(" x y [z] [m] ")";
  numbers: "NaN" in any case (WKTReader.getNextNumber) else Double.parseDouble, which rounds the
  decimal value to nearest (ties to even) -- Python's float() does the same (correctly rounded).
* WKB: byte order byte 1 little endian, else big; (t & 0xffff) % 1000 type, Z / M from the high
  bits or the ISO thousands, SRID word if bit 29; a Point with x or y NaN is empty.
* HEX: WKBReader.hexToBytes (pairs of hex digits, trailing odd digit dropped).

Returns ("ok", x, y) or ("rowpath", reason): the engine's contract is that only rows JTS certainly
reads as a non-empty Point decode on the device; the rest go to the reference row path.
Parity is pinned by the reference's own point fixtures (test/package.scala:70, 91 WKT points) and
by Python's correctly rounded float() on adversarial digit strings (parity of the WKT grammar
corners is otherwise unpinned: no JVM here).
"""
import math
import re
import struct

_NUM = re.compile(r"^[+-]?(\d+\.?\d*|\.\d+)([eE][+-]?\d+)?[fFdD]?$")


def _number(tok):
    if tok.lower() == "nan":
        return float("nan")
    if tok in ("+NaN", "-NaN"):
        return float("nan")
    if tok in ("Infinity", "+Infinity"):
        return math.inf
    if tok == "-Infinity":
        return -math.inf
    if not _NUM.match(tok):
        raise ValueError(tok)
    t = tok[:-1] if tok[-1] in "fFdD" else tok
    return float(t)


def _tokens(s):
    out, i, n = [], 0, len(s)
    while i < n:
        c = s[i]
        if c <= 32:
            i += 1
            continue
        if chr(c).isascii() and (chr(c).isalnum() or chr(c) in "+-.") or c >= 160:
            j = i
            while j < n and ((chr(s[j]).isascii() and (chr(s[j]).isalnum() or chr(s[j]) in "+-.")) or s[j] >= 160):
                j += 1
            out.append(s[i:j].decode("latin-1"))
            i = j
        else:
            out.append(chr(c))
            i += 1
    return out


_MODS = {"z": 1, "m": 2, "zm": 3}


def wkt_point(text):
    s = text.encode("latin-1") if isinstance(text, str) else bytes(text)
    if len(s) > 4096:
        return ("rowpath", "long")
    toks = _tokens(s)
    if not toks or not toks[0][0].isalnum():
        return ("rowpath", "bad")
    kw = toks[0].lower()
    if not kw.startswith("point"):
        return ("rowpath", "notpoint")
    mods = 0
    if len(kw) > 5:
        if kw[5:] not in _MODS:
            return ("rowpath", "bad")
        mods = _MODS[kw[5:]]
    k = 1
    if k < len(toks) and mods == 0 and toks[k].lower() in _MODS:
        mods = _MODS[toks[k].lower()]
        k += 1
    if k < len(toks) and toks[k].lower() in _MODS:
        k += 1
    if k >= len(toks):
        return ("rowpath", "bad")
    if toks[k].lower() == "empty":
        return ("rowpath", "empty")
    if toks[k] != "(":
        return ("rowpath", "bad")
    k += 1
    need = 2 + (mods & 1) + ((mods >> 1) & 1)
    allowed = need + (1 if mods == 0 else 0)
    vals = []
    while k < len(toks) and toks[k] not in ("(", ")", ","):
        if len(vals) == allowed:
            return ("rowpath", "bad")
        try:
            vals.append(_number(toks[k]))
        except ValueError:
            return ("rowpath", "bad")
        k += 1
    if k >= len(toks) or toks[k] != ")" or len(vals) < need or k != len(toks) - 1:
        return ("rowpath", "bad")
    return ("ok", vals[0], vals[1])


def wkb_point(b):
    b = bytes(b)
    if len(b) < 5:
        return ("rowpath", "bad")
    le = b[0] == 1
    t = struct.unpack("<I" if le else ">I", b[1:5])[0]
    p = 5 + (4 if t & 0x20000000 else 0)
    base = t & 0xFFFF
    kind, iso = base % 1000, base // 1000
    if kind != 1:
        return ("rowpath", "notpoint" if 2 <= kind <= 7 else "bad")
    nord = 2 + (1 if (t & 0x80000000 or iso in (1, 3)) else 0) + (1 if (t & 0x40000000 or iso in (2, 3)) else 0)
    if len(b) < p + 8 * nord:
        return ("rowpath", "bad")
    x, y = struct.unpack("<dd" if le else ">dd", b[p:p + 16])
    if math.isnan(x) or math.isnan(y):
        return ("rowpath", "empty")
    return ("ok", x, y)


def hex_point(text):
    s = text if isinstance(text, str) else bytes(text).decode("latin-1")
    if len(s) > 4096:
        return ("rowpath", "long")
    nb = len(s) // 2
    try:
        if not all(c in "0123456789abcdefABCDEF" for c in s[:2 * nb]):
            raise ValueError
        b = bytes.fromhex(s[:2 * nb])
    except ValueError:
        return ("rowpath", "bad")
    return wkb_point(b)


def decode(fmt, row):
    return (wkb_point, wkt_point, hex_point)[fmt](row)


def coords_point(row):
    """The COORDS form (core/types/model/InternalGeometry.scala): row = (type_id, srid, boundaries,
    holes) or None.  MosaicPointJTS.fromInternal (core/geometry/point/MosaicPointJTS.scala:82-89)
    reads boundaries.head.head; InternalCoord(ArrayData) takes 2 values or the first 3.  Returns
    ("null",), ("ok", x, y) or ("path",) (other types: the centroid; rows the reference throws on)."""
    if row is None:
        return ("null",)
    type_id, _srid, boundaries = row[0], row[1], row[2]
    if type_id != 1 or not boundaries or not boundaries[0]:
        return ("path",)
    c = boundaries[0][0]
    if len(c) == 2 or len(c) >= 3:
        return ("ok", float(c[0]), float(c[1]))
    return ("path",)
