"""TEST INFRASTRUCTURE ONLY: exact rational point-in-polygon checker (pure Python, small cases).

Independent of the C oracle's floating-point filter and double-double arithmetic: orientation
signs are computed with ``fractions.Fraction`` on the exact binary values of the doubles, and the
location rules follow JTS 1.19 PointLocator / RayCrossingCounter (see oracle/pip.c for the
reference trail: ST_Contains.scala:34-42 -> MosaicGeometryJTS.scala:101 -> JTS Geometry.contains).
Used to pin the C oracle's contains() on boundary / near-boundary cases.
"""
from fractions import Fraction

INTERIOR, BOUNDARY, EXTERIOR = 0, 1, 2


def orientation(p1, p2, q):
    ax, ay = Fraction(p2[0]) - Fraction(p1[0]), Fraction(p2[1]) - Fraction(p1[1])
    bx, by = Fraction(q[0]) - Fraction(p2[0]), Fraction(q[1]) - Fraction(p2[1])
    det = ax * by - ay * bx
    return (det > 0) - (det < 0)


def locate_in_ring(p, ring):
    px, py = p
    crossings = 0
    for i in range(1, len(ring)):
        p1, p2 = ring[i], ring[i - 1]
        if p1[0] < px and p2[0] < px:
            continue
        if px == p2[0] and py == p2[1]:
            return BOUNDARY
        if p1[1] == py and p2[1] == py:
            if min(p1[0], p2[0]) <= px <= max(p1[0], p2[0]):
                return BOUNDARY
            continue
        if (p1[1] > py and p2[1] <= py) or (p2[1] > py and p1[1] <= py):
            o = orientation(p1, p2, p)
            if o == 0:
                return BOUNDARY
            if p2[1] < p1[1]:
                o = -o
            if o == 1:
                crossings += 1
    return INTERIOR if crossings % 2 == 1 else EXTERIOR


def _env_excludes(p, ring):
    xs = [v[0] for v in ring]
    ys = [v[1] for v in ring]
    return p[0] < min(xs) or p[0] > max(xs) or p[1] < min(ys) or p[1] > max(ys)


def locate_in_polygon(p, rings):
    if not rings or not rings[0]:
        return EXTERIOR
    shell = EXTERIOR if _env_excludes(p, rings[0]) else locate_in_ring(p, rings[0])
    if shell != INTERIOR:
        return shell
    for hole in rings[1:]:
        if _env_excludes(p, hole):
            continue
        h = locate_in_ring(p, hole)
        if h == INTERIOR:
            return EXTERIOR
        if h == BOUNDARY:
            return BOUNDARY
    return INTERIOR


def contains(parts, p):
    """parts: list of polygons, each a list of rings (list of (x, y)); True iff JTS contains."""
    verts = [v for rings in parts for ring in rings for v in ring]
    if not verts:
        return False
    xs = [v[0] for v in verts]
    ys = [v[1] for v in verts]
    if p[0] < min(xs) or p[0] > max(xs) or p[1] < min(ys) or p[1] > max(ys):
        return False
    if len(parts) == 1:
        return locate_in_polygon(p, parts[0]) == INTERIOR
    is_in, nb = False, 0
    for rings in parts:
        loc = locate_in_polygon(p, rings)
        if loc == INTERIOR:
            is_in = True
        elif loc == BOUNDARY:
            nb += 1
    if nb % 2 == 1:
        return False
    return nb > 0 or is_in


def segments_intersect(p1, p2, q1, q2):
    """Closed segments p1p2 and q1q2 share a point, in exact rational arithmetic (the predicate
    JTS RobustLineIntersector.computeIntersect decides with Orientation.index signs)."""
    o1, o2 = orientation(p1, p2, q1), orientation(p1, p2, q2)
    o3, o4 = orientation(q1, q2, p1), orientation(q1, q2, p2)
    if o1 * o2 < 0 and o3 * o4 < 0:
        return True

    def on(a, b, c):  # c collinear with ab: on the closed segment?
        return min(a[0], b[0]) <= c[0] <= max(a[0], b[0]) and min(a[1], b[1]) <= c[1] <= max(a[1], b[1])

    return ((o1 == 0 and on(p1, p2, q1)) or (o2 == 0 and on(p1, p2, q2)) or (o3 == 0 and on(q1, q2, p1))
            or (o4 == 0 and on(q1, q2, p2)))


# ---- area of A n B by vertical slabs (exact rationals): the checker of the engine's
# st_intersection_aggregate areas (a different algorithm from the engine's boundary integral).
# Between consecutive x-coordinates of all vertices and all edge crossings, the edges crossing a
# slab keep their vertical order, so the length of {y : (x, y) in A n B} is linear in x and the
# midpoint rule is exact.  Rings: lists of (x, y), closed (last == first); parts: lists of rings
# (shell first); inside = odd crossing count per part (valid polygons), any part.
def _edges(parts):
    out = []
    for rings in parts:
        for r in rings:
            pts = [(Fraction(x), Fraction(y)) for x, y in r]
            out.extend((pts[i], pts[i + 1]) for i in range(len(pts) - 1) if pts[i] != pts[i + 1])
    return out


def _crossings_x(ea, eb):
    xs = set()
    for (p, q) in ea:
        for (r, s) in eb:
            d = (q[0] - p[0]) * (s[1] - r[1]) - (q[1] - p[1]) * (s[0] - r[0])
            if d == 0:
                continue
            t = ((r[0] - p[0]) * (s[1] - r[1]) - (r[1] - p[1]) * (s[0] - r[0])) / d
            u = ((r[0] - p[0]) * (q[1] - p[1]) - (r[1] - p[1]) * (q[0] - p[0])) / d
            if 0 <= t <= 1 and 0 <= u <= 1:
                xs.add(p[0] + t * (q[0] - p[0]))
    return xs


def _section(edges_by_part, x):
    """per part: sorted y where the vertical line x crosses its edges (x strictly inside a slab)"""
    out = []
    for edges in edges_by_part:
        ys = []
        for (p, q) in edges:
            if (p[0] < x < q[0]) or (q[0] < x < p[0]):
                ys.append(p[1] + (x - p[0]) * (q[1] - p[1]) / (q[0] - p[0]))
        out.append(sorted(ys))
    return out


def _inside_len(sec_a, sec_b):
    """length of the y-set inside some part of A and some part of B"""
    def intervals(sec):
        iv = []
        for ys in sec:
            iv.extend((ys[i], ys[i + 1]) for i in range(0, len(ys) - 1, 2))
        return iv
    ia, ib = intervals(sec_a), intervals(sec_b)
    total = Fraction(0)
    for (a0, a1) in ia:
        for (b0, b1) in ib:
            lo, hi = max(a0, b0), min(a1, b1)
            if hi > lo:
                total += hi - lo
    return total


def intersection_area(parts_a, parts_b):
    ea = [_edges([p]) for p in parts_a]
    eb = [_edges([p]) for p in parts_b]
    fa = [e for es in ea for e in es]
    fb = [e for es in eb for e in es]
    xs = {p[0] for e in fa + fb for p in e} | _crossings_x(fa, fb)
    xs = sorted(xs)
    area = Fraction(0)
    for i in range(len(xs) - 1):
        x0, x1 = xs[i], xs[i + 1]
        xm = (x0 + x1) / 2
        area += (x1 - x0) * _inside_len(_section(ea, xm), _section(eb, xm))
    return area


def polygon_area(parts):
    """JTS getArea: per part |shell| - sum |holes| (shoelace, exact)"""
    total = Fraction(0)
    for rings in parts:
        for k, r in enumerate(rings):
            pts = [(Fraction(x), Fraction(y)) for x, y in r]
            a = sum(pts[i][0] * pts[i + 1][1] - pts[i + 1][0] * pts[i][1] for i in range(len(pts) - 1)) / 2
            total += abs(a) if k == 0 else -abs(a)
    return total


# ---- st_intersection_aggregate's geometry: symmetric difference of an emitted boundary against the
# exact set (float slabs; the checker of overlay.h / isect_geom.cpp, a different algorithm from the
# engine's noding + labelling).  The set is X = union over units u of (some part of A_u holds p) and
# (some part of B_u holds p) -- per joined cell the union of the group's left chips intersected with
# the union of its right chips (None: that side covers everything); the emitted result is a list of
# directed edges (x0, y0, x1, y1), interior on the left, whose winding number W is the result's
# indicator.  Between consecutive abscissae of all vertices and all edge crossings nothing crosses,
# so the length of {y : W != X} is linear in x and the midpoint rule exact (up to rounding).
def symdiff_area(edges, units):
    """(area of {W != X}, area of X, area of {W == 1}); units: [(parts_a, parts_b), ...]"""
    import numpy as np

    segs, ids = [], []  # ids: (unit, side, part) -> flat part number
    part_no = {}
    for u, (pa, pb) in enumerate(units):
        for side, parts in ((0, pa), (1, pb)):
            for k, rings in enumerate(parts or []):
                pid = part_no.setdefault((u, side, k), len(part_no))
                for r in rings:
                    for i in range(len(r) - 1):
                        if tuple(r[i]) != tuple(r[i + 1]):
                            segs.append((r[i][0], r[i][1], r[i + 1][0], r[i + 1][1]))
                            ids.append(pid)
    n_in = len(segs)
    segs += [tuple(e[:4]) for e in edges]
    allsegs = np.array(segs, float).reshape(-1, 4)
    ids = np.array(ids, int)
    xs = set(allsegs[:, 0].tolist()) | set(allsegs[:, 2].tolist())
    p, q = allsegs[:, None, :2], allsegs[:, None, 2:]
    r, s = allsegs[None, :, :2], allsegs[None, :, 2:]
    d = (q[..., 0] - p[..., 0]) * (s[..., 1] - r[..., 1]) - (q[..., 1] - p[..., 1]) * (s[..., 0] - r[..., 0])
    with np.errstate(divide="ignore", invalid="ignore"):
        t = ((r[..., 0] - p[..., 0]) * (s[..., 1] - r[..., 1]) - (r[..., 1] - p[..., 1]) * (s[..., 0] - r[..., 0])) / d
        u = ((r[..., 0] - p[..., 0]) * (q[..., 1] - p[..., 1]) - (r[..., 1] - p[..., 1]) * (q[..., 0] - p[..., 0])) / d
        ok = (d != 0) & (t >= 0) & (t <= 1) & (u >= 0) & (u <= 1)
        cx = p[..., 0] + t * (q[..., 0] - p[..., 0])
    xs |= set(cx[ok].tolist())
    xs = np.array(sorted(xs))
    unit_of = [None] * len(part_no)
    for (uu, side, k), pid in part_no.items():
        unit_of[pid] = (uu, side)
    inp, outp = allsegs[:n_in], allsegs[n_in:]
    sg = np.where(outp[:, 2] > outp[:, 0], 1, -1)

    def cross_y(sg4, xm):
        x0, y0, x1, y1 = sg4[:, 0], sg4[:, 1], sg4[:, 2], sg4[:, 3]
        m = ((x0 < xm) & (xm < x1)) | ((x1 < xm) & (xm < x0))
        with np.errstate(divide="ignore", invalid="ignore"):
            y = y0 + (xm - x0) * (y1 - y0) / (x1 - x0)
        return m, y

    def member(par):
        cov = [[units[uu][0] is None, units[uu][1] is None] for uu in range(len(units))]
        for pid, v in enumerate(par):
            if v:
                uu, side = unit_of[pid]
                cov[uu][side] = True
        return any(a and b for a, b in cov)

    diff = area_x = area_w = 0.0
    for i in range(len(xs) - 1):
        x0, x1 = xs[i], xs[i + 1]
        if x1 <= x0:
            continue
        xm = 0.5 * (x0 + x1)
        m, y = cross_y(inp, xm)
        ev = [(yy, 0, k) for yy, k in zip(y[m].tolist(), ids[m].tolist())]
        m, y = cross_y(outp, xm)
        ev += [(yy, 1, g) for yy, g in zip(y[m].tolist(), sg[m].tolist())]
        ev.sort()
        par = [False] * len(part_no)
        w = 0
        lx = lw = ld = 0.0
        for j, (yy, kind, v) in enumerate(ev):
            if kind == 0:
                par[v] = not par[v]
            else:
                w += v
            if j + 1 < len(ev):
                h = ev[j + 1][0] - yy
                if h > 0:
                    f = member(par)
                    lx += h * f
                    lw += h * (w == 1)
                    ld += h * abs(w - int(f))
        diff += (x1 - x0) * ld
        area_x += (x1 - x0) * lx
        area_w += (x1 - x0) * lw
    return diff, area_x, area_w
