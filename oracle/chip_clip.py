"""TEST INFRASTRUCTURE ONLY: the reference's border chip, restated in pure Python (small cases).

IndexSystem.getBorderChips (src/main/scala/com/databricks/labs/mosaic/core/index/IndexSystem.scala:152-168)
builds a border chip as ``geometry.intersection(indexToGeometry(index))`` -- JTS 1.19 overlay in the
plane of the coordinates against the cell polygon (H3: h3ToGeoBoundary in degrees with straight sides,
H3IndexSystem.scala:93-100; BNG: the square).  Restated independently of mosaic_amd/csrc/llclip.h:

* orientation signs exact (``fractions.Fraction`` on the doubles' binary values, after a float filter);
* crossing points: JTS 1.19 RobustLineIntersector.computeIntersect's rules (endpoint cases, collinear
  overlap) and Intersection.intersection (homogeneous coordinates conditioned by the envelopes'
  intersection midpoint), envelope check with nearestEndpoint as the fallback;
* Weiler-Atherton: rings walked with the interior on the left, pieces labelled by their midpoint
  (pieces on the cell boundary are not inside), inside runs linked counter-clockwise along the cell;
* output: each ring from its lowest vertex (least y, then x), shells counter-clockwise, holes
  clockwise, polygons and holes ordered by that vertex -- the order of the reference's rendered chips
  (tests/golden/notebook_vectors.json; 25 + 68 of its border chips bit-exact, the rest within 3 ulp
  of this restatement, tests/test_notebook_vectors.py).

Only tests/ import this module.
"""
import math
from fractions import Fraction as F


def orient(a, b, c):
    dl = (b[0] - a[0]) * (c[1] - a[1])
    dr = (b[1] - a[1]) * (c[0] - a[0])
    d0 = dl - dr
    if abs(d0) > 1e-12 * (abs(dl) + abs(dr)):
        return int(d0 > 0) - int(d0 < 0)
    d = (F(b[0]) - F(a[0])) * (F(c[1]) - F(a[1])) - (F(b[1]) - F(a[1])) * (F(c[0]) - F(a[0]))
    return int(d > 0) - int(d < 0)


def in_env(r, a, b):
    return min(a[0], b[0]) <= r[0] <= max(a[0], b[0]) and min(a[1], b[1]) <= r[1] <= max(a[1], b[1])


def _pt_seg(p, a, b):
    if a == b:
        return math.sqrt((p[0] - a[0]) ** 2 + (p[1] - a[1]) ** 2)
    len2 = (b[0] - a[0]) * (b[0] - a[0]) + (b[1] - a[1]) * (b[1] - a[1])
    r = ((p[0] - a[0]) * (b[0] - a[0]) + (p[1] - a[1]) * (b[1] - a[1])) / len2
    if r <= 0.0:
        return math.sqrt((p[0] - a[0]) ** 2 + (p[1] - a[1]) ** 2)
    if r >= 1.0:
        return math.sqrt((p[0] - b[0]) ** 2 + (p[1] - b[1]) ** 2)
    s = ((a[1] - p[1]) * (b[0] - a[0]) - (a[0] - p[0]) * (b[1] - a[1])) / len2
    return abs(s) * math.sqrt(len2)


def _nearest_endpoint(p1, p2, q1, q2):
    best, md = p1, _pt_seg(p1, q1, q2)
    for pt, d in ((p2, _pt_seg(p2, q1, q2)), (q1, _pt_seg(q1, p1, p2)), (q2, _pt_seg(q2, p1, p2))):
        if d < md:
            best, md = pt, d
    return best


def intersection(p1, p2, q1, q2):
    """JTS 1.19 Intersection.intersection + RobustLineIntersector's envelope check."""
    imnx = max(min(p1[0], p2[0]), min(q1[0], q2[0]))
    imxx = min(max(p1[0], p2[0]), max(q1[0], q2[0]))
    imny = max(min(p1[1], p2[1]), min(q1[1], q2[1]))
    imxy = min(max(p1[1], p2[1]), max(q1[1], q2[1]))
    mx, my = (imnx + imxx) / 2.0, (imny + imxy) / 2.0
    p1x, p1y, p2x, p2y = p1[0] - mx, p1[1] - my, p2[0] - mx, p2[1] - my
    q1x, q1y, q2x, q2y = q1[0] - mx, q1[1] - my, q2[0] - mx, q2[1] - my
    px, py, pw = p1y - p2y, p2x - p1x, p1x * p2y - p2x * p1y
    qx, qy, qw = q1y - q2y, q2x - q1x, q1x * q2y - q2x * q1y
    x, y, w = py * qw - qy * pw, qx * pw - px * qw, px * qy - qx * py
    r = None
    if w != 0:
        xi, yi = x / w, y / w
        if math.isfinite(xi) and math.isfinite(yi):
            r = (xi + mx, yi + my)
    if r is None or not (in_env(r, p1, p2) and in_env(r, q1, q2)):
        r = _nearest_endpoint(p1, p2, q1, q2)
    return r


def _meet(a, b, c, d):
    """RobustLineIntersector.computeIntersect of a-b with c-d: list of points (0-2)."""
    if max(a[0], b[0]) < min(c[0], d[0]) or min(a[0], b[0]) > max(c[0], d[0]) or \
            max(a[1], b[1]) < min(c[1], d[1]) or min(a[1], b[1]) > max(c[1], d[1]):
        return []
    pq1, pq2 = orient(a, b, c), orient(a, b, d)
    if pq1 * pq2 > 0:
        return []
    qp1, qp2 = orient(c, d, a), orient(c, d, b)
    if qp1 * qp2 > 0:
        return []
    if pq1 == 0 and pq2 == 0 and qp1 == 0 and qp2 == 0:
        ci, di, ai, bi = in_env(c, a, b), in_env(d, a, b), in_env(a, c, d), in_env(b, c, d)
        if ci and di:
            out = [c, d]
        elif ai and bi:
            out = [a, b]
        elif ci and ai:
            out = [c] + ([a] if c != a or not di else [])
        elif ci and bi:
            out = [c] + ([b] if c != b or not di else [])
        elif di and ai:
            out = [d] + ([a] if d != a or not ci else [])
        elif di and bi:
            out = [d] + ([b] if d != b or not ci else [])
        else:
            out = []
        return out[:1] if len(out) == 2 and out[0] == out[1] else out
    if pq1 == 0 or pq2 == 0 or qp1 == 0 or qp2 == 0:
        if a == c or a == d:
            return [a]
        if b == c or b == d:
            return [b]
        if pq1 == 0:
            return [c]
        if pq2 == 0:
            return [d]
        return [a] if qp1 == 0 else [b]
    return [intersection(a, b, c, d)]


def _locate(p, ring):
    """0 exterior, 1 boundary, 2 interior of an open ring."""
    n = len(ring)
    odd = False
    for i in range(n):
        a, b = ring[i], ring[(i + 1) % n]
        if orient(a, b, p) == 0 and in_env(p, a, b):
            return 1
        if (a[1] > p[1]) != (b[1] > p[1]):
            if (orient(a, b, p) > 0) == (b[1] > a[1]):
                odd = not odd
    return 2 if odd else 0


def _pos(C, j, q):
    """(side, parameter) of q on side j of C (C's vertices: (index, 0))."""
    n = len(C)
    c, d = C[j], C[(j + 1) % n]
    if q == c:
        return (j, 0.0)
    if q == d:
        return ((j + 1) % n, 0.0)
    dx, dy = d[0] - c[0], d[1] - c[1]
    s = (q[0] - c[0]) / dx if abs(dx) >= abs(dy) else (q[1] - c[1]) / dy
    return (j, min(max(s, 0.0), 0.99999999999999989))


def _pos_of(C, q):
    for j, c in enumerate(C):
        if q == c:
            return (j, 0.0)
    for j in range(len(C)):
        c, d = C[j], C[(j + 1) % len(C)]
        if in_env(q, c, d) and orient(c, d, q) == 0:
            return _pos(C, j, q)
    raise ValueError("transition off the cell boundary")


def _is_ccw(r):
    """JTS 1.19 Orientation.isCCW of an open ring."""
    ring = list(r) + [r[0]]
    n = len(r)
    up_hi, prev_y, up_low, i_up_hi = ring[0], ring[0][1], None, 0
    for i in range(1, n + 1):
        py = ring[i][1]
        if py > prev_y and py >= up_hi[1]:
            up_hi, i_up_hi, up_low = ring[i], i, ring[i - 1]
        prev_y = py
    if i_up_hi == 0:
        return False
    i_down_low = i_up_hi
    while True:
        i_down_low = (i_down_low + 1) % n
        if i_down_low == i_up_hi or ring[i_down_low][1] != up_hi[1]:
            break
    down_low = ring[i_down_low]
    down_hi = ring[i_down_low - 1 if i_down_low > 0 else n - 1]
    if up_hi == down_hi:
        if up_low == up_hi or down_low == up_hi or up_low == down_low:
            return False
        return orient(up_low, up_hi, down_low) == 1
    return down_hi[0] - up_hi[0] < 0


def _area2(r, o=None):
    o = o or r[0]
    return sum((r[i][0] - o[0]) * (r[(i + 1) % len(r)][1] - o[1]) - (r[(i + 1) % len(r)][0] - o[0]) * (r[i][1] - o[1])
               for i in range(len(r)))


def clip(parts, C):
    """parts: [[closed ring [(x, y)...], ...] (shell first), ...]; C: the cell, counter-clockwise,
    open.  Returns [[shell, hole...], ...] of closed rings in output order ([] for no chip)."""
    n_c = len(C)
    eps2 = 1e-12 * _area2(C)
    shells, holes = [], []
    for pi, part in enumerate(parts):
        chains, whole = [], []
        for ri, ring in enumerate(part):
            r = [tuple(map(float, p)) for p in (ring[:-1] if tuple(ring[0]) == tuple(ring[-1]) else ring)]
            if len(r) < 3:
                continue
            if (ri == 0) != _is_ccw(r):
                r = [r[0]] + r[1:][::-1]
            n = len(r)
            pts, labs = [], []  # points of the walk and the label of the piece after each
            for k in range(n):
                a, b = r[k], r[(k + 1) % n]
                if a == b:
                    continue
                ev = {}
                for j in range(n_c):
                    for q in _meet(a, b, C[j], C[(j + 1) % n_c]):
                        if q != a and q != b and q not in ev:
                            ev[q] = _pos(C, j, q)
                dx, dy = b[0] - a[0], b[1] - a[1]
                order = sorted(ev, key=lambda q: (q[0] - a[0]) / dx if abs(dx) >= abs(dy) else (q[1] - a[1]) / dy)
                la, lb = _locate(a, C), _locate(b, C)
                seq = [a] + order + [b]
                for i in range(len(seq) - 1):
                    p0, p1 = seq[i], seq[i + 1]
                    if i == 0 and la != 1:
                        lab = la == 2
                    elif i == len(seq) - 2 and lb != 1:
                        lab = lb == 2
                    else:
                        lab = _locate(((p0[0] + p1[0]) / 2, (p0[1] + p1[1]) / 2), C) == 2
                    pts.append((p0, ev.get(p0)))
                    labs.append(lab)
            if not labs:
                continue
            if all(labs):
                whole.append((ri, [p for p, _ in pts]))
                continue
            if not any(labs):
                continue
            m = len(labs)
            starts = [i for i in range(m) if not labs[i - 1] and labs[i]]
            for i0 in starts:
                p, ps = pts[i0]
                ch = [p]
                j = i0
                while labs[j]:
                    j = (j + 1) % m
                    ch.append(pts[j][0])
                q, qs = pts[j]
                chains.append(dict(pin=ps if ps is not None else _pos_of(C, p), pts=ch,
                                   pout=qs if qs is not None else _pos_of(C, q)))
        for c in chains:  # next entry counter-clockwise along C
            after = [d for d in chains if d["pin"] >= c["pout"]]
            c["next"] = min(after or chains, key=lambda d: d["pin"])
        seen = set()
        for c0 in chains:
            if id(c0) in seen:
                continue
            ring, c = [], c0
            while True:
                seen.add(id(c))
                ring += c["pts"]
                nx = c["next"]
                m = c["pout"][0] + 1
                wrap = nx["pin"] < c["pout"]
                for _ in range(n_c):
                    if m == n_c:
                        if not wrap:
                            break
                        m = 0
                    if wrap and m > c["pout"][0]:
                        ring.append(C[m])
                    elif (m, 0.0) < nx["pin"]:
                        ring.append(C[m])
                    else:
                        break
                    m += 1
                c = nx
                if c is c0:
                    break
            shells.append((pi, ring))
        for ri, rr in whole:
            (shells if ri == 0 else holes).append((pi, rr))
        if not chains and not any(ri == 0 for ri, _ in whole):
            loc = 1
            for cv in list(C) + [(sum(v[0] for v in C) / n_c, sum(v[1] for v in C) / n_c)]:
                locs = [_locate(cv, [tuple(map(float, p)) for p in ring[:-1]]) for ring in part]
                if any(l == 1 for l in locs):
                    continue
                loc = 2 if locs[0] == 2 and not any(l == 2 for l in locs[1:]) else 0
                break
            if loc == 2:
                shells.append((pi, list(C)))

    def clean(r):
        o = []
        for p in r:
            if not o or o[-1] != p:
                o.append(p)
        while len(o) > 1 and o[0] == o[-1]:
            o.pop()
        return o

    def rot(r):
        k = min(range(len(r)), key=lambda i: (r[i][1], r[i][0]))
        return r[k:] + r[:k]

    shells = [(pi, rot(s)) for pi, s in ((pi, clean(s)) for pi, s in shells) if len(s) >= 3 and abs(_area2(s)) > eps2]
    holes = [(pi, rot(h)) for pi, h in ((pi, clean(h)) for pi, h in holes) if len(h) >= 3 and abs(_area2(h)) > eps2]
    shells.sort(key=lambda t: (t[1][0][1], t[1][0][0]))
    out = [[s] for _, s in shells]
    for pi, h in sorted(holes, key=lambda t: (t[1][0][1], t[1][0][0])):
        own = [i for i, (pj, s) in enumerate(shells) if pj == pi and _locate(h[0], s) == 2]
        cand = own or [i for i, (pj, _) in enumerate(shells) if pj == pi] or [0]
        if out:
            out[cand[0]].append(h)
    return [[r + [r[0]] for r in p] for p in out]
