"""Derive H3 v3.7's base-cell adjacency tables (baseCells.c baseCellNeighbors /
baseCellNeighbor60CCWRots) and the digit-carry tables of h3NeighborRotations (algos.c NEW_DIGIT_II,
NEW_ADJUSTMENT_II, NEW_DIGIT_III, NEW_ADJUSTMENT_III) from the tables already in h3_tables.h /
h3_face_tables.h, and write mosaic_amd/csrc/h3_neighbor_tables.h.

Hexagon base cell b (home face f, res-0 position h): its neighbour in direction d is the base cell at
res-0 position h + UNIT_VECS[d] on f, moved onto the adjacent face by _adjustOverageClassII when it
lies beyond f; the rotation is the 60-degree ccw turns from b's frame to the neighbour's home frame
(the face changes' ccwRot60 plus faceIjkBaseCells' rotation at the landing position).

Pentagon base cell p sits at an icosahedron vertex shared by five faces.  Each of those faces holds
exactly one neighbour of p: the res-0 position next to p inside the face (p at the face's corner
(2,0,0), (0,2,0) or (0,0,2); the neighbour one step toward the face centre: JK, IK or IJ of the
face's frame).  p's frame is its home face's with the k axis deleted, so going counter-clockwise
around the vertex (viewed from outside the sphere: H3's hex2d angles grow counter-clockwise) its
five directions are JK (the home face's neighbour), then IK, I, IJ, J on the next faces.  The
rotation to the neighbour's frame is faceIjkBaseCells' rotation there minus the turns from the face's
frame to p's frame (the angle from the face's inward direction to p's direction).  This reproduces
the published rows recalled for base cells 0 and 4 and is checked by a symmetry test (every
neighbour relation read back from the other side) and, in tests/test_h3_kring.py, by
h3NeighborRotations against a sphere search around all 12 pentagons.

Digit carries: adding unit vector `dir` to child digit `old` in an aperture-7 cluster gives a
position p (child lattice); if p is the centre or a unit vector it is the new digit with no carry,
else p = downAp7(parent unit vector q) + new digit for exactly one q (the carry).

    python tools/h3gen_neighbors.py [out.h]
"""
import math
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K_DIR = 1


def parse_table(text, name, conv=int):
    m = re.search(name + r"\[[^=]*=\s*\{(.*?)\};", text, re.S)
    return [conv(v) for v in re.findall(r"-?\d+(?:\.\d+)?(?:[eE][-+]?\d+)?", m.group(1))]


def norm(c):
    i, j, k = c
    if i < 0:
        j -= i; k -= i; i = 0
    if j < 0:
        i -= j; k -= j; j = 0
    if k < 0:
        i -= k; j -= k; k = 0
    mn = min(i, j, k)
    return (i - mn, j - mn, k - mn)


def add(a, b):
    return norm((a[0] + b[0], a[1] + b[1], a[2] + b[2]))


def sub(a, b):
    return norm((a[0] - b[0], a[1] - b[1], a[2] - b[2]))


def rot60ccw(c):
    i, j, k = c
    return norm((i + k, i + j, j + k))  # i -> (1,1,0), j -> (0,1,1), k -> (1,0,1)


def unit(d):
    return ((d >> 2) & 1, (d >> 1) & 1, d & 1)


def digit_of(c):
    c = norm(c)
    for d in range(7):
        if unit(d) == c:
            return d
    return None


def down_ap7(c):  # Class III: ccw
    i, j, k = c
    return norm((3 * i + j, 3 * j + k, i + 3 * k))


def down_ap7r(c):  # cw
    i, j, k = c
    return norm((3 * i + k, i + 3 * j, j + 3 * k))


# hex2d angle (degrees) of each direction digit: I 0, IJ 60, J 120, JK 180, K 240, IK 300
ANGLE = {4: 0, 6: 60, 2: 120, 3: 180, 1: 240, 5: 300}
INWARD = {(2, 0, 0): 3, (0, 2, 0): 5, (0, 0, 2): 6}  # a face corner's direction toward the face centre


def vec(lat, lng):
    return (math.cos(lat) * math.cos(lng), math.cos(lat) * math.sin(lng), math.sin(lat))


def tables():
    t = open(os.path.join(ROOT, "mosaic_amd", "csrc", "h3_tables.h")).read()
    bcd = parse_table(t, "kH3BaseCellData")
    bcd = [bcd[7 * b:7 * b + 7] for b in range(122)]
    fib = parse_table(t, "kH3FaceIjkBaseCells")
    fcg = parse_table(t, r"double kH3FaceCenterGeo", float)
    fcg = [(fcg[2 * f], fcg[2 * f + 1]) for f in range(20)]
    ft = open(os.path.join(ROOT, "mosaic_amd", "csrc", "h3_face_tables.h")).read()
    fnb = parse_table(ft, "kH3FaceNeighbors")
    fnb = [[fnb[20 * f + 5 * q:20 * f + 5 * q + 5] for q in range(4)] for f in range(20)]
    return bcd, fib, fcg, fnb


def derive():
    bcd, fib, fcg, fnb = tables()

    def base_at(face, c):
        i, j, k = c
        v = fib[((face * 3 + i) * 3 + j) * 3 + k]
        return v >> 3, v & 7

    nbrs, rots = [], []
    for b in range(122):
        face, i, j, k, pent = bcd[b][0], bcd[b][1], bcd[b][2], bcd[b][3], bcd[b][4]
        row_n, row_r = [b] + [127] * 6, [0] + [-1] * 6
        if not pent:
            for d in range(1, 7):
                p = add((i, j, k), unit(d))
                f, rot = face, 0
                # _adjustOverageClassII at res 0 (max dim 2, unit scale 1)
                for _ in range(3):
                    if sum(p) <= 2:
                        break
                    q = (3 if p[1] > 0 else 2) if p[2] > 0 else 1
                    g, ti, tj, tk, r = fnb[f][q]
                    for _ in range(r):
                        p = rot60ccw(p)
                    p = add(p, (ti, tj, tk))
                    f, rot = g, rot + r
                assert max(p) <= 2 and sum(p) <= 2, (b, d, p)
                nb, nr = base_at(f, p)
                row_n[d] = nb
                row_r[d] = (rot + nr) % 6
        else:
            # the five faces around the vertex, counter-clockwise seen from outside, home face first
            places = []
            for g in range(20):
                for q in INWARD:
                    bb, r = base_at(g, q)
                    if bb == b:
                        places.append((g, q, r))
            assert len(places) == 5, (b, places)
            pv = vec(*fcg[face])  # any point of the home face: only the order around the vertex matters
            vtx = None
            # the vertex: the unit vector equidistant from the five face centres
            cs = [vec(*fcg[g]) for g, _, _ in places]
            sx = [sum(c[a] for c in cs) for a in range(3)]
            nrm = math.sqrt(sum(v * v for v in sx))
            vtx = [v / nrm for v in sx]
            # tangent basis at the vertex: e (toward the home face centre), n = vtx x e (ccw)
            hc = vec(*fcg[face])
            dotv = sum(hc[a] * vtx[a] for a in range(3))
            e = [hc[a] - dotv * vtx[a] for a in range(3)]
            en = math.sqrt(sum(v * v for v in e))
            e = [v / en for v in e]
            n = [vtx[1] * e[2] - vtx[2] * e[1], vtx[2] * e[0] - vtx[0] * e[2], vtx[0] * e[1] - vtx[1] * e[0]]

            def ccw_angle(g):
                c = vec(*fcg[g])
                return math.atan2(sum(c[a] * n[a] for a in range(3)), sum(c[a] * e[a] for a in range(3))) % (2 * math.pi)

            places.sort(key=lambda pl: ccw_angle(pl[0]))
            h = [pl[0] for pl in places].index(face)
            places = places[h:] + places[:h]  # (the home face's angle is 0 up to rounding)
            for (g, q, _), d in zip(places, (3, 5, 4, 6, 2)):  # JK, IK, I, IJ, J
                w = INWARD[q]
                nb, nr = base_at(g, add(q, unit(w)))
                eff = ((ANGLE[d] - ANGLE[w]) // 60) % 6
                row_n[d] = nb
                row_r[d] = (nr - eff) % 6
        nbrs.append(row_n)
        rots.append(row_r)
    # the published rows recalled for base cells 0 and 4 (baseCells.c)
    assert nbrs[0] == [0, 1, 5, 2, 4, 3, 8], nbrs[0]
    assert rots[0] == [0, 5, 0, 0, 1, 5, 1], rots[0]
    assert nbrs[4] == [4, 127, 15, 8, 3, 0, 12], nbrs[4]
    assert rots[4] == [0, -1, 1, 0, 3, 4, 2], rots[4]
    # symmetry: every neighbour of b has b among its neighbours
    for b in range(122):
        for d in range(1, 7):
            nb = nbrs[b][d]
            if nb == 127:
                continue
            assert b in nbrs[nb][1:], (b, d, nb, nbrs[nb])
        assert len(set(x for x in nbrs[b][1:] if x != 127)) == (5 if bcd[b][4] else 6), (b, nbrs[b])

    def carries(down):
        nd = [[0] * 7 for _ in range(7)]
        na = [[0] * 7 for _ in range(7)]
        for old in range(7):
            for dr in range(7):
                p = add(unit(old), unit(dr))
                d = digit_of(p)
                if d is not None:
                    nd[old][dr], na[old][dr] = d, 0
                    continue
                hits = [(q, digit_of(sub(p, down(unit(q))))) for q in range(1, 7)]
                hits = [(q, dd) for q, dd in hits if dd is not None]
                assert len(hits) == 1, (old, dr, hits)
                na[old][dr], nd[old][dr] = hits[0]
        return nd, na

    nd_r, na_r = carries(down_ap7r)
    nd_c, na_c = carries(down_ap7)
    pub_ii1 = [1, 4, 3, 6, 5, 2, 0]
    pub_adj_ii1 = [0, 1, 0, 1, 0, 5, 0]
    if nd_r[1] == pub_ii1 and na_r[1] == pub_adj_ii1:
        carry = (nd_r, na_r, nd_c, na_c)
    else:
        assert nd_c[1] == pub_ii1 and na_c[1] == pub_adj_ii1, (nd_r[1], na_r[1], nd_c[1], na_c[1])
        carry = (nd_c, na_c, nd_r, na_r)
    return nbrs, rots, carry


def main(out_path):
    nbrs, rots, (nd_ii, na_ii, nd_iii, na_iii) = derive()

    def fmt(name, rows):
        out = [f"H3_TABLE int {name}[{len(rows)}][{len(rows[0])}] = {{"]
        for r in rows:
            out.append("    {" + ", ".join(str(v) for v in r) + "},")
        out.append("};")
        return out

    lines = ["/* Generated by tools/h3gen_neighbors.py -- do not edit.",
             " * H3 v3.7 baseCells.c baseCellNeighbors / baseCellNeighbor60CCWRots and algos.c NEW_DIGIT_II,",
             " * NEW_ADJUSTMENT_II, NEW_DIGIT_III, NEW_ADJUSTMENT_III, derived from h3_tables.h and",
             " * h3_face_tables.h (the derivation is in the generator).  Include after defining H3_TABLE. */",
             "#pragma once",
             "#ifndef H3_TABLE", "#define H3_TABLE static const", "#endif",
             "/* baseCellNeighbors[base cell][direction digit]; 127: none (a pentagon's deleted k axis) */"]
    lines += fmt("kH3BaseCellNeighbors", nbrs)
    lines.append("/* baseCellNeighbor60CCWRots[base cell][direction digit]; -1: none */")
    lines += fmt("kH3BaseCellNeighborRots", rots)
    lines.append("/* h3NeighborRotations digit carries: [old digit][direction] */")
    lines += fmt("kH3NewDigitII", nd_ii)
    lines += fmt("kH3NewAdjustmentII", na_ii)
    lines += fmt("kH3NewDigitIII", nd_iii)
    lines += fmt("kH3NewAdjustmentIII", na_iii)
    open(out_path, "w").write("\n".join(lines) + "\n")
    print("ok", out_path)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "mosaic_amd", "csrc", "h3_neighbor_tables.h"))
