"""Derive and check the H3 v3.7 constant tables used by geoToH3, then emit them as a C header.

H3 (uber/h3 v3.7.x, bundled in com.uber:h3:3.7.0, reference pom.xml:91-97) is a third-party
dependency that is absent from /root/reference and from this image.  The tables the point->cell
path needs are:

  faceCenterGeo[20]          lat/lng (radians) of the 20 icosahedron face centres
  faceCenterPoint[20]        the same as unit 3-vectors
  faceAxesAzRadsCII[20][3]   azimuth (radians, cw from north) of each face's Class II i/j/k axes
  baseCellData[122]          home face + home IJK + pentagon flag + cw-offset faces per base cell
  faceIjkBaseCells[20][3][3][3]  base cell and ccw 60-degree rotation count for each res-0 face IJK

The face centres are H3's published 18-digit literals.  Everything else is *derived* here from that
icosahedron in 70-digit arithmetic (tools/hp.py) and rounded once to double, then cross-checked
against the values as recalled from the public H3 sources (the ``RECALLED_*`` tables below).  Any
disagreement aborts generation.  Known-answer tests in tests/test_oracle_h3.py then pin the
resulting geoToH3 against the published examples (docs/source/api/spatial-indexing.rst:53-58 of
the reference, and the uber/h3 README examples).

Run:  python tools/h3gen.py  -> writes mosaic_amd/csrc/h3_tables.h
"""
import os
import sys

sys.path.insert(0, os.path.dirname(__file__))
import hp  # noqa: E402
from hp import D  # noqa: E402

# --- H3 v3.7 constants.h literals ---------------------------------------------------------------
M_SQRT7 = D("2.6457513110645905905016157536392604257102")
M_SQRT3_2 = D("0.8660254037844386467637231707529361834714")
M_AP7_ROT_RADS = D("0.333473172251832115336090755351601070065900389")
RES0_U_GNOMONIC = D("0.38196601125010500003")

# faceCenterGeo (faceijk.c) -- the defining literals of H3's icosahedron orientation.
FACE_CENTER_GEO = [
    ("0.803582649718989942", "1.248397419617396099"),
    ("1.307747883455638156", "2.536945009877921159"),
    ("1.054751253523952054", "-1.347517358900396623"),
    ("0.600191595538186799", "-0.450603909469755746"),
    ("0.491715428198773866", "0.401988202911306943"),
    ("0.172745327415618701", "1.678146885280433686"),
    ("0.605929321571350690", "2.953923329812411617"),
    ("0.427370518328979641", "-1.888876200336285401"),
    ("-0.079066118549212831", "-0.733429513380867741"),
    ("-0.230961644455383637", "0.506495587332349035"),
    ("0.079066118549212831", "2.408163140208925497"),
    ("0.230961644455383637", "-2.635097066257444203"),
    ("-0.172745327415618701", "-1.463445768309359553"),
    ("-0.605929321571350690", "-0.187669323777381622"),
    ("-0.427370518328979641", "1.252716453253507838"),
    ("-0.600191595538186799", "2.690988744120037492"),
    ("-0.491715428198773866", "-2.739604450678486295"),
    ("-0.803582649718989942", "-1.893195233972397139"),
    ("-1.307747883455638156", "-0.604647643711872080"),
    ("-1.054751253523952054", "1.794075294689396615"),
]

# Recalled faceCenterPoint literals (cross-check only).
RECALLED_FACE_CENTER_POINT = [
    (0.2199307791404606, 0.6583691780274996, 0.7198475378926182),
    (-0.2139234834501421, 0.1478171829550703, 0.9656017935214205),
    (0.1092625278784797, -0.4811951572873210, 0.8697775121287253),
    (0.7428567301586791, -0.3593941678278028, 0.5648005936517033),
    (0.8112534709140969, 0.3448953237639384, 0.4721387736413930),
    (-0.1055498149613921, 0.9794457296411413, 0.1718874610009365),
    (-0.8075407579970092, 0.1533552485898818, 0.5695261994882688),
    (-0.2846148069787907, -0.8644080972654206, 0.4144792552473539),
    (0.7405621473854482, -0.6673299564565524, -0.0789837646326737),
    (0.8512303986474293, 0.4722343788582681, -0.2289137388687808),
    (-0.7405621473854481, 0.6673299564565524, 0.0789837646326737),
    (-0.8512303986474292, -0.4722343788582682, 0.2289137388687808),
    (0.1055498149613919, -0.9794457296411413, -0.1718874610009365),
    (0.8075407579970092, -0.1533552485898819, -0.5695261994882688),
    (0.2846148069787908, 0.8644080972654204, -0.4144792552473539),
    (-0.7428567301586791, 0.3593941678278027, -0.5648005936517033),
    (-0.8112534709140971, -0.3448953237639382, -0.4721387736413930),
    (-0.2199307791404607, -0.6583691780274996, -0.7198475378926182),
    (0.2139234834501420, -0.1478171829550704, -0.9656017935214205),
    (-0.1092625278784796, 0.4811951572873210, -0.8697775121287253),
]

# Recalled faceAxesAzRadsCII[f][0] (i-axis azimuth); used to pick which vertex is the i-axis.
RECALLED_AXIS0 = [
    "5.619958268523939882", "5.760339081714187279", "0.780213654393430055",
    "0.430469363979999913", "6.130269123335111400", "2.692877706530642877",
    "2.982963003477243874", "3.532912002790141181", "3.494305004259568154",
    "3.003214169499538391", "5.930472956509811562", "0.138378484090254847",
    "0.448714947059150361", "0.158629650112549365", "5.891865957979238535",
    "2.711123289609793325", "3.294508837434268316", "3.804819692245439833",
    "3.664438879055192436", "2.361378999196363184",
]

# Recalled baseCellData: (home face, (i, j, k), isPentagon, cwOffsetPent)
RECALLED_BASE_CELL_DATA = [
    (1, (1, 0, 0), 0, (0, 0)), (2, (1, 1, 0), 0, (0, 0)), (1, (0, 0, 0), 0, (0, 0)),
    (2, (1, 0, 0), 0, (0, 0)), (0, (2, 0, 0), 1, (-1, -1)), (1, (1, 1, 0), 0, (0, 0)),
    (1, (0, 0, 1), 0, (0, 0)), (2, (0, 0, 0), 0, (0, 0)), (0, (1, 0, 0), 0, (0, 0)),
    (2, (0, 1, 0), 0, (0, 0)), (1, (0, 1, 0), 0, (0, 0)), (1, (0, 1, 1), 0, (0, 0)),
    (3, (1, 0, 0), 0, (0, 0)), (3, (1, 1, 0), 0, (0, 0)), (11, (2, 0, 0), 1, (2, 6)),
    (4, (1, 0, 0), 0, (0, 0)), (0, (0, 0, 0), 0, (0, 0)), (6, (0, 1, 0), 0, (0, 0)),
    (0, (0, 0, 1), 0, (0, 0)), (2, (0, 1, 1), 0, (0, 0)), (7, (0, 0, 1), 0, (0, 0)),
    (2, (0, 0, 1), 0, (0, 0)), (0, (1, 1, 0), 0, (0, 0)), (6, (0, 0, 1), 0, (0, 0)),
    (10, (2, 0, 0), 1, (1, 5)), (6, (0, 0, 0), 0, (0, 0)), (3, (0, 0, 0), 0, (0, 0)),
    (11, (1, 0, 0), 0, (0, 0)), (4, (1, 1, 0), 0, (0, 0)), (3, (0, 1, 0), 0, (0, 0)),
    (0, (0, 1, 1), 0, (0, 0)), (4, (0, 0, 0), 0, (0, 0)), (5, (0, 1, 0), 0, (0, 0)),
    (0, (0, 1, 0), 0, (0, 0)), (7, (0, 1, 0), 0, (0, 0)), (11, (1, 1, 0), 0, (0, 0)),
    (7, (0, 0, 0), 0, (0, 0)), (10, (1, 0, 0), 0, (0, 0)), (12, (2, 0, 0), 1, (3, 7)),
    (6, (1, 0, 1), 0, (0, 0)), (7, (1, 0, 1), 0, (0, 0)), (4, (0, 0, 1), 0, (0, 0)),
    (3, (0, 0, 1), 0, (0, 0)), (3, (0, 1, 1), 0, (0, 0)), (4, (0, 1, 0), 0, (0, 0)),
    (6, (1, 0, 0), 0, (0, 0)), (11, (0, 0, 0), 0, (0, 0)), (8, (0, 0, 1), 0, (0, 0)),
    (5, (0, 0, 1), 0, (0, 0)), (14, (2, 0, 0), 1, (0, 9)), (5, (0, 0, 0), 0, (0, 0)),
    (12, (1, 0, 0), 0, (0, 0)), (10, (1, 1, 0), 0, (0, 0)), (4, (0, 1, 1), 0, (0, 0)),
    (12, (1, 1, 0), 0, (0, 0)), (7, (1, 0, 0), 0, (0, 0)), (11, (0, 1, 0), 0, (0, 0)),
    (10, (0, 0, 0), 0, (0, 0)), (13, (2, 0, 0), 1, (4, 8)), (10, (0, 0, 1), 0, (0, 0)),
    (11, (0, 0, 1), 0, (0, 0)), (9, (0, 1, 0), 0, (0, 0)), (8, (0, 1, 0), 0, (0, 0)),
    (6, (2, 0, 0), 1, (11, 15)), (8, (0, 0, 0), 0, (0, 0)), (9, (0, 0, 1), 0, (0, 0)),
    (14, (1, 0, 0), 0, (0, 0)), (5, (1, 0, 1), 0, (0, 0)), (16, (0, 1, 1), 0, (0, 0)),
    (8, (1, 0, 1), 0, (0, 0)), (5, (1, 0, 0), 0, (0, 0)), (12, (0, 0, 0), 0, (0, 0)),
    (7, (2, 0, 0), 1, (12, 16)), (12, (0, 1, 0), 0, (0, 0)), (10, (0, 1, 0), 0, (0, 0)),
    (9, (0, 0, 0), 0, (0, 0)), (13, (1, 0, 0), 0, (0, 0)), (16, (0, 0, 1), 0, (0, 0)),
    (15, (0, 1, 1), 0, (0, 0)), (15, (0, 1, 0), 0, (0, 0)), (16, (0, 1, 0), 0, (0, 0)),
    (14, (1, 1, 0), 0, (0, 0)), (13, (1, 1, 0), 0, (0, 0)), (5, (2, 0, 0), 1, (10, 19)),
    (8, (1, 0, 0), 0, (0, 0)), (14, (0, 0, 0), 0, (0, 0)), (9, (1, 0, 1), 0, (0, 0)),
    (14, (0, 0, 1), 0, (0, 0)), (17, (0, 0, 1), 0, (0, 0)), (12, (0, 0, 1), 0, (0, 0)),
    (16, (0, 0, 0), 0, (0, 0)), (17, (0, 1, 1), 0, (0, 0)), (15, (0, 0, 1), 0, (0, 0)),
    (16, (1, 0, 1), 0, (0, 0)), (9, (1, 0, 0), 0, (0, 0)), (15, (0, 0, 0), 0, (0, 0)),
    (13, (0, 0, 0), 0, (0, 0)), (8, (2, 0, 0), 1, (13, 17)), (13, (0, 1, 0), 0, (0, 0)),
    (17, (1, 0, 1), 0, (0, 0)), (19, (0, 1, 0), 0, (0, 0)), (14, (0, 1, 0), 0, (0, 0)),
    (19, (0, 1, 1), 0, (0, 0)), (17, (0, 1, 0), 0, (0, 0)), (13, (0, 0, 1), 0, (0, 0)),
    (17, (0, 0, 0), 0, (0, 0)), (16, (1, 0, 0), 0, (0, 0)), (9, (2, 0, 0), 1, (14, 18)),
    (15, (1, 0, 1), 0, (0, 0)), (15, (1, 0, 0), 0, (0, 0)), (18, (0, 1, 1), 0, (0, 0)),
    (18, (0, 0, 1), 0, (0, 0)), (19, (0, 0, 1), 0, (0, 0)), (17, (1, 0, 0), 0, (0, 0)),
    (19, (0, 0, 0), 0, (0, 0)), (18, (0, 1, 0), 0, (0, 0)), (18, (1, 0, 1), 0, (0, 0)),
    (19, (2, 0, 0), 1, (-1, -1)), (19, (1, 0, 0), 0, (0, 0)), (18, (0, 0, 0), 0, (0, 0)),
    (19, (1, 0, 1), 0, (0, 0)), (18, (1, 0, 0), 0, (0, 0)),
]

# Recalled faceIjkBaseCells for face 0 ([i][j][k] -> (baseCell, ccwRot60)); calibrates the
# rotation-sign convention of the derivation and checks it.
RECALLED_FACE0 = [
    [[(16, 0), (18, 0), (24, 0)], [(33, 0), (30, 0), (32, 3)], [(49, 1), (48, 3), (50, 3)]],
    [[(8, 0), (5, 5), (10, 5)], [(22, 0), (16, 0), (18, 0)], [(41, 1), (33, 0), (30, 0)]],
    [[(4, 0), (0, 5), (2, 5)], [(15, 1), (8, 0), (5, 5)], [(31, 0), (22, 0), (16, 0)]],
]


# --- high-precision vector helpers --------------------------------------------------------------
def vec_from_geo(lat, lng):
    cl = hp.cos(lat)
    return (cl * hp.cos(lng), cl * hp.sin(lng), hp.sin(lat))


def dot(a, b):
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def sub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def add(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def scale(a, s):
    return (a[0] * s, a[1] * s, a[2] * s)


def cross(a, b):
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def norm(a):
    n = dot(a, a).sqrt()
    return (a[0] / n, a[1] / n, a[2] / n)


def geo_of(v):
    return hp.asin(v[2]), hp.atan2(v[1], v[0])


def north_east(lat, lng):
    sl, cl = hp.sin(lat), hp.cos(lat)
    sg, cg = hp.sin(lng), hp.cos(lng)
    n = (-sl * cg, -sl * sg, cl)
    e = (-sg, cg, D(0))
    return n, e


def azimuth(c_lat, c_lng, p):
    """Azimuth (cw from north) of unit vector p seen from (c_lat, c_lng)."""
    n, e = north_east(c_lat, c_lng)
    return hp.atan2(dot(p, e), dot(p, n))


def pos_angle(a):
    two_pi = 2 * hp.pi()
    while a < 0:
        a += two_pi
    while a >= two_pi:
        a -= two_pi
    return a


def hex2d_to_vec(face, x, y, axis0, centers_geo):
    """Inverse gnomonic map of hex2d (x, y) at res 0 on `face` to a unit vector."""
    lat, lng = centers_geo[face]
    c = vec_from_geo(lat, lng)
    r = (x * x + y * y).sqrt()
    if r == 0:
        return c
    theta = hp.atan2(y, x)
    dist = hp.atan(r * RES0_U_GNOMONIC)
    az = pos_angle(axis0[face] - theta)
    n, e = north_east(lat, lng)
    dirv = add(scale(n, hp.cos(az)), scale(e, hp.sin(az)))
    return add(scale(c, hp.cos(dist)), scale(dirv, hp.sin(dist)))


def ijk_to_hex2d(i, j, k):
    ii = D(i - k)
    jj = D(j - k)
    return ii - jj / 2, jj * M_SQRT3_2


def main(out_path):
    centers_geo = [(D(a), D(b)) for a, b in FACE_CENTER_GEO]
    centers = [vec_from_geo(a, b) for a, b in centers_geo]

    # 1. faceCenterPoint: derive and cross-check the recalled literals.
    fcp = []
    for f in range(20):
        dv = tuple(hp.to_double(c) for c in centers[f])
        rec = RECALLED_FACE_CENTER_POINT[f]
        for a, b in zip(dv, rec):
            if abs(a - b) > 2e-16:
                raise SystemExit(f"faceCenterPoint mismatch face {f}: {dv} vs {rec}")
        if dv != rec:
            print(f"note: face {f} faceCenterPoint derived {dv} != recalled literal {rec}; "
                  "using the recalled literal", file=sys.stderr)
        fcp.append(rec)

    # 2. icosahedron: neighbours (3 per face) and vertices (3 per face).
    nbrs = []
    for f in range(20):
        ds = sorted(((dot(centers[f], centers[g]), g) for g in range(20) if g != f), reverse=True)
        nb = [g for _, g in ds[:3]]
        # the 3 nearest are strictly nearer than the 4th
        assert ds[2][0] - ds[3][0] > D("0.1"), (f, ds[:4])
        nbrs.append(nb)
    face_vertices = []
    for f in range(20):
        a, b, c = nbrs[f]
        verts = []
        for n1, n2 in ((a, b), (b, c), (a, c)):
            v = norm(cross(sub(centers[n1], centers[f]), sub(centers[n2], centers[f])))
            if dot(v, centers[f]) < 0:
                v = scale(v, -1)
            verts.append(v)
        face_vertices.append(verts)

    # 3. faceAxesAzRadsCII: azimuth toward the face vertex nearest the recalled i-axis azimuth.
    axes = []
    two_pi_3 = 2 * hp.pi() / 3
    for f in range(20):
        lat, lng = centers_geo[f]
        azs = [pos_angle(azimuth(lat, lng, v)) for v in face_vertices[f]]
        rec = D(RECALLED_AXIS0[f])
        best = min(azs, key=lambda a: min(abs(a - rec), 2 * hp.pi() - abs(a - rec)))
        if abs(best - rec) > D("1e-15"):
            raise SystemExit(f"axis0 mismatch face {f}: derived {best} recalled {rec}")
        a0 = best
        a1 = pos_angle(a0 - two_pi_3)
        a2 = pos_angle(a0 - 2 * two_pi_3)
        # the other two vertices sit at the j and k axes (each 120 degrees cw in azimuth)
        for a in (a1, a2):
            assert min(abs(a - z) for z in azs) < D("1e-12"), (f, a, azs)
        axes.append((a0, a1, a2))
    axis0 = [a[0] for a in axes]
    # also check the rounding of the recalled literal equals the derived double
    for f in range(20):
        if hp.to_double(axis0[f]) != float(RECALLED_AXIS0[f]):
            print(f"note: face {f} axis0 derived double {hp.to_double(axis0[f])!r} "
                  f"!= recalled literal {float(RECALLED_AXIS0[f])!r}; using the recalled literal",
                  file=sys.stderr)

    # 4. res-0 cell centres for every face IJK in {0,1,2}^3.
    def fijk_vec(f, i, j, k):
        x, y = ijk_to_hex2d(i, j, k)
        return hex2d_to_vec(f, x, y, axis0, centers_geo)

    bc_pos = []
    for bc, (face, ijk, pent, cw) in enumerate(RECALLED_BASE_CELL_DATA):
        bc_pos.append(fijk_vec(face, *ijk))
    # distinct positions
    for a in range(122):
        for b in range(a + 1, 122):
            if dot(bc_pos[a], bc_pos[b]) > D("0.999"):
                raise SystemExit(f"base cells {a} and {b} coincide")
    # pentagons sit on icosahedron vertices
    all_vertices = [v for vs in face_vertices for v in vs]
    for bc, (face, ijk, pent, cw) in enumerate(RECALLED_BASE_CELL_DATA):
        on_vertex = any(dot(bc_pos[bc], v) > 1 - D("1e-20") for v in all_vertices)
        if bool(pent) != on_vertex:
            raise SystemExit(f"pentagon flag mismatch for base cell {bc}")
        if pent and cw[0] >= 0:
            for cf in cw:
                faces_at = [g for g in range(20) if any(dot(v, bc_pos[bc]) > 1 - D("1e-20")
                                                        for v in face_vertices[g])]
                if cf not in faces_at or cf == face:
                    raise SystemExit(f"cw offset face {cf} invalid for pentagon {bc}")

    # 5. faceIjkBaseCells with rotations.
    def local_axes(f, i, j, k):
        """Unit tangent of +x (i direction) of face f's res-0 hex2d frame at lattice point ijk."""
        x, y = ijk_to_hex2d(i, j, k)
        eps = D("1e-25")
        p0 = hex2d_to_vec(f, x, y, axis0, centers_geo)
        p1 = hex2d_to_vec(f, x + eps, y, axis0, centers_geo)
        t = sub(p1, p0)
        t = sub(t, scale(p0, dot(t, p0)))
        return p0, norm(t)

    def angle_between(p, t_from, t_to):
        # signed ccw angle (viewed from outside) from t_from to t_to in the tangent plane at p
        s = dot(p, cross(t_from, t_to))
        c = dot(t_from, t_to)
        return hp.atan2(s, c)

    table = [[[[None] * 3 for _ in range(3)] for _ in range(3)] for _ in range(20)]
    sixty = hp.pi() / 3
    for f in range(20):
        for i in range(3):
            for j in range(3):
                for k in range(3):
                    p, t_f = local_axes(f, i, j, k)
                    best = max(range(122), key=lambda b: dot(bc_pos[b], p))
                    if dot(bc_pos[best], p) < D("0.99"):
                        raise SystemExit(f"no base cell near face {f} ijk {(i, j, k)}")
                    hface, hijk, pent, _ = RECALLED_BASE_CELL_DATA[best]
                    if pent:
                        table[f][i][j][k] = (best, None)
                        continue
                    ph, t_h = local_axes(hface, *hijk)
                    ang = angle_between(p, t_f, t_h)
                    m = ang / sixty
                    mr = int(m.to_integral_value())
                    if abs(m - mr) > D("0.35"):
                        raise SystemExit(f"rotation not near a multiple of 60: face {f} {(i, j, k)} {m}")
                    table[f][i][j][k] = (best, mr)

    # calibrate the sign convention against the recalled face-0 table (majority vote)
    votes = {1: 0, -1: 0}
    for i in range(3):
        for j in range(3):
            for k in range(3):
                bc, mr = table[0][i][j][k]
                rbc, rrot = RECALLED_FACE0[i][j][k]
                if bc != rbc:
                    raise SystemExit(f"face0 base cell mismatch at {(i, j, k)}: {bc} vs {rbc}")
                if mr is None or mr % 6 == 0:
                    continue
                for s_ in (1, -1):
                    if (s_ * mr) % 6 == rrot:
                        votes[s_] += 1
    sign = 1 if votes[1] > votes[-1] else -1
    final = [[[[None] * 3 for _ in range(3)] for _ in range(3)] for _ in range(20)]
    for f in range(20):
        for i in range(3):
            for j in range(3):
                for k in range(3):
                    bc, mr = table[f][i][j][k]
                    final[f][i][j][k] = (bc, None if mr is None else (sign * mr) % 6)
    bad = []
    for i in range(3):
        for j in range(3):
            for k in range(3):
                if final[0][i][j][k][1] is None:
                    continue
                if final[0][i][j][k] != RECALLED_FACE0[i][j][k]:
                    bad.append(((i, j, k), final[0][i][j][k], RECALLED_FACE0[i][j][k]))
    if bad:
        print("note: face0 rotation disagreements (derived, recalled):", bad, file=sys.stderr)
        if len(bad) > 1:
            raise SystemExit(1)

    # Pentagon base cells.  Frames of the five faces around an icosahedron vertex do not close
    # (60-degree deficit), so the face->home rotation depends on the path taken around the vertex.
    # Adjacent-face rotations come from the shared edge cells (hexagons, derived above); the path is
    # the clockwise one from the home face for the ten non-polar pentagons (this reproduces the
    # recalled face-0 entries for base cells 24 and 49) and the counter-clockwise one for the polar
    # pentagons 4 and 117 (cwOffsetPent = -1).  Unpinned beyond those entries: see DESIGN.md.
    edge_ijk = [(1, 1, 0), (1, 0, 1), (0, 1, 1)]
    vert_ijk = [(2, 0, 0), (0, 2, 0), (0, 0, 2)]

    def rot_between(fa, fb):
        # rotation taking frame fa to frame fb, via their shared edge cell
        for ea in edge_ijk:
            bca, ra = final[fa][ea[0]][ea[1]][ea[2]]
            for eb in edge_ijk:
                bcb, rb = final[fb][eb[0]][eb[1]][eb[2]]
                if bca == bcb:
                    return (ra - rb) % 6
        raise SystemExit(f"faces {fa} and {fb} share no edge cell")

    for bc, (hface, hijk, pent, cw) in enumerate(RECALLED_BASE_CELL_DATA):
        if not pent:
            continue
        p = bc_pos[bc]
        around = [f for f in range(20) for v in vert_ijk if final[f][v[0]][v[1]][v[2]][0] == bc]
        assert len(around) == 5 and hface in around, (bc, around)
        plat, plng = hp.asin(p[2]), hp.atan2(p[1], p[0])
        n_, e_ = north_east(plat, plng)
        order = sorted(around, key=lambda f: -hp.atan2(dot(centers[f], e_), dot(centers[f], n_)))
        step = 1 if cw[0] < 0 else -1
        i0 = order.index(hface)
        for f in around:
            r = 0
            cur, idx = hface, i0
            if cw[0] >= 0 and order[(i0 - step) % 5] == f:
                # the face next to the home face across the pentagon's deleted k sector: its frame
                # is one edge crossing from the home face's, not four around the vertex (fixed by
                # H3's round trip geoToH3(h3ToGeo(h)) == h over every cell of the base cell,
                # tools/probes/pent_rot_probe.cpp; the four-step path overshoots by the vertex's
                # 60-degree deficit)
                r = rot_between(f, hface)
                cur = f
            while cur != f:
                idx = (idx + step) % 5
                nxt = order[idx]
                r = (r + rot_between(nxt, cur)) % 6
                cur = nxt
            for i in range(3):
                for j in range(3):
                    for k in range(3):
                        if final[f][i][j][k][0] == bc:
                            final[f][i][j][k] = (bc, r)
    for i in range(3):
        for j in range(3):
            for k in range(3):
                if final[0][i][j][k] != RECALLED_FACE0[i][j][k]:
                    print("note: face0 entry", (i, j, k), final[0][i][j][k], "recalled",
                          RECALLED_FACE0[i][j][k], file=sys.stderr)
    assert final[0][0][2][0] == (49, 1) and final[0][0][0][2] == (24, 0)
    for f in range(20):
        for i in range(3):
            for j in range(3):
                for k in range(3):
                    assert final[f][i][j][k][1] is not None

    # every base cell's home FaceIJK maps to itself with zero rotation
    for bc, (face, ijk, pent, cw) in enumerate(RECALLED_BASE_CELL_DATA):
        got = final[face][ijk[0]][ijk[1]][ijk[2]]
        assert got[0] == bc and got[1] in (0, None), (bc, got)

    # base cells are numbered in order of decreasing latitude of their centres
    lats = [hp.asin(p[2]) for p in bc_pos]
    assert all(lats[b] > lats[b + 1] for b in range(121)), "base cell latitude order violated"

    axes = [(D(RECALLED_AXIS0[f]), a[1], a[2]) for f, a in enumerate(axes)]
    write_header(out_path, centers_geo, fcp, axes, final)
    print(f"wrote {out_path}")


def fmt(x):
    return repr(hp.to_double(x))


def write_header(path, centers_geo, fcp, axes, final):
    L = []
    L.append("/* Generated by tools/h3gen.py -- do not edit.")
    L.append(" * H3 v3.7 constant tables for geoToH3 (face centres, face axes, base cells).")
    L.append(" * faceCenterGeo are H3's published literals; the rest is derived from them in 70-digit")
    L.append(" * arithmetic, rounded once to double, and cross-checked against recalled H3 literals.")
    L.append(" * Include after defining H3_TABLE (storage qualifier, e.g. `static const`). */")
    L.append("#ifndef MOSAIC_H3_TABLES_H")
    L.append("#define MOSAIC_H3_TABLES_H")
    L.append("#ifndef H3_TABLE")
    L.append("#define H3_TABLE static const")
    L.append("#endif")
    L.append("H3_TABLE double kH3FaceCenterGeo[20][2] = {")
    for lat, lng in centers_geo:
        L.append(f"    {{{fmt(lat)}, {fmt(lng)}}},")
    L.append("};")
    L.append("H3_TABLE double kH3FaceCenterPoint[20][3] = {")
    for v in fcp:
        L.append(f"    {{{v[0]!r}, {v[1]!r}, {v[2]!r}}},")
    L.append("};")
    L.append("H3_TABLE double kH3FaceAxesAzRadsCII[20][3] = {")
    for a in axes:
        L.append(f"    {{{fmt(a[0])}, {fmt(a[1])}, {fmt(a[2])}}},")
    L.append("};")
    L.append("/* baseCellData: home face, home i, j, k, isPentagon, cwOffsetPent[2] */")
    L.append("H3_TABLE int kH3BaseCellData[122][7] = {")
    for face, ijk, pent, cw in RECALLED_BASE_CELL_DATA:
        L.append(f"    {{{face}, {ijk[0]}, {ijk[1]}, {ijk[2]}, {pent}, {cw[0]}, {cw[1]}}},")
    L.append("};")
    L.append("/* faceIjkBaseCells packed as (baseCell << 3) | ccwRot60, indexed [face][i][j][k] */")
    L.append("H3_TABLE unsigned short kH3FaceIjkBaseCells[20][3][3][3] = {")
    for f in range(20):
        rows = []
        for i in range(3):
            js = []
            for j in range(3):
                ks = ", ".join(str((final[f][i][j][k][0] << 3) | final[f][i][j][k][1]) for k in range(3))
                js.append("{" + ks + "}")
            rows.append("{" + ", ".join(js) + "}")
        L.append("    {" + ", ".join(rows) + "},")
    L.append("};")
    L.append("#endif")
    with open(path, "w") as fh:
        fh.write("\n".join(L) + "\n")


# --- x87 extended-precision constants (used by the exact device path) -----------------------------
LD_CONSTANTS = {
    "M_2PI": "6.28318530717958647692528676655900576839433",
    "M_SQRT7": "2.6457513110645905905016157536392604257102",
    "M_SIN60": "0.8660254037844386467637231707529361834714",
    "M_AP7_ROT_RADS": "0.333473172251832115336090755351601070065900389",
    "EPSILON": "0.0000000000000001",
}


def ld_round(text):
    """Round a decimal literal to x87 double-extended (64-bit significand, RNE) exactly as gcc does
    for an L-suffixed literal.  Returns (m64, e) with value = m64 * 2**e, 2**63 <= m64 < 2**64."""
    from fractions import Fraction
    v = Fraction(text)
    e = 0
    while v * Fraction(2) ** (-e) >= 2 ** 64:
        e += 1
    while v * Fraction(2) ** (-e) < 2 ** 63:
        e -= 1
    q = v * Fraction(2) ** (-e)
    m = q.numerator // q.denominator
    rem = q - m
    if rem > Fraction(1, 2) or (rem == Fraction(1, 2) and m % 2 == 1):
        m += 1
    if m == 2 ** 64:
        m //= 2
        e += 1
    return m, e


def double_up(m, e):
    """Smallest double >= m * 2**e."""
    import math
    from fractions import Fraction
    v = Fraction(m) * Fraction(2) ** e
    d = float(v)
    if Fraction(d) < v:
        d = math.nextafter(d, math.inf)
    return d


def write_ld_header(path):
    L = ["/* Generated by tools/h3gen.py -- do not edit.",
         " * H3 v3.7 long-double (L-suffixed) constants as x87 double-extended values:",
         " * value = m * 2^e with a 64-bit significand m (bit 63 set), rounded RNE from the literal",
         " * exactly as gcc does on x86-64.  *_DUP is the smallest double >= the value. */",
         "#ifndef MOSAIC_H3_LD_CONSTANTS_H", "#define MOSAIC_H3_LD_CONSTANTS_H"]
    for name, text in LD_CONSTANTS.items():
        m, e = ld_round(text)
        L.append(f"#define H3LD_{name}_M 0x{m:016x}ULL")
        L.append(f"#define H3LD_{name}_E ({e})")
        L.append(f"#define H3LD_{name}_DUP {double_up(m, e)!r}")
    L.append("#endif")
    with open(path, "w") as fh:
        fh.write("\n".join(L) + "\n")



# --- fast projective path tables ------------------------------------------------------------------
def write_fast_header(path):
    """Per-face gnomonic basis for the fast point->hex2d path (h3_device.h):
    x = SCALE[res] * (EI . p) / (FC . p),  y = SCALE[res] * (EP . p) / (FC . p)
    where FC is the unit face centre, EI the unit tangent along the face's Class II i-axis
    (azimuth faceAxesAzRadsCII[f][0]) and EP that rotated 90 degrees counter-clockwise; the Class III
    (odd resolution) pair is the same basis rotated by -M_AP7_ROT_RADS.  This is geoToH3's
    acos/azimuth/tan chain written as the projective map it is mathematically."""
    cg = [(D(a), D(b)) for a, b in FACE_CENTER_GEO]
    rot = M_AP7_ROT_RADS
    cr, sr = hp.cos(rot), hp.sin(rot)
    rows = []
    for f in range(20):
        lat, lng = cg[f]
        c = vec_from_geo(lat, lng)
        n_, e_ = north_east(lat, lng)
        az = D(RECALLED_AXIS0[f])
        ca, sa = hp.cos(az), hp.sin(az)
        ei2 = add(scale(n_, ca), scale(e_, sa))
        ep2 = sub(scale(n_, sa), scale(e_, ca))
        ei3 = add(scale(ei2, cr), scale(ep2, sr))
        ep3 = sub(scale(ep2, cr), scale(ei2, sr))
        rows.append((c, ei2, ep2, ei3, ep3))
    L = ["/* Generated by tools/h3gen.py -- do not edit.  Fast projective geoToH3 tables. */",
         "#ifndef MOSAIC_H3_FAST_TABLES_H", "#define MOSAIC_H3_FAST_TABLES_H",
         "#ifndef H3_TABLE", "#define H3_TABLE static const", "#endif",
         "/* per face: FC[3], EI2[3], EP2[3], EI3[3], EP3[3] */",
         "H3_TABLE double kH3FastBasis[20][15] = {"]
    for r in rows:
        vals = [hp.to_double(v) for vec in r for v in vec]
        L.append("    {" + ", ".join(repr(v) for v in vals) + "},")
    L.append("};")
    # sin / cos of k / 64 for k in [-201, 201] (covers |x| <= pi), correctly rounded
    L.append("/* kH3SinCos64[k + 201] = {sin(k/64), cos(k/64)}, correctly rounded */")
    L.append("H3_TABLE double kH3SinCos64[403][2] = {")
    for k in range(-201, 202):
        a = D(k) / 64
        L.append(f"    {{{hp.to_double(hp.sin(a))!r}, {hp.to_double(hp.cos(a))!r}}},")
    L.append("};")
    L.append("/* SCALE[res] = sqrt(7)^res / RES0_U_GNOMONIC */")
    L.append("H3_TABLE double kH3FastScale[16] = {")
    sq7 = D(7).sqrt()
    L.append("    " + ", ".join(repr(hp.to_double(sq7 ** r / RES0_U_GNOMONIC)) for r in range(16)))
    L.append("};")
    L.append("#endif")
    with open(path, "w") as fh:
        fh.write("\n".join(L) + "\n")


def write_face_lut(path):
    """1-degree lat/lng cells whose every point has the same closest icosahedron face with a
    dot-product gap of at least 3e-3 (checked on an 11 x 11 sample grid; the gap changes by at most
    2 * 1.3e-3 between samples, |grad| <= |c_f - c_g| <= 2): face id, else 255 (full search)."""
    import numpy as np
    cg = [(float(a), float(b)) for a, b in FACE_CENTER_GEO]
    C = np.array([[np.cos(a) * np.cos(b), np.cos(a) * np.sin(b), np.sin(a)] for a, b in cg])
    lut = np.full((180, 360), 255, np.uint8)
    t = np.linspace(0.0, 1.0, 11)
    for i in range(180):
        lat = np.radians(-90.0 + i + t)
        for j in range(360):
            lon = np.radians(-180.0 + j + t)
            LA, LO = np.meshgrid(lat, lon, indexing="ij")
            P = np.stack([np.cos(LA) * np.cos(LO), np.cos(LA) * np.sin(LO), np.sin(LA)], -1).reshape(-1, 3)
            d = P @ C.T
            o = np.sort(d, axis=1)
            best = np.argmax(d, axis=1)
            if np.all(best == best[0]) and np.min(o[:, -1] - o[:, -2]) > 3e-3:
                lut[i, j] = best[0]
    L = ["/* Generated by tools/h3gen.py -- do not edit.  Closest-face lookup on 1-degree cells:",
         " * kH3FaceLut[floor(lat + 90)][floor(lng + 180)] = face, or 255 near face boundaries. */",
         "#ifndef MOSAIC_H3_FACE_LUT_H", "#define MOSAIC_H3_FACE_LUT_H",
         "#ifndef H3_LUT", "#define H3_LUT static const", "#endif",
         "H3_LUT unsigned char kH3FaceLut[180][360] = {"]
    for i in range(180):
        L.append("    {" + ",".join(str(int(v)) for v in lut[i]) + "},")
    L.append("};")
    L.append("#endif")
    with open(path, "w") as fh:
        fh.write("\n".join(L) + "\n")
    print("face lut: pure cells", int((lut != 255).sum()), "of", lut.size)


if __name__ == "__main__":
    here = os.path.dirname(os.path.abspath(__file__))
    out = os.path.join(here, "..", "mosaic_amd", "csrc", "h3_tables.h")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    main(os.path.normpath(out))
    write_ld_header(os.path.normpath(os.path.join(here, "..", "mosaic_amd", "csrc", "h3_ld_constants.h")))
    write_fast_header(os.path.normpath(os.path.join(here, "..", "mosaic_amd", "csrc", "h3_fast_tables.h")))
    write_face_lut(os.path.normpath(os.path.join(here, "..", "mosaic_amd", "csrc", "h3_face_lut.h")))
