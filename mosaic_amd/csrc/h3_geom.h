// H3 cell geometry on the device and the host: h3ToGeo (cell centre) and h3ToGeoBoundary, as the
// reference reaches them (H3IndexSystem.indexToGeometry -> h3.h3ToGeoBoundary,
// core/index/H3IndexSystem.scala:93-100; getBufferRadius :73-80; polyfill's cell centres :113-126).
//
// H3 C v3.7 restated with x86-64 semantics, as h3_device.h does for geoToH3: the long-double steps
// (M_SQRT7, M_SQRT3_2, M_AP7_ROT_RADS, M_2PI, EPSILON) through the exact x87 emulation (x87.h),
// `float t` in _v2dIntersect, and glibc 2.35's sincos / atan2 / atan / asin restated bit for bit
// (glibc_math.h; gcc fuses H3's sin / cos pairs into sincos, as the oracle's object code shows).
// Face adjacency: h3_face_tables.h (tools/h3gen_faces.py).  Oracle: oracle/h3.c
// (oracle_h3_to_geo, oracle_h3_to_geo_boundary) with real long double and the host glibc.
#pragma once
#include <stdint.h>

#include "glibc_math.h"
#include "h3_grid.h"
#include "x87.h"

namespace mosaic {
namespace h3geom {

using h3::IJK;

struct FaceIJK {
    int face;
    IJK c;
};

MOSAIC_HD double ld_sqrt3_2_times(double v) { return x87::mul_ld(v, H3LD_M_SIN60_M, H3LD_M_SIN60_E); }

// coordijk.c _ijkToHex2d
MOSAIC_HD void ijk_to_hex2d(IJK c, double* x, double* y) {
    const int i = c.i - c.k, j = c.j - c.k;
    *x = i - 0.5 * j;
    *y = ld_sqrt3_2_times((double)j);
}

// geoCoord.c constrainLng
MOSAIC_HD double constrain_lng(double lng) {
    const double pi = 3.14159265358979323846;
    while (lng > pi) lng = lng - (2 * pi);
    while (lng < -pi) lng = lng + (2 * pi);
    return lng;
}

// geoCoord.c _geoAzDistanceRads
MOSAIC_HD void geo_az_distance_rads(double lat1, double lon1, double az, double distance, double* lat2, double* lon2) {
    const double eps = H3LD_EPSILON_DUP;  // x < EPSILON (long double) <=> x < eps
    const double pi = 3.14159265358979323846, pi_2 = 1.57079632679489661923;
    if (distance < eps) {
        *lat2 = lat1;
        *lon2 = lon1;
        return;
    }
    az = h3::pos_angle_rads(az);
    if (az < eps || fabs(az - pi) < eps) {
        *lat2 = az < eps ? lat1 + distance : lat1 - distance;
        if (fabs(*lat2 - pi_2) < eps) {
            *lat2 = pi_2;
            *lon2 = 0.0;
        } else if (fabs(*lat2 + pi_2) < eps) {
            *lat2 = -pi_2;
            *lon2 = 0.0;
        } else {
            *lon2 = constrain_lng(lon1);
        }
        return;
    }
    double s1, c1, sd, cd, sa, ca;
    glibc::sincos(lat1, &s1, &c1);
    glibc::sincos(distance, &sd, &cd);
    glibc::sincos(az, &sa, &ca);
    double sinlat = s1 * cd + c1 * sd * ca;
    if (sinlat > 1.0) sinlat = 1.0;
    if (sinlat < -1.0) sinlat = -1.0;
    *lat2 = glibc::asin(sinlat);
    if (fabs(*lat2 - pi_2) < eps) {
        *lat2 = pi_2;
        *lon2 = 0.0;
    } else if (fabs(*lat2 + pi_2) < eps) {
        *lat2 = -pi_2;
        *lon2 = 0.0;
    } else {
        double s2, c2;
        glibc::sincos(*lat2, &s2, &c2);
        double sinlon = sa * sd / c2;
        double coslon = (cd - s1 * s2) / c1 / c2;
        if (sinlon > 1.0) sinlon = 1.0;
        if (sinlon < -1.0) sinlon = -1.0;
        if (coslon > 1.0) coslon = 1.0;
        if (coslon < -1.0) coslon = -1.0;
        *lon2 = constrain_lng(lon1 + glibc::atan2(sinlon, coslon));
    }
}

// faceijk.c _hex2dToGeo (radians)
MOSAIC_HD void hex2d_to_geo(double vx, double vy, int face, int res, bool substrate, double* lat, double* lon) {
    double r = sqrt(vx * vx + vy * vy);
    if (r < H3LD_EPSILON_DUP) {
        *lat = h3::kH3FaceCenterGeo[face][0];
        *lon = h3::kH3FaceCenterGeo[face][1];
        return;
    }
    double theta = glibc::atan2(vy, vx);
    for (int i = 0; i < res; i++) r = x87::div_ld(r, H3LD_M_SQRT7_M, H3LD_M_SQRT7_E);
    if (substrate) {
        r /= 3.0;
        if (res & 1) r = x87::div_ld(r, H3LD_M_SQRT7_M, H3LD_M_SQRT7_E);
    }
    r *= h3::kRes0UGnomonic;
    r = glibc::atan(r);
    if (!substrate && (res & 1))
        theta = h3::pos_angle_rads(x87::add_ld(theta, H3LD_M_AP7_ROT_RADS_M, H3LD_M_AP7_ROT_RADS_E, false));
    theta = h3::pos_angle_rads(h3::kH3FaceAxesAzRadsCII[face][0] - theta);
    geo_az_distance_rads(h3::kH3FaceCenterGeo[face][0], h3::kH3FaceCenterGeo[face][1], theta, r, lat, lon);
}

// coordijk.c _ijkRotate60cw
MOSAIC_HD void rotate60cw(IJK& c) {
    IJK r{c.i + c.j, c.j + c.k, c.i + c.k};
    h3::ijk_normalize(r);
    c = r;
}

// faceijk.c _adjustOverageClassII: 0 NO_OVERAGE, 1 FACE_EDGE, 2 NEW_FACE
MOSAIC_HD int adjust_overage(FaceIJK& f, int res, bool pent_leading4, bool substrate) {
    IJK& ijk = f.c;
    int max_dim = h3grid::max_dim_c2(res);
    if (substrate) max_dim *= 3;
    const int sum = ijk.i + ijk.j + ijk.k;
    if (substrate && sum == max_dim) return 1;
    if (sum <= max_dim) return 0;
    int q;
    if (ijk.k > 0) {
        if (ijk.j > 0) {
            q = 3;
        } else {
            q = 2;
            if (pent_leading4) {
                IJK t{ijk.i - max_dim, ijk.j, ijk.k};
                rotate60cw(t);
                ijk = IJK{t.i + max_dim, t.j, t.k};
            }
        }
    } else {
        q = 1;
    }
    const int* o = h3grid::kH3FaceNeighbors[f.face][q];
    f.face = o[0];
    for (int r = 0; r < o[4]; r++) h3grid::rotate60ccw(ijk);
    int s = h3grid::unit_scale_c2(res);
    if (substrate) s *= 3;
    ijk = h3grid::add(ijk, IJK{o[1] * s, o[2] * s, o[3] * s});
    h3::ijk_normalize(ijk);
    return (substrate && ijk.i + ijk.j + ijk.k == max_dim) ? 1 : 2;
}

MOSAIC_HD int res_of(uint64_t h) { return (int)((h >> 52) & 15); }
MOSAIC_HD int base_cell_of(uint64_t h) { return (int)((h >> 45) & 127); }

// h3Index.c _h3ToFaceIjk; false for ids that are not valid cells
MOSAIC_HD bool h3_to_faceijk(uint64_t h, FaceIJK* f) {
    if (((h >> 59) & 15) != 1) return false;
    const int res = res_of(h), bc = base_cell_of(h);
    if (bc >= 122) return false;
    // digits 1 .. res must not be 7: bit tests, no loop exit (a bool decided inside a divergent loop
    // and read after it is what gfx950 code got wrong in round 4: h3_device.h leading_nonzero_digit)
    const uint64_t low = 0x1249249249249ULL, D = h & 0x1fffffffffffULL;
    const uint64_t used = low & ~((1ULL << (3 * (15 - res))) - 1ULL);  // digit groups 1 .. res
    if (D & (D >> 1) & (D >> 2) & used) return false;
    const bool pent = h3::kH3BaseCellData[bc][4] != 0;
    if (pent && h3::leading_nonzero_digit(h, res) == 5) h = h3::rotate_all(h, res, false);
    f->face = h3::kH3BaseCellData[bc][0];
    f->c = IJK{h3::kH3BaseCellData[bc][1], h3::kH3BaseCellData[bc][2], h3::kH3BaseCellData[bc][3]};
    const bool possible = !(!pent && (res == 0 || (f->c.i == 0 && f->c.j == 0 && f->c.k == 0)));
    for (int q = 1; q <= res; q++) {
        if (q & 1) h3grid::down_ap7(f->c);
        else h3grid::down_ap7r(f->c);
        const int d = h3::get_digit(h, q);
        if (d) {
            f->c = h3grid::add(f->c, h3grid::unit(d));
            h3::ijk_normalize(f->c);
        }
    }
    if (!possible) return true;
    const IJK orig = f->c;
    int r2 = res;
    if (res & 1) {
        h3grid::down_ap7r(f->c);
        r2++;
    }
    const bool pent4 = pent && h3::leading_nonzero_digit(h, res) == 4;
    if (adjust_overage(*f, r2, pent4, false)) {
        if (pent)
            for (int it = 0; it < 8 && adjust_overage(*f, r2, false, false); it++) {
            }
        if (r2 != res) h3grid::up_ap7r(f->c);
    } else if (r2 != res) {
        f->c = orig;
    }
    return true;
}

// h3ToGeo: the cell centre in radians; false for invalid ids
MOSAIC_HD bool h3_to_geo(uint64_t h, double* lat, double* lon) {
    FaceIJK f;
    if (!h3_to_faceijk(h, &f)) return false;
    double x, y;
    ijk_to_hex2d(f.c, &x, &y);
    hex2d_to_geo(x, y, f.face, res_of(h), false, lat, lon);
    return true;
}

// coordijk.c _downAp3 / _downAp3r
MOSAIC_HD void down_ap3(IJK& c) {
    IJK r{2 * c.i + c.j, 2 * c.j + c.k, c.i + 2 * c.k};
    h3::ijk_normalize(r);
    c = r;
}
MOSAIC_HD void down_ap3r(IJK& c) {
    IJK r{2 * c.i + c.k, c.i + 2 * c.j, c.j + 2 * c.k};
    h3::ijk_normalize(r);
    c = r;
}

// vec2d.c _v2dIntersect (H3 v3.7 declares t as float)
MOSAIC_HD void v2d_intersect(double p0x, double p0y, double p1x, double p1y, double p2x, double p2y, double p3x,
                             double p3y, double* ix, double* iy) {
    const double s1x = p1x - p0x, s1y = p1y - p0y, s2x = p3x - p2x, s2y = p3y - p2y;
    const float t = (float)((s2x * (p0y - p2y) - s2y * (p0x - p2x)) / (-s2x * s1y + s1x * s2y));
    *ix = p0x + ((double)t * s1x);
    *iy = p0y + ((double)t * s1y);
}

// the icosahedron face edge in quadrant dir (1 IJ, 2 KI, 3 JK) at Class II substrate scale max_dim
MOSAIC_HD void face_edge(int dir, int max_dim, double e[4]) {
    // 3.0 * M_SQRT3_2 * maxDim, evaluated in long double and rounded once
    const double h = x87::to_double(x87::mul(x87::mul(x87::from_double(3.0), x87::make(H3LD_M_SIN60_M, H3LD_M_SIN60_E)),
                                             x87::from_double((double)max_dim)));
    const double v0x = 3.0 * max_dim, v0y = 0.0, v1x = -1.5 * max_dim, v1y = h, v2x = -1.5 * max_dim, v2y = -h;
    if (dir == 1) {
        e[0] = v0x, e[1] = v0y, e[2] = v1x, e[3] = v1y;
    } else if (dir == 3) {
        e[0] = v1x, e[1] = v1y, e[2] = v2x, e[3] = v2y;
    } else {
        e[0] = v2x, e[1] = v2y, e[2] = v0x, e[3] = v0y;
    }
}

// h3ToGeoBoundary: vertices (lat, lng radians) into out[2 n], n <= 10; -1 for invalid ids
MOSAIC_HD int h3_to_geo_boundary(uint64_t h, double* out) {
    FaceIJK center;
    if (!h3_to_faceijk(h, &center)) return -1;
    const int res = res_of(h);
    const bool pent = h3::kH3BaseCellData[base_cell_of(h)][4] && h3::leading_nonzero_digit(h, res) == 0;
    const int nv = pent ? 5 : 6;
    const int cII[6][3] = {{2, 1, 0}, {1, 2, 0}, {0, 2, 1}, {0, 1, 2}, {1, 0, 2}, {2, 0, 1}};
    const int cIII[6][3] = {{5, 4, 0}, {1, 5, 0}, {0, 5, 4}, {0, 1, 5}, {4, 0, 5}, {5, 0, 1}};
    int adj = res;
    FaceIJK c = center;
    down_ap3(c.c);
    down_ap3r(c.c);
    if (res & 1) {
        h3grid::down_ap7r(c.c);
        adj++;
    }
    FaceIJK fv[6];
    for (int v = 0; v < nv; v++) {
        const int* d = (res & 1) ? cIII[v] : cII[v];
        fv[v].face = c.face;
        fv[v].c = IJK{c.c.i + d[0], c.c.j + d[1], c.c.k + d[2]};
        h3::ijk_normalize(fv[v].c);
    }
    const int max_dim = h3grid::max_dim_c2(adj);
    int n = 0;
    if (!pent) {
        int last_face = -1, last_overage = 0;
        for (int vert = 0; vert < 7; vert++) {
            const int v = vert % 6;
            FaceIJK f = fv[v];
            const int overage = adjust_overage(f, adj, false, true);
            if ((res & 1) && vert > 0 && f.face != last_face && last_overage != 1) {
                const int lv = (v + 5) % 6;
                double o0x, o0y, o1x, o1y, e[4], ix, iy;
                ijk_to_hex2d(fv[lv].c, &o0x, &o0y);
                ijk_to_hex2d(fv[v].c, &o1x, &o1y);
                const int face2 = (last_face == center.face) ? f.face : last_face;
                face_edge(h3grid::kH3AdjacentFaceDir[center.face][face2], max_dim, e);
                v2d_intersect(o0x, o0y, o1x, o1y, e[0], e[1], e[2], e[3], &ix, &iy);
                if (!((o0x == ix && o0y == iy) || (o1x == ix && o1y == iy))) {
                    hex2d_to_geo(ix, iy, center.face, adj, true, &out[2 * n], &out[2 * n + 1]);
                    n++;
                }
            }
            if (vert < 6) {
                double vx, vy;
                ijk_to_hex2d(f.c, &vx, &vy);
                hex2d_to_geo(vx, vy, f.face, adj, true, &out[2 * n], &out[2 * n + 1]);
                n++;
            }
            last_face = f.face;
            last_overage = overage;
        }
    } else {
        FaceIJK last = fv[0];
        for (int vert = 0; vert < 6; vert++) {
            const int v = vert % 5;
            FaceIJK f = fv[v];
            for (int it = 0; it < 8 && adjust_overage(f, adj, false, true) == 2; it++) {
            }
            if ((res & 1) && vert > 0) {
                FaceIJK t = f;
                double o0x, o0y, o1x, o1y, e[4], ix, iy;
                ijk_to_hex2d(last.c, &o0x, &o0y);
                const int dir = h3grid::kH3AdjacentFaceDir[t.face][last.face];
                const int* o = h3grid::kH3FaceNeighbors[t.face][dir];
                t.face = o[0];
                for (int r = 0; r < o[4]; r++) h3grid::rotate60ccw(t.c);
                const int s = h3grid::unit_scale_c2(adj) * 3;
                t.c = h3grid::add(t.c, IJK{o[1] * s, o[2] * s, o[3] * s});
                h3::ijk_normalize(t.c);
                ijk_to_hex2d(t.c, &o1x, &o1y);
                face_edge(h3grid::kH3AdjacentFaceDir[t.face][f.face], max_dim, e);
                v2d_intersect(o0x, o0y, o1x, o1y, e[0], e[1], e[2], e[3], &ix, &iy);
                hex2d_to_geo(ix, iy, t.face, adj, true, &out[2 * n], &out[2 * n + 1]);
                n++;
            }
            if (vert < 5) {
                double vx, vy;
                ijk_to_hex2d(f.c, &vx, &vy);
                hex2d_to_geo(vx, vy, f.face, adj, true, &out[2 * n], &out[2 * n + 1]);
                n++;
            }
            last = f;
        }
    }
    return n;
}

// java.lang.Math.toDegrees (h3-java converts the C library's radians): JDK 8 rad * 180.0 / PI,
// JDK 9+ rad * RADIANS_TO_DEGREES
MOSAIC_HD double to_degrees(double rad, int jdk) {
    return jdk <= 8 ? rad * 180.0 / 3.141592653589793 : rad * 57.29577951308232;
}

}  // namespace h3geom
}  // namespace mosaic
