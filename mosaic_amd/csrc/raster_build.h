// Geometry of the point-raster classification (tiles.h, tiles_build.cpp), shared by the host
// builder (g++) and the device builder (k_raster_* in mosaic_hip.hip): the same operations on the
// same inputs, so both builders produce the same raster bit for bit (-ffp-contract=off on both
// sides; IEEE division and sqrt).  The hexagon extents' cos / sin values come from a table the host
// fills once with its libm (HexTable) and hands to the device.
#pragma once
#include <math.h>
#include <stdint.h>

#if !defined(MOSAIC_HD)
#if defined(__HIPCC__)
#define MOSAIC_HD __host__ __device__ inline
#else
#define MOSAIC_HD inline
#endif
#endif

namespace mosaic {
namespace rbuild {

static const double kS60 = 0.86602540378443864676;

struct P2 {
    double x, y;
};

MOSAIC_HD double dmin(double a, double b) { return b < a ? b : a; }  // std::min
MOSAIC_HD double dmax(double a, double b) { return a < b ? b : a; }  // std::max

// cos / sin of the hexagon vertex directions 30 + 60 k degrees (host libm)
struct HexTable {
    double c[6], s[6];
};
inline HexTable hex_table() {
    HexTable t;
    for (int k = 0; k < 6; k++) {
        const double ang = (30.0 + 60.0 * k) * 0.017453292519943295;
        t.c[k] = cos(ang);
        t.s[k] = sin(ang);
    }
    return t;
}

// Convex polygon q[n] (counter-clockwise) meets the Voronoi hexagon of lattice centre c within
// tolerance t (separating axes: the hexagon's 3 edge normals and the polygon's n).
MOSAIC_HD bool poly_meets_hex(const P2* q, int n, P2 c, double t, const HexTable& ht) {
    // hexagon: vertices at 30 + 60k degrees, radius 1/sqrt(3); apothem 1/2 along 0, 60, 120 degrees
    const double ax[3][2] = {{1.0, 0.0}, {0.5, kS60}, {-0.5, kS60}};
    for (int k = 0; k < 3; k++) {
        const double hc = c.x * ax[k][0] + c.y * ax[k][1];
        double lo = INFINITY, hi = -INFINITY;
        for (int v = 0; v < n; v++) {
            const double d = q[v].x * ax[k][0] + q[v].y * ax[k][1];
            lo = dmin(lo, d);
            hi = dmax(hi, d);
        }
        if (lo > hc + 0.5 + t || hi < hc - 0.5 - t) return false;
    }
    const double r = 0.57735026918962576451;
    for (int e = 0; e < n; e++) {
        const P2 a = q[e], b = q[(e + 1) % n];
        double nx = -(b.y - a.y), ny = b.x - a.x;
        const double len = sqrt(nx * nx + ny * ny);
        if (!(len > 0)) continue;
        nx /= len;
        ny /= len;
        double lo = INFINITY, hi = -INFINITY;
        for (int v = 0; v < n; v++) {
            const double d = q[v].x * nx + q[v].y * ny;
            lo = dmin(lo, d);
            hi = dmax(hi, d);
        }
        const double hc = c.x * nx + c.y * ny;
        double ext = 0.0;
        for (int k = 0; k < 6; k++) ext = dmax(ext, fabs(r * (ht.c[k] * nx + ht.s[k] * ny)));
        if (lo > hc + ext + t || hi < hc - ext - t) return false;
    }
    return true;
}

MOSAIC_HD double cross(P2 o, P2 a, P2 b) { return (a.x - o.x) * (b.y - o.y) - (a.y - o.y) * (b.x - o.x); }

MOSAIC_HD double seg_point_dist(P2 a, P2 b, P2 p) {
    const double dx = b.x - a.x, dy = b.y - a.y, l2 = dx * dx + dy * dy;
    double t = l2 > 0 ? ((p.x - a.x) * dx + (p.y - a.y) * dy) / l2 : 0.0;
    t = t < 0 ? 0 : (t > 1 ? 1 : t);
    const double ex = a.x + t * dx - p.x, ey = a.y + t * dy - p.y;
    return sqrt(ex * ex + ey * ey);
}

// Segment (a, b) comes within eps of the convex polygon q[n] (counter-clockwise).
MOSAIC_HD bool seg_meets_poly(P2 a, P2 b, const P2* q, int n, double eps) {
    auto inside = [&](P2 p) {
        for (int e = 0; e < n; e++) {
            const P2 u = q[e], v = q[(e + 1) % n];
            const double len = sqrt((v.x - u.x) * (v.x - u.x) + (v.y - u.y) * (v.y - u.y));
            if (len > 0 && cross(u, v, p) / len < -eps) return false;
        }
        return true;
    };
    if (inside(a) || inside(b)) return true;
    for (int e = 0; e < n; e++) {
        const P2 u = q[e], v = q[(e + 1) % n];
        const double d1 = cross(a, b, u), d2 = cross(a, b, v), d3 = cross(u, v, a), d4 = cross(u, v, b);
        if (((d1 <= 0 && d2 >= 0) || (d1 >= 0 && d2 <= 0)) && ((d3 <= 0 && d4 >= 0) || (d3 >= 0 && d4 <= 0))) return true;
        if (seg_point_dist(a, b, u) <= eps || seg_point_dist(a, b, v) <= eps || seg_point_dist(u, v, a) <= eps ||
            seg_point_dist(u, v, b) <= eps)
            return true;
    }
    return false;
}

// Clip the segment to [x0, x1] x [y0, y1] (Liang-Barsky); false when it misses the box.
MOSAIC_HD bool clip_seg(double& ax, double& ay, double& bx, double& by, double x0, double y0, double x1, double y1) {
    double t0 = 0.0, t1 = 1.0;
    const double dx = bx - ax, dy = by - ay;
    const double p[4] = {-dx, dx, -dy, dy}, qv[4] = {ax - x0, x1 - ax, ay - y0, y1 - ay};
    for (int k = 0; k < 4; k++) {
        if (p[k] == 0) {
            if (qv[k] < 0) return false;
        } else {
            const double t = qv[k] / p[k];
            if (p[k] < 0) t0 = dmax(t0, t);
            else t1 = dmin(t1, t);
        }
    }
    if (t0 > t1) return false;
    const double nax = ax + t0 * dx, nay = ay + t0 * dy;
    bx = ax + t1 * dx;
    by = ay + t1 * dy;
    ax = nax;
    ay = nay;
    return true;
}

// Convex polygon q[n] clipped to the half-plane a x + b y + c >= 0 (Sutherland-Hodgman)
MOSAIC_HD int clip_half(const P2* q, int n, double a, double b, double c, P2* out) {
    int m = 0;
    for (int e = 0; e < n; e++) {
        const P2 u = q[e], v = q[(e + 1) % n];
        const double su = a * u.x + b * u.y + c, sv = a * v.x + b * v.y + c;
        if (su >= 0) out[m++] = u;
        if ((su >= 0) != (sv >= 0)) {
            const double t = su / (su - sv);
            out[m++] = P2{u.x + t * (v.x - u.x), u.y + t * (v.y - u.y)};
        }
    }
    return m;
}

// The line-record margins tried, narrowest first (sub-block units)
MOSAIC_HD double line_margin(int k) { return k == 0 ? 1.0 / 2048 : (k == 1 ? 1.0 / 512 : (k == 2 ? 1.0 / 128 : 1.0 / 32)); }

// Sub-block line records live in the TILE frame: s = A ut + B vt + Ct with (ut, vt) the point's
// offset from the tile's corner in sub-block units (0 <= ut, vt <= S), the line through the chip
// segment that holds the longest clipped piece -- so every sub-block one edge splits gets the same
// record and the tile keeps one copy.  The device evaluates fmaf(A / C, u, fmaf(B / C, v, Ct)) with
// (u, v) the tile-local leaf-cell offsets (exact in f32: S C 2^kFixBits <= 2^24 fixed-point units,
// truncated to one unit; the float kernels round to less than one).  A sub-block's two sides are
// certified beyond 1 - line_slack_tile: kLineSlack sub-block units per axis (the offsets' error,
// as in the sub-block frame) plus the two f32 roundings of the evaluation (each <= 2^-24 of its
// result, |inner| <= |B| S + |Ct|, |outer| <= |A| S + |inner|).
MOSAIC_HD double line_slack_tile(double A, double B, double Ct, int S, double kslack) {
    const double aa = fabs(A), ab = fabs(B);
    const double inner = ab * S + fabs(Ct), outer = aa * S + inner;
    return (aa + ab) * kslack + (inner + outer) * (1.0 / 8388608.0);
}

}  // namespace rbuild
}  // namespace mosaic
