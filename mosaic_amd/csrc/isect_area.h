// Areas for st_intersection_aggregate over the chip join (expressions/geometry/
// ST_IntersectionAggregate.scala update/merge): the aggregate of a (left key, right key) group is
// the JTS union of, per joined chip pair, `left.is_core && right.is_core ? cell : left.is_core ?
// right.wkb : right.is_core ? left.wkb : left.wkb intersection right.wkb`.  The reference's tests
// compare st_area of that union with the flat intersection's area within 1e-8
// (ST_IntersectionBehaviors.scala:22-71, 73-135); the engine computes that area.
//
// area(A n B) without building the intersection: with every ring oriented interior-left (shells
// counter-clockwise, holes clockwise, from the sign of its shoelace area), the indicator of a
// valid polygon is the sum over its edges (a, b) of sign(a x b) times the indicator of the triangle
// (O, a, b) fanned from a common origin O.  The area of A n B is then the bilinear sum over edge
// pairs of sign_a sign_b |T_a n T_b| -- two triangles, one convex clip each (Sutherland-Hodgman,
// at most 9 vertices).  Zero-width bridges a clipped ring can carry (an edge and its reverse)
// cancel term by term, coincident sides of two chips need no special case, and the pairs spread
// over a wave's lanes without sorting or point location.  O is the lower-left corner of the two
// bounding boxes: coordinates stay small, and every triangle is a sector within 90 degrees, so
// pairs of disjoint sectors are rejected with two cross products.
#pragma once
#include <math.h>
#include <stdint.h>

#include "pip_device.h"

namespace mosaic {
namespace isect {

// +1 / -1: the factor that orients ring r interior-left
MOSAIC_HD double ring_sign(const pip::GeomStore& s, uint32_t r, bool shell) {
    const uint32_t a = s.ring_start[r], b = s.ring_start[r + 1];
    double sum = 0;
    const double ox = s.verts[a].x, oy = s.verts[a].y;
    for (uint32_t i = a; i + 1 < b; i++)
        sum += (s.verts[i].x - ox) * (s.verts[i + 1].y - oy) - (s.verts[i + 1].x - ox) * (s.verts[i].y - oy);
    const bool ccw = sum > 0;
    return (shell ? ccw : !ccw) ? 1.0 : -1.0;
}

// flat edge index e of geometry g -> (ring, first vertex index, is-shell); false past the end
MOSAIC_HD bool edge_at(const pip::GeomStore& s, uint32_t g, uint32_t e, uint32_t* ring, uint32_t* v, bool* shell) {
    for (uint32_t p = s.geom_part[g]; p < s.geom_part[g + 1]; p++)
        for (uint32_t r = s.part_ring[p]; r < s.part_ring[p + 1]; r++) {
            const uint32_t n = s.ring_start[r + 1] - s.ring_start[r];
            const uint32_t ne = n > 1 ? n - 1 : 0;
            if (e < ne) {
                *ring = r;
                *v = s.ring_start[r] + e;
                *shell = r == s.part_ring[p];
                return true;
            }
            e -= ne;
        }
    return false;
}

MOSAIC_HD uint32_t edge_count(const pip::GeomStore& s, uint32_t g) {
    uint32_t n = 0;
    for (uint32_t p = s.geom_part[g]; p < s.geom_part[g + 1]; p++)
        for (uint32_t r = s.part_ring[p]; r < s.part_ring[p + 1]; r++) {
            const uint32_t k = s.ring_start[r + 1] - s.ring_start[r];
            n += k > 1 ? k - 1 : 0;
        }
    return n;
}

// |T1 n T2| for counter-clockwise triangles (0, a0, a1) and (0, b0, b1): T1 clipped by T2's three
// half-planes, then the shoelace
MOSAIC_HD double tri_overlap(double a0x, double a0y, double a1x, double a1y, double b0x, double b0y, double b1x,
                             double b1y) {
    double px[10], py[10], qx[10], qy[10];
    int n = 3;
    px[0] = 0.0, py[0] = 0.0, px[1] = a0x, py[1] = a0y, px[2] = a1x, py[2] = a1y;
    const double cx[3] = {0.0, b0x, b1x}, cy[3] = {0.0, b0y, b1y};
    for (int e = 0; e < 3 && n > 0; e++) {
        const double ux = cx[e], uy = cy[e], vx = cx[e == 2 ? 0 : e + 1], vy = cy[e == 2 ? 0 : e + 1];
        const double dx = vx - ux, dy = vy - uy;
        int m = 0;
        for (int i = 0; i < n; i++) {
            const int j = i + 1 == n ? 0 : i + 1;
            const double si = dx * (py[i] - uy) - dy * (px[i] - ux);  // >= 0: inside (left of the edge)
            const double sj = dx * (py[j] - uy) - dy * (px[j] - ux);
            if (si >= 0) {
                qx[m] = px[i];
                qy[m] = py[i];
                m++;
            }
            if ((si >= 0) != (sj >= 0)) {
                const double t = si / (si - sj);
                qx[m] = px[i] + t * (px[j] - px[i]);
                qy[m] = py[i] + t * (py[j] - py[i]);
                m++;
            }
        }
        n = m;
        for (int i = 0; i < n; i++) {
            px[i] = qx[i];
            py[i] = qy[i];
        }
    }
    double a = 0;
    for (int i = 0; i < n; i++) {
        const int j = i + 1 == n ? 0 : i + 1;
        a += px[i] * py[j] - px[j] * py[i];
    }
    return 0.5 * fabs(a);
}

// The term of the edge pair (p0 -> p1 of A, ring factor sa; q0 -> q1 of B, ring factor sb),
// coordinates relative to the common origin
MOSAIC_HD double pair_term(double p0x, double p0y, double p1x, double p1y, double sa, double q0x, double q0y,
                           double q1x, double q1y, double sb) {
    const double ca = p0x * p1y - p1x * p0y, cb = q0x * q1y - q1x * q0y;
    if (ca == 0.0 || cb == 0.0) return 0.0;
    const double s = sa * sb * (ca > 0 ? 1.0 : -1.0) * (cb > 0 ? 1.0 : -1.0);
    // both triangles counter-clockwise; the orientations went into the sign
    const double ax0 = ca > 0 ? p0x : p1x, ay0 = ca > 0 ? p0y : p1y, ax1 = ca > 0 ? p1x : p0x, ay1 = ca > 0 ? p1y : p0y;
    const double bx0 = cb > 0 ? q0x : q1x, by0 = cb > 0 ? q0y : q1y, bx1 = cb > 0 ? q1x : q0x, by1 = cb > 0 ? q1y : q0y;
    // with the origin at the lower-left corner of both bounding boxes every vertex lies within 90
    // degrees of +x, so two triangles overlap only where their angular sectors do
    if (ax0 * by1 - ay0 * bx1 <= 0.0 || bx0 * ay1 - by0 * ax1 <= 0.0) return 0.0;
    return s * tri_overlap(ax0, ay0, ax1, ay1, bx0, by0, bx1, by1);
}

}  // namespace isect
}  // namespace mosaic
