// JTS 1.19 `Geometry.contains(Point)` for Polygon / MultiPolygon chips on gfx950 -- the
// st_contains(chip.wkb, point) filter of the chip join (reference
// src/main/scala/com/databricks/labs/mosaic/expressions/geometry/ST_Contains.scala:34-42 ->
// core/geometry/MosaicGeometryJTS.scala:101 -> JTS Geometry.contains).
//
// Semantics (identical to oracle/pip.c): inclusive envelope pre-check; PointLocator with the
// Mod-2 boundary rule (point on a boundary -> not contained; MultiPolygon parts accumulate
// isIn / numBoundaries); per ring an inclusive ring-envelope check and RayCrossingCounter over
// segments (ring[i], ring[i-1]) with the half-open straddle rule; orientation from JTS's
// CGAlgorithmsDD: FP64 filter (errbound 1e-15 * detsum) then a double-double determinant.
// Compiled with -ffp-contract=off: every filter / DD step is one IEEE operation, as in Java.
//
// Chip geometry layout in HBM (built by capi.hip from the chips' WKB):
//   verts      double2[V]   all ring vertices, ring after ring (x = lon/easting, y = lat/northing)
//   ring_start uint32[R+1]  ring r = verts[ring_start[r] .. ring_start[r+1])
//   ring_bbox  double4[R]   (minx, miny, maxx, maxy) per ring
//   part_ring  uint32[P+1]  part p = rings [part_ring[p] .. part_ring[p+1]); first ring = shell
//   geom_part  uint32[G+1]  geometry g = parts [geom_part[g] .. geom_part[g+1])
//   geom_bbox  double4[G]   envelope of geometry g
#pragma once
#include <stdint.h>

#if !defined(MOSAIC_HD)
#if defined(__HIPCC__)
#define MOSAIC_HD __host__ __device__ inline
#else
#define MOSAIC_HD inline
#endif
#endif

namespace mosaic {
namespace pip {

struct Vec2 {
    double x, y;
};
struct Box {
    double minx, miny, maxx, maxy;
};

struct GeomStore {
    const Vec2* verts;
    const uint32_t* ring_start;
    const Box* ring_bbox;
    const uint32_t* part_ring;
    const uint32_t* geom_part;
    const Box* geom_bbox;
};

MOSAIC_HD int signum(double x) { return x > 0 ? 1 : (x < 0 ? -1 : 0); }

struct DD {
    double hi, lo;
};

// JTS DD.selfAdd(yhi, ylo)
MOSAIC_HD DD dd_add(DD a, double yhi, double ylo) {
    double H, h, T, t, S, s, e, f;
    S = a.hi + yhi;
    T = a.lo + ylo;
    e = S - a.hi;
    f = T - a.lo;
    s = S - e;
    t = T - f;
    s = (yhi - e) + (a.hi - s);
    t = (ylo - f) + (a.lo - t);
    e = s + T;
    H = S + e;
    h = e + (S - H);
    e = t + h;
    DD r;
    r.hi = H + e;
    r.lo = e + (H - r.hi);
    return r;
}

// JTS DD.selfMultiply(yhi, ylo) (Dekker split, SPLIT = 2^27 + 1)
MOSAIC_HD DD dd_mul(DD a, double yhi, double ylo) {
    const double SPLIT = 134217729.0;
    double hx, tx, hy, ty, C, c;
    C = SPLIT * a.hi;
    hx = C - a.hi;
    c = SPLIT * yhi;
    hx = C - hx;
    tx = a.hi - hx;
    hy = c - yhi;
    C = a.hi * yhi;
    hy = c - hy;
    ty = yhi - hy;
    c = ((((hx * hy - C) + hx * ty) + tx * hy) + tx * ty) + (a.hi * ylo + a.lo * yhi);
    DD r;
    r.hi = C + c;
    hx = C - r.hi;
    r.lo = c + hx;
    return r;
}

// CGAlgorithmsDD.orientationIndex(p1, p2, q): 1 left (ccw), -1 right, 0 collinear
MOSAIC_HD int orientation_index(double p1x, double p1y, double p2x, double p2y, double qx, double qy) {
    double detleft = (p1x - qx) * (p2y - qy);
    double detright = (p1y - qy) * (p2x - qx);
    double det = detleft - detright;
    double detsum;
    if (detleft > 0.0) {
        if (detright <= 0.0) return signum(det);
        detsum = detleft + detright;
    } else if (detleft < 0.0) {
        if (detright >= 0.0) return signum(det);
        detsum = -detleft - detright;
    } else {
        return signum(det);
    }
    double errbound = 1e-15 * detsum;
    if ((det >= errbound) || (-det >= errbound)) return signum(det);
    DD dx1 = dd_add(DD{p2x, 0.0}, -p1x, 0.0);
    DD dy1 = dd_add(DD{p2y, 0.0}, -p1y, 0.0);
    DD dx2 = dd_add(DD{qx, 0.0}, -p2x, 0.0);
    DD dy2 = dd_add(DD{qy, 0.0}, -p2y, 0.0);
    DD a = dd_mul(dx1, dy2.hi, dy2.lo);
    DD b = dd_mul(dy1, dx2.hi, dx2.lo);
    DD d = dd_add(a, -b.hi, -b.lo);
    if (d.hi > 0) return 1;
    if (d.hi < 0) return -1;
    if (d.lo > 0) return 1;
    if (d.lo < 0) return -1;
    return 0;
}

// One RayCrossingCounter.countSegment step on an explicit segment record {p1, p2}
// (p1 = ring[i], p2 = ring[i-1]): sets `on` for a point on the segment, `cross` for a counted
// crossing of the rightward ray.
struct Edge {
    double p1x, p1y, p2x, p2y;
};

MOSAIC_HD void edge_rec_flags(const Edge& e, double px, double py, bool& on, bool& cross) {
    on = false;
    cross = false;
    if (e.p1x < px && e.p2x < px) return;
    if (px == e.p2x && py == e.p2y) {
        on = true;
    } else if (e.p1y == py && e.p2y == py) {
        double minx = e.p1x < e.p2x ? e.p1x : e.p2x;
        double maxx = e.p1x < e.p2x ? e.p2x : e.p1x;
        on = (px >= minx && px <= maxx);
    } else if (((e.p1y > py) && (e.p2y <= py)) || ((e.p2y > py) && (e.p1y <= py))) {
        int orient = orientation_index(e.p1x, e.p1y, e.p2x, e.p2y, px, py);
        if (orient == 0) {
            on = true;
        } else {
            if (e.p2y < e.p1y) orient = -orient;
            cross = orient == 1;
        }
    }
}

enum { LOC_INTERIOR = 0, LOC_BOUNDARY = 1, LOC_EXTERIOR = 2 };

MOSAIC_HD bool box_excludes(const Box& b, double px, double py) {
    return px < b.minx || px > b.maxx || py < b.miny || py > b.maxy;
}

// PointLocation.locateInRing via RayCrossingCounter
MOSAIC_HD int locate_in_ring(const Vec2* v, uint32_t n, double px, double py) {
    int crossings = 0;
    Vec2 p2 = v[0];
    for (uint32_t i = 1; i < n; i++) {
        Vec2 p1 = v[i];
        if (!(p1.x < px && p2.x < px)) {
            if (px == p2.x && py == p2.y) return LOC_BOUNDARY;
            if (p1.y == py && p2.y == py) {
                double minx = p1.x < p2.x ? p1.x : p2.x;
                double maxx = p1.x < p2.x ? p2.x : p1.x;
                if (px >= minx && px <= maxx) return LOC_BOUNDARY;
            } else if (((p1.y > py) && (p2.y <= py)) || ((p2.y > py) && (p1.y <= py))) {
                int orient = orientation_index(p1.x, p1.y, p2.x, p2.y, px, py);
                if (orient == 0) return LOC_BOUNDARY;
                if (p2.y < p1.y) orient = -orient;
                if (orient == 1) crossings++;
            }
        }
        p2 = p1;
    }
    return (crossings & 1) ? LOC_INTERIOR : LOC_EXTERIOR;
}

MOSAIC_HD int locate_in_polygon(const GeomStore& s, uint32_t part, double px, double py) {
    uint32_t r0 = s.part_ring[part], r1 = s.part_ring[part + 1];
    if (r1 <= r0) return LOC_EXTERIOR;
    uint32_t v0 = s.ring_start[r0], v1 = s.ring_start[r0 + 1];
    if (v1 <= v0) return LOC_EXTERIOR;
    if (box_excludes(s.ring_bbox[r0], px, py)) return LOC_EXTERIOR;
    int shell = locate_in_ring(s.verts + v0, v1 - v0, px, py);
    if (shell != LOC_INTERIOR) return shell;
    for (uint32_t r = r0 + 1; r < r1; r++) {
        if (box_excludes(s.ring_bbox[r], px, py)) continue;
        uint32_t a = s.ring_start[r], b = s.ring_start[r + 1];
        int hole = locate_in_ring(s.verts + a, b - a, px, py);
        if (hole == LOC_INTERIOR) return LOC_EXTERIOR;
        if (hole == LOC_BOUNDARY) return LOC_BOUNDARY;
    }
    return LOC_INTERIOR;
}

// Geometry.contains(POINT(px py)) for geometry g of the store
MOSAIC_HD bool contains(const GeomStore& s, uint32_t g, double px, double py) {
    uint32_t p0 = s.geom_part[g], p1 = s.geom_part[g + 1];
    if (p1 <= p0) return false;
    if (box_excludes(s.geom_bbox[g], px, py)) return false;
    if (p1 - p0 == 1) return locate_in_polygon(s, p0, px, py) == LOC_INTERIOR;
    bool is_in = false;
    int nb = 0;
    for (uint32_t p = p0; p < p1; p++) {
        int loc = locate_in_polygon(s, p, px, py);
        if (loc == LOC_INTERIOR) is_in = true;
        if (loc == LOC_BOUNDARY) nb++;
    }
    if (nb & 1) return false;
    return nb > 0 || is_in;
}


// ---- polygonal intersects (st_intersects_aggregate's chip test) ----
// JTS 1.19 RobustLineIntersector.computeIntersect's "is there an intersection" part for closed
// segments p1p2, q1q2: envelope test, the four Orientation.index signs (CGAlgorithmsDD, as above),
// and for four zero signs computeCollinearIntersection's envelope containments.
MOSAIC_HD bool in_seg_env(Vec2 a, Vec2 b, Vec2 q) {
    return q.x >= (a.x < b.x ? a.x : b.x) && q.x <= (a.x > b.x ? a.x : b.x) && q.y >= (a.y < b.y ? a.y : b.y) &&
           q.y <= (a.y > b.y ? a.y : b.y);
}
MOSAIC_HD bool segments_intersect(Vec2 p1, Vec2 p2, Vec2 q1, Vec2 q2) {
    // Envelope.intersects(p1, p2, q1, q2)
    const double pminx = p1.x < p2.x ? p1.x : p2.x, pmaxx = p1.x < p2.x ? p2.x : p1.x;
    const double qminx = q1.x < q2.x ? q1.x : q2.x, qmaxx = q1.x < q2.x ? q2.x : q1.x;
    if (qminx > pmaxx || qmaxx < pminx) return false;
    const double pminy = p1.y < p2.y ? p1.y : p2.y, pmaxy = p1.y < p2.y ? p2.y : p1.y;
    const double qminy = q1.y < q2.y ? q1.y : q2.y, qmaxy = q1.y < q2.y ? q2.y : q1.y;
    if (qminy > pmaxy || qmaxy < pminy) return false;
    const int pq1 = orientation_index(p1.x, p1.y, p2.x, p2.y, q1.x, q1.y);
    const int pq2 = orientation_index(p1.x, p1.y, p2.x, p2.y, q2.x, q2.y);
    if ((pq1 > 0 && pq2 > 0) || (pq1 < 0 && pq2 < 0)) return false;
    const int qp1 = orientation_index(q1.x, q1.y, q2.x, q2.y, p1.x, p1.y);
    const int qp2 = orientation_index(q1.x, q1.y, q2.x, q2.y, p2.x, p2.y);
    if ((qp1 > 0 && qp2 > 0) || (qp1 < 0 && qp2 < 0)) return false;
    if (pq1 == 0 && pq2 == 0 && qp1 == 0 && qp2 == 0)
        return in_seg_env(p1, p2, q1) || in_seg_env(p1, p2, q2) || in_seg_env(q1, q2, p1) || in_seg_env(q1, q2, p2);
    return true;
}
MOSAIC_HD bool boxes_meet(const Box& a, const Box& b) {
    return !(a.maxx < b.minx || b.maxx < a.minx || a.maxy < b.miny || b.maxy < a.miny);
}
// Some vertex of geometry g (the first vertex of each polygon's shell) lies in the interior or on
// the boundary of geometry h.  Once no boundary segments of g and h meet, every polygon of g lies
// wholly inside or wholly outside h (and vice versa), so this decides the rest of intersects.
MOSAIC_HD bool shell_vertex_in(const GeomStore& sg, uint32_t g, const GeomStore& sh, uint32_t h) {
    for (uint32_t p = sg.geom_part[g]; p < sg.geom_part[g + 1]; p++) {
        const uint32_t r0 = sg.part_ring[p];
        if (sg.part_ring[p + 1] <= r0 || sg.ring_start[r0 + 1] <= sg.ring_start[r0]) continue;
        const Vec2 v = sg.verts[sg.ring_start[r0]];
        if (box_excludes(sh.geom_bbox[h], v.x, v.y)) continue;
        for (uint32_t q = sh.geom_part[h]; q < sh.geom_part[h + 1]; q++)
            if (locate_in_polygon(sh, q, v.x, v.y) != LOC_EXTERIOR) return true;
    }
    return false;
}
// Geometry.intersects of two polygonal geometries (JTS 1.19 Geometry.intersects -> RelateOp
// isIntersects: the closed point sets share a point), one thread.
MOSAIC_HD bool intersects(const GeomStore& sa, uint32_t a, const GeomStore& sb, uint32_t b) {
    if (sa.geom_part[a + 1] <= sa.geom_part[a] || sb.geom_part[b + 1] <= sb.geom_part[b]) return false;
    if (!boxes_meet(sa.geom_bbox[a], sb.geom_bbox[b])) return false;
    const uint32_t ra0 = sa.part_ring[sa.geom_part[a]], ra1 = sa.part_ring[sa.geom_part[a + 1]];
    const uint32_t rb0 = sb.part_ring[sb.geom_part[b]], rb1 = sb.part_ring[sb.geom_part[b + 1]];
    for (uint32_t ra = ra0; ra < ra1; ra++) {
        if (!boxes_meet(sa.ring_bbox[ra], sb.geom_bbox[b])) continue;
        for (uint32_t rb = rb0; rb < rb1; rb++) {
            if (!boxes_meet(sa.ring_bbox[ra], sb.ring_bbox[rb])) continue;
            for (uint32_t i = sa.ring_start[ra]; i + 1 < sa.ring_start[ra + 1]; i++)
                for (uint32_t j = sb.ring_start[rb]; j + 1 < sb.ring_start[rb + 1]; j++)
                    if (segments_intersect(sa.verts[i], sa.verts[i + 1], sb.verts[j], sb.verts[j + 1])) return true;
        }
    }
    return shell_vertex_in(sb, b, sa, a) || shell_vertex_in(sa, a, sb, b);
}

}  // namespace pip
}  // namespace mosaic
