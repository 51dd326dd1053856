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

}  // namespace pip
}  // namespace mosaic
