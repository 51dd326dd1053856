/*
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  CPU restatement of JTS 1.19 Geometry.contains for a
 * Polygon / MultiPolygon chip and a Point, as reached from ST_Contains
 * (src/main/scala/com/databricks/labs/mosaic/expressions/geometry/ST_Contains.scala:34-42 ->
 *  core/geometry/MosaicGeometryJTS.scala:101).
 *
 * JTS (org.locationtech.jts:jts-core:1.19.0, reference pom.xml:98-102) is absent here; restated:
 *   Geometry.contains: envelope pre-check (inclusive) then relate(..).isContains(), which for a
 *     point argument is PointLocator.locate(p, A) == INTERIOR (Mod-2 boundary rule);
 *   PointLocator.locateInPolygon / MultiPolygon accumulation (isIn, numBoundaries);
 *   PointLocation.locateInRing -> RayCrossingCounter.countSegment(ring[i], ring[i-1]);
 *   CGAlgorithmsDD.orientationIndex: orientationIndexFilter (DP_SAFE_EPSILON = 1e-15) then the
 *     double-double determinant of (p2 - p1) x (q - p2).
 * The rectangle fast path (RectangleContains) returns the same answer for points.
 * Build with -ffp-contract=off: the filter and the double-double steps rely on IEEE rounding of
 * every individual operation.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

/* ---- JTS DD (double-double), the subset used by orientationIndex ---- */
typedef struct {
    double hi, lo;
} DD;

static DD dd_self_add(DD a, double yhi, double ylo) {
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
    double zhi = H + e;
    double zlo = e + (H - zhi);
    DD r = {zhi, zlo};
    return r;
}

static DD dd_self_multiply(DD a, double yhi, double ylo) {
    const double SPLIT = 134217729.0; /* 2^27 + 1 */
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
    double zhi = C + c;
    hx = C - zhi;
    double zlo = c + hx;
    DD r = {zhi, zlo};
    return r;
}

static int dd_signum(DD a) {
    if (a.hi > 0) return 1;
    if (a.hi < 0) return -1;
    if (a.lo > 0) return 1;
    if (a.lo < 0) return -1;
    return 0;
}

static int signum(double x) { return x > 0 ? 1 : (x < 0 ? -1 : 0); }

/* CGAlgorithmsDD.orientationIndexFilter */
static int orientation_filter(double pax, double pay, double pbx, double pby, double pcx, double pcy) {
    double detsum;
    double detleft = (pax - pcx) * (pby - pcy);
    double detright = (pay - pcy) * (pbx - pcx);
    double det = detleft - detright;
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
    return 2; /* FAILURE */
}

/* CGAlgorithmsDD.orientationIndex(p1, p2, q) */
int oracle_orientation_index(double p1x, double p1y, double p2x, double p2y, double qx, double qy) {
    int index = orientation_filter(p1x, p1y, p2x, p2y, qx, qy);
    if (index <= 1) return index;
    DD dx1 = dd_self_add((DD){p2x, 0.0}, -p1x, 0.0);
    DD dy1 = dd_self_add((DD){p2y, 0.0}, -p1y, 0.0);
    DD dx2 = dd_self_add((DD){qx, 0.0}, -p2x, 0.0);
    DD dy2 = dd_self_add((DD){qy, 0.0}, -p2y, 0.0);
    DD a = dd_self_multiply(dx1, dy2.hi, dy2.lo);
    DD b = dd_self_multiply(dy1, dx2.hi, dx2.lo);
    DD d = dd_self_add(a, -b.hi, -b.lo);
    return dd_signum(d);
}

enum { LOC_INTERIOR = 0, LOC_BOUNDARY = 1, LOC_EXTERIOR = 2 };

/* PointLocation.locateInRing via RayCrossingCounter; xy holds n vertices (closed ring) */
static int locate_in_ring(double px, double py, const double* xy, int64_t n) {
    int crossings = 0;
    for (int64_t i = 1; i < n; i++) {
        double p1x = xy[2 * i], p1y = xy[2 * i + 1];
        double p2x = xy[2 * (i - 1)], p2y = xy[2 * (i - 1) + 1];
        if (p1x < px && p2x < px) continue;
        if (px == p2x && py == p2y) return LOC_BOUNDARY;
        if (p1y == py && p2y == py) {
            double minx = p1x, maxx = p2x;
            if (minx > maxx) {
                minx = p2x;
                maxx = p1x;
            }
            if (px >= minx && px <= maxx) return LOC_BOUNDARY;
            continue;
        }
        if (((p1y > py) && (p2y <= py)) || ((p2y > py) && (p1y <= py))) {
            int orient = oracle_orientation_index(p1x, p1y, p2x, p2y, px, py);
            if (orient == 0) return LOC_BOUNDARY;
            if (p2y < p1y) orient = -orient;
            if (orient == 1) crossings++;
        }
    }
    return (crossings & 1) ? LOC_INTERIOR : LOC_EXTERIOR;
}

/* PointLocator.locateInPolygonRing: envelope check then locateInRing */
static int locate_in_polygon_ring(double px, double py, const double* xy, int64_t n) {
    if (n == 0) return LOC_EXTERIOR;
    double minx = xy[0], maxx = xy[0], miny = xy[1], maxy = xy[1];
    for (int64_t i = 1; i < n; i++) {
        double x = xy[2 * i], y = xy[2 * i + 1];
        if (x < minx) minx = x;
        if (x > maxx) maxx = x;
        if (y < miny) miny = y;
        if (y > maxy) maxy = y;
    }
    if (px < minx || px > maxx || py < miny || py > maxy) return LOC_EXTERIOR;
    return locate_in_ring(px, py, xy, n);
}

/* PointLocator.locateInPolygon */
static int locate_in_polygon(const oracle_geom* g, int64_t part, double px, double py) {
    int64_t r0 = g->part_rings[part], r1 = g->part_rings[part + 1];
    if (r1 <= r0) return LOC_EXTERIOR;
    int64_t v0 = g->ring_offsets[r0], v1 = g->ring_offsets[r0 + 1];
    if (v1 <= v0) return LOC_EXTERIOR; /* empty polygon */
    int shell = locate_in_polygon_ring(px, py, g->xy + 2 * v0, v1 - v0);
    if (shell == LOC_EXTERIOR) return LOC_EXTERIOR;
    if (shell == LOC_BOUNDARY) return LOC_BOUNDARY;
    for (int64_t r = r0 + 1; r < r1; r++) {
        int64_t a = g->ring_offsets[r], b = g->ring_offsets[r + 1];
        int hole = locate_in_polygon_ring(px, py, g->xy + 2 * a, b - a);
        if (hole == LOC_INTERIOR) return LOC_EXTERIOR;
        if (hole == LOC_BOUNDARY) return LOC_BOUNDARY;
    }
    return LOC_INTERIOR;
}

/* Geometry.contains(point): envelope test, then PointLocator (Mod-2) == INTERIOR */
int oracle_contains(const oracle_geom* g, double px, double py) {
    /* envelope of the whole geometry (inclusive containment of the point) */
    int64_t nv = g->ring_offsets[g->part_rings[g->n_parts]] - g->ring_offsets[g->part_rings[0]];
    if (g->n_parts == 0 || nv == 0) return 0;
    int64_t v0 = g->ring_offsets[g->part_rings[0]];
    double minx = INFINITY, maxx = -INFINITY, miny = INFINITY, maxy = -INFINITY;
    for (int64_t i = v0; i < v0 + nv; i++) {
        double x = g->xy[2 * i], y = g->xy[2 * i + 1];
        if (x < minx) minx = x;
        if (x > maxx) maxx = x;
        if (y < miny) miny = y;
        if (y > maxy) maxy = y;
    }
    if (px < minx || px > maxx || py < miny || py > maxy) return 0;
    if (g->n_parts == 1) return locate_in_polygon(g, 0, px, py) == LOC_INTERIOR;
    int is_in = 0, nb = 0;
    for (int64_t p = 0; p < g->n_parts; p++) {
        int loc = locate_in_polygon(g, p, px, py);
        if (loc == LOC_INTERIOR) is_in = 1;
        if (loc == LOC_BOUNDARY) nb++;
    }
    if (nb % 2 == 1) return 0; /* BOUNDARY */
    return (nb > 0 || is_in);
}

/* ---- WKB (OGC / JTS WKBReader subset: Polygon, MultiPolygon; both byte orders) ---- */
typedef struct {
    const uint8_t* p;
    int64_t len, pos;
} rd;

static int rd_u8(rd* r, uint8_t* v) {
    if (r->pos + 1 > r->len) return -1;
    *v = r->p[r->pos++];
    return 0;
}
static int rd_u32(rd* r, int le, uint32_t* v) {
    if (r->pos + 4 > r->len) return -1;
    const uint8_t* b = r->p + r->pos;
    *v = le ? ((uint32_t)b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16 | (uint32_t)b[3] << 24)
            : ((uint32_t)b[3] | (uint32_t)b[2] << 8 | (uint32_t)b[1] << 16 | (uint32_t)b[0] << 24);
    r->pos += 4;
    return 0;
}
static int rd_f64(rd* r, int le, double* v) {
    if (r->pos + 8 > r->len) return -1;
    uint64_t u = 0;
    const uint8_t* b = r->p + r->pos;
    for (int i = 0; i < 8; i++) u |= (uint64_t)b[le ? i : 7 - i] << (8 * i);
    memcpy(v, &u, 8);
    r->pos += 8;
    return 0;
}

typedef struct {
    double* xy;
    int64_t nv, cv;
    int64_t* ring_off;
    int64_t nr, cr;
    int64_t* part_rings;
    int64_t np, cp;
} builder;

static int push_v(builder* b, double x, double y) {
    if (b->nv == b->cv) {
        b->cv = b->cv ? 2 * b->cv : 64;
        b->xy = realloc(b->xy, sizeof(double) * 2 * b->cv);
    }
    b->xy[2 * b->nv] = x;
    b->xy[2 * b->nv + 1] = y;
    b->nv++;
    return 0;
}
static void push_ring(builder* b) {
    if (b->nr + 1 >= b->cr) {
        b->cr = b->cr ? 2 * b->cr : 16;
        b->ring_off = realloc(b->ring_off, sizeof(int64_t) * (b->cr + 1));
    }
    b->ring_off[++b->nr] = b->nv;
}
static void push_part(builder* b) {
    if (b->np + 1 >= b->cp) {
        b->cp = b->cp ? 2 * b->cp : 8;
        b->part_rings = realloc(b->part_rings, sizeof(int64_t) * (b->cp + 1));
    }
    b->part_rings[++b->np] = b->nr;
}

static int read_header(rd* r, int* le, uint32_t* type, int* dims) {
    uint8_t bo;
    if (rd_u8(r, &bo)) return -1;
    *le = bo == 1;
    uint32_t t;
    if (rd_u32(r, *le, &t)) return -1;
    int has_z = (t & 0x80000000u) != 0, has_m = (t & 0x40000000u) != 0;
    int has_srid = (t & 0x20000000u) != 0;
    t &= 0x0fffffffu;
    if (t >= 3000) {
        has_z = has_m = 1;
        t -= 3000;
    } else if (t >= 2000) {
        has_m = 1;
        t -= 2000;
    } else if (t >= 1000) {
        has_z = 1;
        t -= 1000;
    }
    if (has_srid) {
        uint32_t srid;
        if (rd_u32(r, *le, &srid)) return -1;
    }
    *type = t;
    *dims = 2 + has_z + has_m;
    return 0;
}

static int read_polygon_body(rd* r, int le, int dims, builder* b) {
    uint32_t nrings;
    if (rd_u32(r, le, &nrings)) return -1;
    for (uint32_t ri = 0; ri < nrings; ri++) {
        uint32_t npts;
        if (rd_u32(r, le, &npts)) return -1;
        for (uint32_t k = 0; k < npts; k++) {
            double x, y, z;
            if (rd_f64(r, le, &x) || rd_f64(r, le, &y)) return -1;
            for (int d = 2; d < dims; d++)
                if (rd_f64(r, le, &z)) return -1;
            push_v(b, x, y);
        }
        push_ring(b);
    }
    push_part(b);
    return 0;
}

typedef struct {
    builder b;
    oracle_geom g;
} parsed_geom;

/* Decode one WKB into rings; NULL on parse error. */
void* oracle_wkb_parse(const uint8_t* wkb, int64_t len) {
    rd r = {wkb, len, 0};
    parsed_geom* pg = calloc(1, sizeof(parsed_geom));
    builder* b = &pg->b;
    b->ring_off = malloc(sizeof(int64_t) * 17);
    b->cr = 16;
    b->ring_off[0] = 0;
    b->part_rings = malloc(sizeof(int64_t) * 9);
    b->cp = 8;
    b->part_rings[0] = 0;
    int le, dims, rc = 0;
    uint32_t type;
    if (read_header(&r, &le, &type, &dims)) {
        rc = -1;
    } else if (type == 3) {
        rc = read_polygon_body(&r, le, dims, b);
    } else if (type == 6) {
        uint32_t nparts;
        if (rd_u32(&r, le, &nparts)) rc = -1;
        for (uint32_t p = 0; rc == 0 && p < nparts; p++) {
            int le2, dims2;
            uint32_t t2;
            if (read_header(&r, &le2, &t2, &dims2) || t2 != 3)
                rc = -1;
            else
                rc = read_polygon_body(&r, le2, dims2, b);
        }
    } else {
        rc = -1;
    }
    if (rc != 0) {
        oracle_parsed_free(pg);
        return NULL;
    }
    pg->g.xy = b->xy;
    pg->g.ring_offsets = b->ring_off;
    pg->g.part_rings = b->part_rings;
    pg->g.n_parts = b->np;
    return pg;
}

void oracle_parsed_free(void* p) {
    parsed_geom* pg = (parsed_geom*)p;
    if (!pg) return;
    free(pg->b.xy);
    free(pg->b.ring_off);
    free(pg->b.part_rings);
    free(pg);
}

int oracle_parsed_contains(const void* p, double px, double py) {
    const parsed_geom* pg = (const parsed_geom*)p;
    if (!pg->b.xy) return 0;
    return oracle_contains(&pg->g, px, py);
}

int oracle_wkb_contains(const uint8_t* wkb, int64_t len, double px, double py) {
    void* p = oracle_wkb_parse(wkb, len);
    if (!p) return -1;
    int r = oracle_parsed_contains(p, px, py);
    oracle_parsed_free(p);
    return r;
}

/* ---- JTS 1.19 Geometry.intersects for two polygonal geometries (st_intersects_aggregate) ----
 * Reached from ST_IntersectsAggregate.update (expressions/geometry/ST_IntersectsAggregate.scala:28-39)
 * -> MosaicGeometryJTS.intersects -> Geometry.intersects: envelope pre-check, then
 * RelateOp(...).isIntersects(), i.e. the closed point sets share a point.  Restated as:
 *   (1) some boundary segment of a meets some boundary segment of b, decided as
 *       RobustLineIntersector.computeIntersect does: Envelope.intersects(p1, p2, q1, q2), the four
 *       Orientation.index (CGAlgorithmsDD) signs, and for four zero signs
 *       computeCollinearIntersection's Envelope.intersects(p1, p2, q) containments;
 *   (2) otherwise the boundaries are disjoint, so each polygon of one geometry lies wholly inside or
 *       outside the other: the first shell vertex of each polygon of b located in a (PointLocator,
 *       INTERIOR or BOUNDARY), and of a in b. */
static int in_seg_env(double ax, double ay, double bx, double by, double qx, double qy) {
    return qx >= fmin(ax, bx) && qx <= fmax(ax, bx) && qy >= fmin(ay, by) && qy <= fmax(ay, by);
}

int oracle_segments_intersect(double p1x, double p1y, double p2x, double p2y, double q1x, double q1y, double q2x,
                              double q2y) {
    if (fmin(q1x, q2x) > fmax(p1x, p2x) || fmax(q1x, q2x) < fmin(p1x, p2x)) return 0;
    if (fmin(q1y, q2y) > fmax(p1y, p2y) || fmax(q1y, q2y) < fmin(p1y, p2y)) return 0;
    int pq1 = oracle_orientation_index(p1x, p1y, p2x, p2y, q1x, q1y);
    int pq2 = oracle_orientation_index(p1x, p1y, p2x, p2y, q2x, q2y);
    if ((pq1 > 0 && pq2 > 0) || (pq1 < 0 && pq2 < 0)) return 0;
    int qp1 = oracle_orientation_index(q1x, q1y, q2x, q2y, p1x, p1y);
    int qp2 = oracle_orientation_index(q1x, q1y, q2x, q2y, p2x, p2y);
    if ((qp1 > 0 && qp2 > 0) || (qp1 < 0 && qp2 < 0)) return 0;
    if (pq1 == 0 && pq2 == 0 && qp1 == 0 && qp2 == 0)
        return in_seg_env(p1x, p1y, p2x, p2y, q1x, q1y) || in_seg_env(p1x, p1y, p2x, p2y, q2x, q2y) ||
               in_seg_env(q1x, q1y, q2x, q2y, p1x, p1y) || in_seg_env(q1x, q1y, q2x, q2y, p2x, p2y);
    return 1;
}

static void geom_env(const oracle_geom* g, double* e) {
    e[0] = e[1] = INFINITY;
    e[2] = e[3] = -INFINITY;
    int64_t v0 = g->ring_offsets[g->part_rings[0]], v1 = g->ring_offsets[g->part_rings[g->n_parts]];
    for (int64_t i = v0; i < v1; i++) {
        e[0] = fmin(e[0], g->xy[2 * i]);
        e[1] = fmin(e[1], g->xy[2 * i + 1]);
        e[2] = fmax(e[2], g->xy[2 * i]);
        e[3] = fmax(e[3], g->xy[2 * i + 1]);
    }
}

static int shell_vertex_in(const oracle_geom* g, const oracle_geom* h) {
    for (int64_t p = 0; p < g->n_parts; p++) {
        int64_t r0 = g->part_rings[p];
        if (g->part_rings[p + 1] <= r0 || g->ring_offsets[r0 + 1] <= g->ring_offsets[r0]) continue;
        double x = g->xy[2 * g->ring_offsets[r0]], y = g->xy[2 * g->ring_offsets[r0] + 1];
        for (int64_t q = 0; q < h->n_parts; q++)
            if (locate_in_polygon(h, q, x, y) != LOC_EXTERIOR) return 1;
    }
    return 0;
}

int oracle_intersects(const oracle_geom* a, const oracle_geom* b) {
    if (a->n_parts == 0 || b->n_parts == 0) return 0;
    double ea[4], eb[4];
    geom_env(a, ea);
    geom_env(b, eb);
    if (!(ea[0] <= ea[2]) || !(eb[0] <= eb[2])) return 0; /* empty */
    if (ea[2] < eb[0] || eb[2] < ea[0] || ea[3] < eb[1] || eb[3] < ea[1]) return 0;
    int64_t ra1 = a->part_rings[a->n_parts], rb1 = b->part_rings[b->n_parts];
    for (int64_t ra = a->part_rings[0]; ra < ra1; ra++)
        for (int64_t rb = b->part_rings[0]; rb < rb1; rb++)
            for (int64_t i = a->ring_offsets[ra]; i + 1 < a->ring_offsets[ra + 1]; i++)
                for (int64_t j = b->ring_offsets[rb]; j + 1 < b->ring_offsets[rb + 1]; j++)
                    if (oracle_segments_intersect(a->xy[2 * i], a->xy[2 * i + 1], a->xy[2 * i + 2], a->xy[2 * i + 3],
                                                  b->xy[2 * j], b->xy[2 * j + 1], b->xy[2 * j + 2], b->xy[2 * j + 3]))
                        return 1;
    return shell_vertex_in(b, a) || shell_vertex_in(a, b);
}

int oracle_wkb_intersects(const uint8_t* wa, int64_t la, const uint8_t* wb, int64_t lb) {
    void* pa = oracle_wkb_parse(wa, la);
    if (!pa) return -1;
    void* pb = oracle_wkb_parse(wb, lb);
    if (!pb) {
        oracle_parsed_free(pa);
        return -1;
    }
    const parsed_geom* ga = (const parsed_geom*)pa;
    const parsed_geom* gb = (const parsed_geom*)pb;
    int r = (ga->b.xy && gb->b.xy) ? oracle_intersects(&ga->g, &gb->g) : 0;
    oracle_parsed_free(pa);
    oracle_parsed_free(pb);
    return r;
}
