/* TEST INFRASTRUCTURE ONLY (never linked into the product): CPU restatement of grid_polyfill for
 * H3 and BNG, the checker of the mosaic_polyfill kernels.
 *
 * H3: reference H3IndexSystem.polyfill (core/index/H3IndexSystem.scala:113-126) calls
 * h3.polyfill(shell, holes, res) per polygon part (h3-java 3.7.0 -> H3 C v3.7 algos.c
 * _polyfillInternal), vertices through Math.toRadians.  Restated here from the published H3 C
 * algorithm with the host glibc (the reference's libm):
 *   - the search set: every edge of the shell and the holes (closing edge included) sampled at
 *     lineHexEstimate points (_getEdgeHexagons), each sample's cell once, in sample order;
 *   - breadth-first rounds: each searched cell's kRing(1) cells not yet accepted are accepted when
 *     their h3ToGeo centre is inside the part (pointInsidePolygon: H3's ray cast with the westerly
 *     DBL_EPSILON tie-break, bbox pre-test, holes) and searched in the next round;
 *   - the output order: H3 stores accepted cells in an open-addressing table of maxPolyfillSize
 *     slots (home slot cell % size, linear probing, insertion in acceptance order) and h3-java
 *     returns its non-empty slots in slot order.
 * Independence from the product: the kRing(1) neighbours come from a geometric construction
 * (each boundary edge's midpoint, reflected centre -> geoToH3), not from H3's ring walk, so the
 * oracle's acceptance order within a round differs from H3's; the slot order it reports is
 * therefore H3's exactly when no cell was displaced by probing, which *collision_free reports.
 * Sets are exact either way.  Pinned by the reference docs' res-0 example
 * (docs/source/api/spatial-indexing.rst:213-221, order included).
 *
 * BNG: reference BNGIndexSystem.polyfill (core/index/BNGIndexSystem.scala:185-204): breadth-first
 * from the cells of every shell / hole vertex and of the geometry's centroid; a visited cell is kept
 * when the geometry (JTS contains) holds its square's centroid (x + e / 2, y + e / 2), and then its
 * kLoop(1) cells are visited.  The result set is returned (the reference's Scala Set order is not
 * restated). */
#include <math.h>
#include <float.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define EARTH_RADIUS_KM 6371.007180918475

/* ---- a small open-addressing set of nonzero int64 ---- */
typedef struct {
    int64_t* k;
    int64_t cap;
} Set64;

static int set_init(Set64* s, int64_t want) {
    s->cap = 64;
    while (s->cap < 2 * want + 16) s->cap *= 2;
    s->k = (int64_t*)calloc((size_t)s->cap, 8);
    return s->k != NULL;
}
static uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    return x;
}
/* 1 if inserted, 0 if present, -1 full */
static int set_add(Set64* s, int64_t v) {
    uint64_t m = (uint64_t)s->cap - 1, h = mix64((uint64_t)v) & m;
    for (int64_t n = 0; n < s->cap; n++, h = (h + 1) & m) {
        if (s->k[h] == v) return 0;
        if (s->k[h] == 0) {
            s->k[h] = v;
            return 1;
        }
    }
    return -1;
}
static int set_has(const Set64* s, int64_t v) {
    uint64_t m = (uint64_t)s->cap - 1, h = mix64((uint64_t)v) & m;
    for (int64_t n = 0; n < s->cap; n++, h = (h + 1) & m) {
        if (s->k[h] == v) return 1;
        if (s->k[h] == 0) return 0;
    }
    return 0;
}

/* ---- H3 C v3.7 pieces (geoCoord.c, bbox.c, polygonAlgos.h, polygon.c) ---- */
static double dist_km(double alat, double alon, double blat, double blon) {
    double sin_lat = sin((blat - alat) / 2.0);
    double sin_lng = sin((blon - alon) / 2.0);
    double A = sin_lat * sin_lat + cos(alat) * cos(blat) * sin_lng * sin_lng;
    return 2 * atan2(sqrt(A), sqrt(1 - A)) * EARTH_RADIUS_KM;
}

typedef struct {
    double north, south, east, west;
} BBox;

static void loop_bbox(const double* lat, const double* lon, int64_t n, BBox* b) {
    if (n == 0) {
        memset(b, 0, sizeof *b);
        return;
    }
    b->south = DBL_MAX;
    b->west = DBL_MAX;
    b->north = -DBL_MAX;
    b->east = -DBL_MAX;
    double min_pos = DBL_MAX, max_neg = -DBL_MAX;
    int tm = 0;
    for (int64_t i = 0; i < n; i++) {
        double la = lat[i], lo = lon[i], nlo = lon[(i + 1) % n];
        if (la < b->south) b->south = la;
        if (lo < b->west) b->west = lo;
        if (la > b->north) b->north = la;
        if (lo > b->east) b->east = lo;
        if (lo > 0 && lo < min_pos) min_pos = lo;
        if (lo < 0 && lo > max_neg) max_neg = lo;
        if (fabs(lo - nlo) > M_PI) tm = 1;
    }
    if (tm) {
        b->east = max_neg;
        b->west = min_pos;
    }
}

static int bbox_has(const BBox* b, double lat, double lon) {
    int tm = b->east < b->west;
    if (!(lat >= b->south && lat <= b->north)) return 0;
    return tm ? (lon >= b->west || lon <= b->east) : (lon >= b->west && lon <= b->east);
}

#define NORM_LON(lon, tm) ((tm) && (lon) < 0 ? (lon) + (double)(2 * M_PI) : (lon))

static int loop_inside(const double* lat, const double* lon, int64_t n, const BBox* b, double plat, double plon) {
    if (!bbox_has(b, plat, plon)) return 0;
    int tm = b->east < b->west, in = 0;
    double lng = NORM_LON(plon, tm);
    for (int64_t i = 0; i < n; i++) {
        double alat = lat[i], alon = lon[i], blat = lat[(i + 1) % n], blon = lon[(i + 1) % n];
        if (alat > blat) {
            double t = alat;
            alat = blat;
            blat = t;
            t = alon;
            alon = blon;
            blon = t;
        }
        if (plat < alat || plat > blat) continue;
        double al = NORM_LON(alon, tm), bl = NORM_LON(blon, tm);
        if (al == lng || bl == lng) lng -= DBL_EPSILON;
        double ratio = (plat - alat) / (blat - alat);
        double test = NORM_LON(al + (bl - al) * ratio, tm);
        if (test > lng) in = !in;
    }
    return in;
}

typedef struct {
    const double *lat, *lon;
    const int64_t* ring_off;
    int n_rings;
    BBox* boxes;
} Part;

static int part_inside(const Part* p, double lat, double lon) {
    const int64_t a = p->ring_off[0], b = p->ring_off[1];
    if (!loop_inside(p->lat + a, p->lon + a, b - a, &p->boxes[0], lat, lon)) return 0;
    for (int r = 1; r < p->n_rings; r++) {
        const int64_t s = p->ring_off[r], e = p->ring_off[r + 1];
        if (loop_inside(p->lat + s, p->lon + s, e - s, &p->boxes[r], lat, lon)) return 0;
    }
    return 1;
}

static double pent_radius_km(int res) {
    uint64_t h = (uint64_t)1 << 59 | (uint64_t)res << 52 | (uint64_t)4 << 45;
    for (int r = res + 1; r <= 15; r++) h |= (uint64_t)7 << ((15 - r) * 3);
    double clat, clon, v[20];
    oracle_h3_to_geo((int64_t)h, &clat, &clon);
    oracle_h3_to_geo_boundary((int64_t)h, v);
    return dist_km(clat, clon, v[0], v[1]);
}

static void unit3(double lat, double lon, double* v) {
    v[0] = cos(lat) * cos(lon);
    v[1] = cos(lat) * sin(lon);
    v[2] = sin(lat);
}

/* kRing(h, 1) as a set: h, then per boundary edge the cell just beyond the edge's midpoint (the
 * unit vector m + (m - c) / 8, m the edge midpoint on the sphere, c the centre); returns the count
 * (<= 11) */
static int ring1(int64_t h, int res, int64_t* out) {
    double clat, clon, v[20], c[3], a[3], b[3];
    oracle_h3_to_geo(h, &clat, &clon);
    int nv = oracle_h3_to_geo_boundary(h, v), n = 0;
    out[n++] = h;
    unit3(clat, clon, c);
    for (int k = 0; k < nv; k++) {
        int k2 = (k + 1) % nv;
        unit3(v[2 * k], v[2 * k + 1], a);
        unit3(v[2 * k2], v[2 * k2 + 1], b);
        double m[3], q[3];
        for (int d = 0; d < 3; d++) m[d] = a[d] + b[d];
        double mn = sqrt(m[0] * m[0] + m[1] * m[1] + m[2] * m[2]);
        for (int d = 0; d < 3; d++) q[d] = m[d] / mn + (m[d] / mn - c[d]) / 8;
        double lat = atan2(q[2], sqrt(q[0] * q[0] + q[1] * q[1])), lon = atan2(q[1], q[0]);
        int64_t nb = oracle_h3_geo_to_h3(lat, lon, res);
        int seen = nb == 0;
        for (int t = 0; t < n && !seen; t++) seen = out[t] == nb;
        if (!seen) out[n++] = nb;
    }
    return n;
}

int oracle_h3_ring1(int64_t h, int64_t* out) { return ring1(h, (int)((h >> 52) & 15), out); }

/* One polygon part: rings [0, n_rings) at lat / lon (radians) + ring_off; returns the cell count
 * written to out (in H3's slot order), -1 if cap is too small / allocation failed. */
int64_t oracle_h3_polyfill(const double* lat, const double* lon, const int64_t* ring_off, int n_rings, int res,
                           int64_t* out, int64_t cap, int* collision_free) {
    *collision_free = 1;
    if (n_rings < 1) return 0;
    BBox* boxes = (BBox*)calloc((size_t)n_rings, sizeof(BBox));
    for (int r = 0; r < n_rings; r++)
        loop_bbox(lat + ring_off[r], lon + ring_off[r], ring_off[r + 1] - ring_off[r], &boxes[r]);
    Part part = {lat, lon, ring_off, n_rings, boxes};
    const double pr = pent_radius_km(res);
    /* maxPolyfillSize */
    const double area = 0.8 * (2.59807621135 * pr * pr);
    const double d = dist_km(boxes[0].north, boxes[0].east, boxes[0].south, boxes[0].west);
    const double aa = d * d / fmin(3.0, fabs((boxes[0].east - boxes[0].west) / (boxes[0].north - boxes[0].south)));
    int64_t M = (int64_t)(int)ceil(aa / area);
    if (M == 0) M = 1;
    int64_t total_verts = ring_off[n_rings] - ring_off[0];
    if (M < total_verts) M = total_verts;
    M += 12;
    /* _getEdgeHexagons over the shell and the holes */
    int64_t n_search = 0, search_cap = 1024;
    int64_t* search = (int64_t*)malloc((size_t)search_cap * 8);
    Set64 seen;
    set_init(&seen, 1024);
    for (int r = 0; r < n_rings; r++) {
        const int64_t s = ring_off[r], e = ring_off[r + 1], nv = e - s;
        for (int64_t i = 0; i < nv; i++) {
            const int64_t i2 = i == nv - 1 ? s : s + i + 1;
            const double olat = lat[s + i], olon = lon[s + i], dlat = lat[i2], dlon = lon[i2];
            int est = (int)ceil(dist_km(olat, olon, dlat, dlon) / (2 * pr));
            if (est == 0) est = 1;
            for (int j = 0; j < est; j++) {
                double la = (olat * (est - j) / est) + (dlat * j / est);
                double lo = (olon * (est - j) / est) + (dlon * j / est);
                int64_t hx = oracle_h3_geo_to_h3(la, lo, res);
                if (hx == 0 || !set_add(&seen, hx)) continue;
                if (seen.cap < 4 * (n_search + 16)) { /* grow */
                    Set64 g;
                    set_init(&g, 4 * (n_search + 16));
                    for (int64_t t = 0; t < seen.cap; t++)
                        if (seen.k[t]) set_add(&g, seen.k[t]);
                    free(seen.k);
                    seen = g;
                }
                if (n_search == search_cap) {
                    search_cap *= 2;
                    search = (int64_t*)realloc(search, (size_t)search_cap * 8);
                }
                search[n_search++] = hx;
            }
        }
    }
    free(seen.k);
    /* breadth-first rounds */
    Set64 acc;
    set_init(&acc, M);
    int64_t n_res = 0, res_cap = 1024;
    int64_t* acc_list = (int64_t*)malloc((size_t)res_cap * 8);
    int64_t* found = NULL;
    int64_t n_found = 0, found_cap = 0;
    int fail = 0;
    while (n_search > 0 && !fail) {
        n_found = 0;
        for (int64_t i = 0; i < n_search && !fail; i++) {
            int64_t ring[12];
            int m = ring1(search[i], res, ring);
            for (int j = 0; j < m; j++) {
                if (set_has(&acc, ring[j])) continue;
                double clat, clon;
                oracle_h3_to_geo(ring[j], &clat, &clon);
                if (!part_inside(&part, clat, clon)) continue;
                if (set_add(&acc, ring[j]) < 0) {
                    fail = 1;
                    break;
                }
                if (n_found == found_cap) {
                    found_cap = found_cap ? 2 * found_cap : 1024;
                    found = (int64_t*)realloc(found, (size_t)found_cap * 8);
                }
                found[n_found++] = ring[j];
                if (n_res == res_cap) {
                    res_cap *= 2;
                    acc_list = (int64_t*)realloc(acc_list, (size_t)res_cap * 8);
                }
                acc_list[n_res++] = ring[j];
            }
        }
        int64_t* t = search;
        search = found;
        found = t;
        int64_t tc = search_cap;
        search_cap = found_cap;
        found_cap = tc;
        n_search = n_found;
    }
    free(search);
    free(found);
    free(acc.k);
    free(boxes);
    if (fail || n_res > cap) {
        free(acc_list);
        return -1;
    }
    /* H3's output table: home slot cell % M, linear probing, in acceptance order */
    int64_t* slots = (int64_t*)calloc((size_t)M, 8);
    for (int64_t i = 0; i < n_res; i++) {
        int64_t loc = (int64_t)((uint64_t)acc_list[i] % (uint64_t)M);
        if (slots[loc] != 0) *collision_free = 0;
        while (slots[loc] != 0) loc = (loc + 1) % M;
        slots[loc] = acc_list[i];
    }
    int64_t n = 0;
    for (int64_t i = 0; i < M; i++)
        if (slots[i]) out[n++] = slots[i];
    free(slots);
    free(acc_list);
    return n;
}

/* ---- BNG ---- */
/* JTS 1.19 Orientation.isCCW(ring) (ring closed: n points, last == first) */
static int jts_is_ccw(const double* xy, int64_t n) {
    int64_t npts = n - 1;
    if (npts < 3) return 0;
    int64_t up_hi = 0, up_low = -1;
    double prev_y = xy[1], hi_y = xy[1];
    for (int64_t i = 1; i <= npts; i++) {
        double py = xy[2 * i + 1];
        if (py > prev_y && py >= hi_y) {
            up_hi = i;
            hi_y = py;
            up_low = i - 1;
        }
        prev_y = py;
    }
    if (up_hi == 0) return 0;
    int64_t down_low = up_hi;
    do {
        down_low = (down_low + 1) % npts;
    } while (down_low != up_hi && xy[2 * down_low + 1] == hi_y);
    int64_t down_hi = down_low > 0 ? down_low - 1 : npts - 1;
#define EQ2(a, b) (xy[2 * (a)] == xy[2 * (b)] && xy[2 * (a) + 1] == xy[2 * (b) + 1])
    if (EQ2(up_hi, down_hi)) {
        if (EQ2(up_low, up_hi) || EQ2(down_low, up_hi) || EQ2(up_low, down_low)) return 0;
        return oracle_orientation_index(xy[2 * up_low], xy[2 * up_low + 1], xy[2 * up_hi], xy[2 * up_hi + 1],
                                        xy[2 * down_low], xy[2 * down_low + 1]) == 1;
    }
#undef EQ2
    return xy[2 * down_hi] - xy[2 * up_hi] < 0;
}

/* JTS 1.19 Centroid.getCentroid of a polygonal geometry (area part; every shell resets the
 * triangle-fan base point); 0 if the area is 0 (the reference then takes the line centroid, not
 * restated: such geometries are reported as unsupported) */
int oracle_jts_centroid(const oracle_geom* g, double* cx, double* cy) {
    double sx = 0, sy = 0, a2 = 0, bx = 0, by = 0;
    for (int64_t p = 0; p < g->n_parts; p++)
        for (int64_t r = g->part_rings[p]; r < g->part_rings[p + 1]; r++) {
            const double* xy = g->xy + 2 * g->ring_offsets[r];
            int64_t n = g->ring_offsets[r + 1] - g->ring_offsets[r];
            if (n == 0) continue;
            int shell = r == g->part_rings[p];
            if (shell) {
                bx = xy[0];
                by = xy[1];
            }
            int ccw = jts_is_ccw(xy, n);
            double sign = (shell ? !ccw : ccw) ? 1.0 : -1.0;
            for (int64_t i = 0; i + 1 < n; i++) {
                double p1x = xy[2 * i], p1y = xy[2 * i + 1], p2x = xy[2 * i + 2], p2y = xy[2 * i + 3];
                double tcx = bx + p1x + p2x, tcy = by + p1y + p2y;
                double area2 = (p1x - bx) * (p2y - by) - (p2x - bx) * (p1y - by);
                sx += sign * area2 * tcx;
                sy += sign * area2 * tcy;
                a2 += sign * area2;
            }
        }
    if (!(fabs(a2) > 0.0)) return 0;
    *cx = sx / 3 / a2;
    *cy = sy / 3 / a2;
    return 1;
}

static int queue_push(int64_t** q, int64_t* n, int64_t* cap, int64_t v) {
    if (*n == *cap) {
        *cap *= 2;
        int64_t* t = (int64_t*)realloc(*q, (size_t)*cap * 8);
        if (!t) return 0;
        *q = t;
    }
    (*q)[(*n)++] = v;
    return 1;
}

static int set_add_grow(Set64* s, int64_t v, int64_t size_hint) {
    if (s->cap < 4 * (size_hint + 16)) {
        Set64 g;
        if (!set_init(&g, 4 * (size_hint + 16))) return -1;
        for (int64_t t = 0; t < s->cap; t++)
            if (s->k[t]) set_add(&g, s->k[t]);
        free(s->k);
        *s = g;
    }
    return set_add(s, v);
}

/* Returns the number of cells (in breadth-first order) written to out; -1 on overflow of cap, a NaN
 * vertex or a geometry without area. */
int64_t oracle_bng_polyfill(const oracle_geom* g, int res, int64_t* out, int64_t cap) {
    const int64_t v0 = g->ring_offsets[g->part_rings[0]], v1 = g->ring_offsets[g->part_rings[g->n_parts]];
    if (v1 == v0) return 0;
    Set64 visited;
    set_init(&visited, 1024);
    int64_t qcap = 1024, nq = 0, n = 0;
    int64_t* queue = (int64_t*)malloc((size_t)qcap * 8);
    int err = 0;
    double cx, cy;
    if (!oracle_jts_centroid(g, &cx, &cy)) goto fail;
    for (int64_t v = v0; v <= v1; v++) {
        double x = v < v1 ? g->xy[2 * v] : cx, y = v < v1 ? g->xy[2 * v + 1] : cy;
        int64_t c = oracle_bng_point_to_index(x, y, res, &err);
        if (err) goto fail;
        if (set_add_grow(&visited, c, nq) == 1 && !queue_push(&queue, &nq, &qcap, c)) goto fail;
    }
    for (int64_t head = 0; head < nq; head++) {
        int32_t o[4];
        if (!oracle_bng_cell_origin(queue[head], o)) continue;
        const double px = (double)o[2] + (double)o[1] / 2, py = (double)o[3] + (double)o[1] / 2;
        if (!oracle_contains(g, px, py)) continue;
        if (n >= cap) goto fail;
        out[n++] = queue[head];
        int64_t nb[8];
        int m = oracle_bng_kloop(queue[head], 1, nb);
        for (int j = 0; j < m; j++)
            if (set_add_grow(&visited, nb[j], nq) == 1 && !queue_push(&queue, &nq, &qcap, nb[j])) goto fail;
    }
    free(queue);
    free(visited.k);
    return n;
fail:
    free(queue);
    free(visited.k);
    return -1;
}

/* getBufferRadius (H3IndexSystem.scala:73-80): the cell of the geometry's JTS centroid
 * (h3.geoToH3(centroid.y, centroid.x) through Math.toRadians), its indexToGeometry polygon
 * (h3ToGeoBoundary through Math.toDegrees, closed with the first vertex), that polygon's JTS
 * centroid, the largest Coordinate.distance of a ring point from it.  NaN without area. */
static double to_degrees(double rad, int jdk) { return jdk <= 8 ? rad * 180.0 / M_PI : rad * 57.29577951308232; }

double oracle_h3_buffer_radius(const oracle_geom* g, int res, int jdk) {
    double cx, cy;
    if (!oracle_jts_centroid(g, &cx, &cy)) return NAN;
    int64_t cell = oracle_h3_geo_to_h3(oracle_to_radians(cy, jdk), oracle_to_radians(cx, jdk), res);
    double v[20], xy[22];
    int nv = oracle_h3_to_geo_boundary(cell, v);
    for (int k = 0; k < nv; k++) {
        xy[2 * k] = to_degrees(v[2 * k + 1], jdk);
        xy[2 * k + 1] = to_degrees(v[2 * k], jdk);
    }
    xy[2 * nv] = xy[0];
    xy[2 * nv + 1] = xy[1];
    int64_t ro[2] = {0, nv + 1}, pr[2] = {0, 1};
    oracle_geom hex = {xy, ro, pr, 1};
    double hx, hy;
    if (!oracle_jts_centroid(&hex, &hx, &hy)) return NAN;
    double r = 0;
    for (int k = 0; k <= nv; k++) {
        double dx = xy[2 * k] - hx, dy = xy[2 * k + 1] - hy, d = sqrt(dx * dx + dy * dy);
        if (d > r) r = d;
    }
    return r;
}
