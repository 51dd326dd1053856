/*
 * TEST INFRASTRUCTURE ONLY -- the CPU oracle for the Mosaic PIP chip-join hot path.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker (or the timed CPU baseline), never as the product.  The product is
 * libmosaic_hip.so (mosaic_amd/csrc); it never links or calls anything here.
 *
 * Restated algorithms (each function cites what it follows):
 *   h3.c    H3 v3.7 geoToH3 as called by H3IndexSystem.pointToIndex
 *           (reference src/main/scala/com/databricks/labs/mosaic/core/index/H3IndexSystem.scala:140-142).
 *           H3 itself (com.uber:h3:3.7.0, reference pom.xml:91-97) is absent from the reference and
 *           from this image: the published algorithm is restated; constants come from
 *           mosaic_amd/csrc/h3_tables.h (tools/h3gen.py).  Pinned by the known answers in
 *           tests/test_oracle_h3.py.
 *   bng.c   BNGIndexSystem.pointToIndex / getQuadrant / encode / format
 *           (reference core/index/BNGIndexSystem.scala:114-129, 277-327, 528-541).  Pinned by the
 *           reference's golden vectors (TestBNGIndexSystem.scala:10-90).
 *   pip.c   JTS 1.19 Geometry.contains(Point) for Polygon/MultiPolygon chips (MosaicGeometryJTS.scala:101,
 *           ST_Contains.scala:34-42): PointLocator (Mod-2 boundary rule), RayCrossingCounter,
 *           CGAlgorithmsDD.orientationIndex (FP filter + double-double).  Pinned by
 *           ST_ContainsBehaviors.scala:22-36 and an exact rational checker (oracle/exact.py).
 *   join.c  The Quickstart chip join: cell = pointToIndex(point); pairs with every chip whose
 *           index_id == cell and (is_core OR st_contains(chip.wkb, point))
 *           (notebooks/examples/python/QuickstartNotebook.py:205-219, PointInPolygonJoin.scala:68-84).
 */
#ifndef MOSAIC_ORACLE_H
#define MOSAIC_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- H3 ---- */
/* H3 C geoToH3(lat, lng in radians, res); 0 (H3_NULL) for res out of range or non-finite input. */
int64_t oracle_h3_geo_to_h3(double lat_rad, double lng_rad, int res);
/* java.lang.Math.toRadians: jdk==8 -> deg / 180.0 * PI; jdk>=9 -> deg * DEGREES_TO_RADIANS. */
double oracle_to_radians(double deg, int jdk);
/* H3IndexSystem.pointToIndex(lon, lat, res) = h3.geoToH3(lat, lon, res) through h3-java. */
void oracle_h3_point_to_index(const double* lon, const double* lat, int64_t n, int res, int jdk,
                              int64_t* out);
/* Intermediate state of geoToH3 for diagnostics: face, hex2d x/y, res ijk. */
/* The host libm H3 C reaches: fn 0 sin, 1 cos (via sincos), 2 tan, 3 acos, 4 atan2(a, b). */
void oracle_libm_eval(int fn, const double* a, const double* b, int64_t n, double* out);
/* h3ToGeo (radians) and kRing as a set found on the sphere (oracle of the H3 k-ring kernels) */
void oracle_h3_to_geo(int64_t h3, double* lat, double* lon);
int64_t oracle_h3_kring_set(int64_t h3, int k, int64_t* out, int32_t* dist, int64_t cap);
int oracle_h3_is_pentagon(int64_t h3);
int oracle_h3_to_geo_boundary(int64_t h3, double* out);
void oracle_h3_debug(double lat_rad, double lng_rad, int res, int* face, double* x, double* y,
                     int* ijk);

/* ---- BNG ---- */
/* BNGIndexSystem.pointToIndex; returns 0 and sets *err=1 for NaN input (IllegalStateException). */
int64_t oracle_bng_point_to_index(double eastings, double northings, int res, int* err);
void oracle_bng_point_to_index_batch(const double* e, const double* n, int64_t count, int res,
                                     int64_t* out, uint8_t* err);
/* BNGIndexSystem.format: writes a NUL-terminated string; returns its length or -1. */
int oracle_bng_format(int64_t id, char* buf, int cap);
/* BNGIndexSystem.parse: 1 and *out, or 0 where the reference throws. */
int oracle_bng_parse(const char* s, int n, int64_t* out);
/* BNGIndexSystem.isValid / kLoop / kRing: cell count written to out (<= 8k / 1 + 4k(k+1)), -1 if
 * the id cannot be decoded. */
int oracle_bng_is_valid(int64_t id);
int oracle_bng_kloop(int64_t id, int k, int64_t* out);
int oracle_bng_kring(int64_t id, int n, int64_t* out);
/* (resolution, edge, x, y) of a cell for indexToGeometry; 0 if undecodable. */
int oracle_bng_cell_origin(int64_t id, int32_t* out4);

/* ---- JTS contains ---- */
/* Geometry described as rings: ring_offsets[r]..ring_offsets[r+1] index into xy (pairs);
 * part_rings[p]..part_rings[p+1] index rings of polygon part p (first ring = shell). */
typedef struct {
    const double* xy;            /* interleaved x,y */
    const int64_t* ring_offsets; /* n_rings + 1, in vertices */
    const int64_t* part_rings;   /* n_parts + 1, in rings */
    int64_t n_parts;
} oracle_geom;
/* 1 iff JTS Geometry.contains(geom, POINT(px py)). */
int oracle_contains(const oracle_geom* g, double px, double py);
/* JTS Orientation.index(p1, p2, q): 1 left, -1 right, 0 collinear. */
int oracle_orientation_index(double p1x, double p1y, double p2x, double p2y, double qx, double qy);
/* WKB (either byte order; Polygon, MultiPolygon, empty) -> contains. Returns -1 on parse error. */
int oracle_wkb_contains(const uint8_t* wkb, int64_t len, double px, double py);
void* oracle_wkb_parse(const uint8_t* wkb, int64_t len);
int oracle_parsed_contains(const void* parsed, double px, double py);
void oracle_parsed_free(void* parsed);
/* JTS RobustLineIntersector: closed segments p1p2 and q1q2 share a point (1) or not (0). */
int oracle_segments_intersect(double p1x, double p1y, double p2x, double p2y, double q1x, double q1y, double q2x,
                              double q2y);
/* JTS Geometry.intersects of two polygonal geometries (closed point sets share a point). */
int oracle_intersects(const oracle_geom* a, const oracle_geom* b);
/* The same from two WKBs; -1 on parse error. */
int oracle_wkb_intersects(const uint8_t* wa, int64_t la, const uint8_t* wb, int64_t lb);

/* ---- grid_polyfill (polyfill.c) ---- */
/* H3 polyfill of one polygon part (rings [0, n_rings) in lat / lon radians, ring_off[n_rings + 1]);
 * cells in H3's output-slot order; *collision_free = 0 when probing displaced a cell (then only the
 * set is certain).  -1: cap too small. */
int64_t oracle_h3_polyfill(const double* lat, const double* lon, const int64_t* ring_off, int n_rings, int res,
                           int64_t* out, int64_t cap, int* collision_free);
/* kRing(h, 1) as a set from the cell geometry (h first). */
int oracle_h3_ring1(int64_t h, int64_t* out);
/* JTS Centroid of a polygonal geometry (area-weighted); 0 when its area is 0. */
int oracle_jts_centroid(const oracle_geom* g, double* cx, double* cy);
/* H3 getBufferRadius of a geometry (degrees); NaN without area. */
double oracle_h3_buffer_radius(const oracle_geom* g, int res, int jdk);
/* BNG polyfill of a geometry: cells in breadth-first order; -1 on cap overflow / NaN / no area. */
int64_t oracle_bng_polyfill(const oracle_geom* g, int res, int64_t* out, int64_t cap);

/* ---- chip join ---- */
typedef struct {
    int64_t n_chips;
    const int64_t* index_id;
    const uint8_t* is_core;
    const int32_t* polygon_key;
    const int64_t* wkb_offsets; /* n_chips + 1 */
    const uint8_t* wkb;
} oracle_chips;
/* grid: 0 = H3, 1 = BNG.  counts[n_polygons] += matched pairs per polygon key.
 * If pair_row/pair_key are non-null, writes up to cap pairs (row, key) in row-major chip order.
 * Returns number of pairs. */
int64_t oracle_pip_join(const oracle_chips* chips, int grid, int res, int jdk, const double* x,
                        const double* y, int64_t n, int64_t* counts, int64_t n_polygons,
                        int64_t* pair_row, int32_t* pair_key, int64_t cap, int n_threads);
/* Brute force: every geometry (chips->wkb, keyed by polygon_key; is_core ignored) against every point. */
int64_t oracle_brute_force_count(const oracle_chips* geoms, const double* x, const double* y, int64_t n,
                                 int64_t* counts, int64_t n_polygons);

#ifdef __cplusplus
}
#endif
#endif
