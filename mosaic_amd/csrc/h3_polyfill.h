// H3 polyfill pieces shared by the device kernels and the host side of mosaic_polyfill: the
// reference's H3IndexSystem.polyfill = h3.polyfill(shell, holes, res) per polygon part
// (core/index/H3IndexSystem.scala:113-126) -> H3 C v3.7 algos.c _polyfillInternal.
//
// H3 C v3.7 restated (radians; glibc 2.35 sin / cos / atan2 via glibc_math.h, so host and device
// give the same bits as the reference's glibc-linked H3):
//   geoCoord.c   pointDistRads / pointDistKm (haversine)
//   bbox.c       bboxContains, bboxIsTransmeridian, bboxHexEstimate, lineHexEstimate
//   polygonAlgos.h bboxFromGeofence (GENERIC_LOOP_ALGO(bbox)), pointInsideGeofence
//                (GENERIC_LOOP_ALGO(pointInside): westerly DBL_EPSILON tie-break that persists
//                along the loop, NORMALIZE_LON for transmeridian loops)
//   polygon.c    pointInsidePolygon (shell, then holes)
//   algos.c      maxPolyfillSize (+ POLYFILL_BUFFER 12), _getEdgeHexagons' interpolation
//   h3Index.c    getPentagonIndexes (pentagon 0 = base cell 4), _hexRadiusKm
#pragma once
#include <float.h>
#include <math.h>
#include <stdint.h>

#include "h3_geom.h"
#include "h3_grid.h"
#include "h3_neighbors.h"

namespace mosaic {
namespace h3fill {

constexpr double kEarthRadiusKm = 6371.007180918475;
constexpr int kPolyfillBuffer = 12;

struct Box {
    double north, south, east, west;
};

// geoCoord.c H3_EXPORT(pointDistRads)
MOSAIC_HD double point_dist_rads(double alat, double alon, double blat, double blon) {
    double sin_lat, c0, sin_lng, c1, s2, cos_a, s3, cos_b;
    glibc::sincos((blat - alat) / 2.0, &sin_lat, &c0);
    glibc::sincos((blon - alon) / 2.0, &sin_lng, &c1);
    glibc::sincos(alat, &s2, &cos_a);
    glibc::sincos(blat, &s3, &cos_b);
    const double A = sin_lat * sin_lat + cos_a * cos_b * sin_lng * sin_lng;
    return 2 * glibc::atan2(sqrt(A), sqrt(1 - A));
}
MOSAIC_HD double point_dist_km(double alat, double alon, double blat, double blon) {
    return point_dist_rads(alat, alon, blat, blon) * kEarthRadiusKm;
}

// h3Index.c setH3Index(res, baseCell 4, digit 0): getPentagonIndexes(res)[0]
MOSAIC_HD uint64_t pentagon0(int res) {
    uint64_t h = (uint64_t)1 << 59 | (uint64_t)res << 52 | (uint64_t)4 << 45;
    for (int r = res + 1; r <= 15; r++) h |= (uint64_t)7 << ((15 - r) * 3);
    return h;
}

// bbox.c _hexRadiusKm(pentagons[0]): centre to the first boundary vertex
MOSAIC_HD double pentagon_radius_km(int res) {
    const uint64_t p = pentagon0(res);
    double clat, clon, v[20];
    h3geom::h3_to_geo(p, &clat, &clon);
    h3geom::h3_to_geo_boundary(p, v);
    return point_dist_km(clat, clon, v[0], v[1]);
}

// bbox.c lineHexEstimate
MOSAIC_HD int line_hex_estimate(double olat, double olon, double dlat, double dlon, double pent_radius_km) {
    const double dist = point_dist_km(olat, olon, dlat, dlon);
    int estimate = (int)ceil(dist / (2 * pent_radius_km));
    if (estimate == 0) estimate = 1;
    return estimate;
}

// bbox.c bboxHexEstimate
MOSAIC_HD int bbox_hex_estimate(const Box& b, double pent_radius_km) {
    const double pent_area_km2 = 0.8 * (2.59807621135 * pent_radius_km * pent_radius_km);
    const double d = point_dist_km(b.north, b.east, b.south, b.west);
    const double a = d * d / fmin(3.0, fabs((b.east - b.west) / (b.north - b.south)));
    int estimate = (int)ceil(a / pent_area_km2);
    if (estimate == 0) estimate = 1;
    return estimate;
}

// polygonAlgos.h GENERIC_LOOP_ALGO(bbox) over a Geofence of n (lat, lon) vertices
MOSAIC_HD Box bbox_from_loop(const double* lat, const double* lon, int64_t n) {
    if (n == 0) return Box{0, 0, 0, 0};
    Box b{-DBL_MAX, DBL_MAX, -DBL_MAX, DBL_MAX};
    double min_pos_lon = DBL_MAX, max_neg_lon = -DBL_MAX;
    bool transmeridian = false;
    for (int64_t i = 0; i < n; i++) {
        const double la = lat[i], lo = lon[i];
        const double next_lo = lon[i + 1 == n ? 0 : i + 1];
        if (la < b.south) b.south = la;
        if (lo < b.west) b.west = lo;
        if (la > b.north) b.north = la;
        if (lo > b.east) b.east = lo;
        if (lo > 0 && lo < min_pos_lon) min_pos_lon = lo;
        if (lo < 0 && lo > max_neg_lon) max_neg_lon = lo;
        if (fabs(lo - next_lo) > M_PI) transmeridian = true;
    }
    if (transmeridian) {
        b.east = max_neg_lon;
        b.west = min_pos_lon;
    }
    return b;
}

MOSAIC_HD bool bbox_is_transmeridian(const Box& b) { return b.east < b.west; }

MOSAIC_HD bool bbox_contains(const Box& b, double lat, double lon) {
    return lat >= b.south && lat <= b.north &&
           (bbox_is_transmeridian(b) ? (lon >= b.west || lon <= b.east) : (lon >= b.west && lon <= b.east));
}

MOSAIC_HD double normalize_lon(double lon, bool tm) { return tm && lon < 0 ? lon + (double)(2 * M_PI) : lon; }

// polygonAlgos.h GENERIC_LOOP_ALGO(pointInside) for a Geofence (the loop's closing edge included)
MOSAIC_HD bool point_inside_loop(const double* lat, const double* lon, int64_t n, const Box& b, double plat,
                                 double plon) {
    if (!bbox_contains(b, plat, plon)) return false;
    const bool tm = bbox_is_transmeridian(b);
    bool contains = false;
    double lng = normalize_lon(plon, tm);
    for (int64_t i = 0; i < n; i++) {
        const int64_t j = i + 1 == n ? 0 : i + 1;
        double alat = lat[i], alon = lon[i], blat = lat[j], blon = lon[j];
        if (alat > blat) {
            double t = alat;
            alat = blat;
            blat = t;
            t = alon;
            alon = blon;
            blon = t;
        }
        if (plat < alat || plat > blat) continue;
        const double a_lng = normalize_lon(alon, tm), b_lng = normalize_lon(blon, tm);
        if (a_lng == lng || b_lng == lng) lng -= DBL_EPSILON;
        const double ratio = (plat - alat) / (blat - alat);
        const double test_lng = normalize_lon(a_lng + (b_lng - a_lng) * ratio, tm);
        if (test_lng > lng) contains = !contains;
    }
    return contains;
}

// _getEdgeHexagons: sample j of numHexesEstimate n along the edge origin -> destination
MOSAIC_HD void edge_sample(double olat, double olon, double dlat, double dlon, int n, int j, double* lat,
                           double* lon) {
    *lat = (olat * (n - j) / n) + (dlat * j / n);
    *lon = (olon * (n - j) / n) + (dlon * j / n);
}

MOSAIC_HD void unit3(double lat, double lon, double* v) {
    double sl, cl, so, co;
    glibc::sincos(lat, &sl, &cl);
    glibc::sincos(lon, &so, &co);
    v[0] = cl * co;
    v[1] = cl * so;
    v[2] = sl;
}

// kRing(h, 1) as polyfill's search uses it (H3 v3.7 _polyfillInternal: kRing(searchHex, 1, ring)
// and the ring's non-zero entries in array order): H3's hexRange order where the walk succeeds,
// else its _kRingInternal table of maxKringSize(1) = 7 slots read in slot order (h3_neighbors.h).
// Returns the cell count (5 or 7 with a pentagon in reach; -1 for an invalid index).
MOSAIC_HD int kring1(uint64_t h, int res, int64_t* out) {
    (void)res;
    const int n = h3nb::kring_fast(h, 1, 0, out);
    if (n != -3) return n < 0 ? -1 : n;
    int64_t tab[8];
    int32_t dist[7];
    return h3nb::kring_slow(h, 1, 0, out, tab, dist);
}

}  // namespace h3fill
}  // namespace mosaic
