// Point-in-ring walks of the tile join (join_binned.hip k_join_tiles) on LDS vertex images: JTS
// PointLocation.locateInRing == INTERIOR, exactly (pip_device.h's RayCrossingCounter and
// CGAlgorithmsDD orientation).  Host-compilable for tests/native/ring_walk_check.cpp.
#pragma once
#include <math.h>
#include <stdint.h>

#include "pip_device.h"

#if defined(__HIPCC__)
#define MOSAIC_NOINLINE __device__ __noinline__
#else
#define MOSAIC_NOINLINE static inline
#endif

namespace mosaic {
namespace ringwalk {

struct alignas(16) V2 {
    double x, y;
};

// PointLocation.locateInRing(p, ring) == INTERIOR for a closed ring of n vertices (x, y pairs):
// pip::locate_in_ring's RayCrossingCounter steps and CGAlgorithmsDD orientation, operation for
// operation.  A point outside the ring's envelope gets EXTERIOR from the walk itself (no crossing
// counted twice), so the envelope pre-test of locate_in_polygon changes no answer.
MOSAIC_NOINLINE bool ring_interior_exact(const double* v, uint32_t n, double px, double py) {
    int crossings = 0;
    double p2x = v[0], p2y = v[1];
    for (uint32_t i = 1; i < n; i++) {
        const double p1x = v[2 * i], p1y = v[2 * i + 1];
        if (!(p1x < px && p2x < px)) {
            if (px == p2x && py == p2y) return false;
            if (p1y == py && p2y == py) {
                const double mnx = p1x < p2x ? p1x : p2x, mxx = p1x < p2x ? p2x : p1x;
                if (px >= mnx && px <= mxx) return false;
            } else if (((p1y > py) && (p2y <= py)) || ((p2y > py) && (p1y <= py))) {
                int orient = pip::orientation_index(p1x, p1y, p2x, p2y, px, py);
                if (orient == 0) return false;
                if (p2y < p1y) orient = -orient;
                if (orient == 1) crossings++;
            }
        }
        p2x = p1x;
        p2y = p1y;
    }
    return crossings & 1;
}

// The same answer without per-edge branches: every edge evaluates its flags and the orientation's
// floating-point filter (CGAlgorithmsDD.orientationIndexFilter); a "boundary" flag replaces the
// early returns (the answer is false once it is set, as there).  A lane whose straddling edge the
// filter cannot decide takes ring_interior_exact (the double-double orientation).
MOSAIC_HD bool ring_interior(const double* v, uint32_t n, double px, double py) {
    bool on = false, slow = false;
    uint32_t cross = 0;
    const V2* w = (const V2*)v;
    V2 p2 = w[0];
    for (uint32_t i = 1; i < n; i++) {
        const V2 p1 = w[i];
        const bool right = !(p1.x < px && p2.x < px);
        const bool vert = px == p2.x && py == p2.y;
        const bool horiz = p1.y == py && p2.y == py;
        const bool on_h = horiz && px >= fmin(p1.x, p2.x) && px <= fmax(p1.x, p2.x);
        const bool strad = !horiz && ((p1.y > py) != (p2.y > py));
        const double dl = (p1.x - px) * (p2.y - py), dr = (p1.y - py) * (p2.x - px), det = dl - dr;
        const bool same = (dl > 0.0 && dr > 0.0) || (dl < 0.0 && dr < 0.0);
        const bool ok = !same || fabs(det) >= 1e-15 * fabs(dl + dr);
        const int o = (det > 0.0) - (det < 0.0);
        const bool use = right && !vert && strad;
        slow |= use && !ok;
        on |= right && (vert || on_h || (strad && o == 0));
        cross += (use && ((p2.y < p1.y) ? -o : o) == 1) ? 1u : 0u;
        p2 = p1;
    }
    if (slow) return ring_interior_exact(v, n, px, py);
    return !on && (cross & 1u);
}

// ---- the f32 walk: the same decisions from single-precision differences, each certified by an
// error bound or reported undecided (the caller then takes a double-precision walk).
// Frame: coordinates relative to the chip's outward-rounded f32 envelope minimum (fminx, fminy),
// vertices stored as float(v - fmin) (round to nearest), the point as float(p - fmin) with p - fmin
// in double.  M bounds |relative coordinate| of the vertices (within the f32 envelope) and of a
// point that passed the f32 envelope test (float(p) within the envelope, |p - float(p)| <= 2^-24
// |p| <= 1.1e-5 for |p| <= 184).  Each stored / converted value is within u M of the exact
// difference (u = 2^-24), so a computed difference d = fl(a - q), |a - q| <= 2M, is within
// 2uM + 2uM = 4uM of the exact one: |d| > tol = 5uM fixes its sign (and with it JTS's strict
// comparisons p1.y > p.y, p1.x < p.x).  The orientation determinant x1 y2 - y1 x2 of such
// differences (|.| <= 2M) is within 2 (2M 4uM + 2M 4uM) (products of perturbed factors)
// + 2 u 4M^2 (product roundings) + u 8M^2 (subtraction) = 48uM^2 of the exact one: |det| > 52uM^2
// fixes its sign.  Constants are rounded up.
struct F32Frame {
    float qx, qy, tol, bound;
};
MOSAIC_HD F32Frame f32_frame(float fminx, float fminy, float fmaxx, float fmaxy, double px, double py) {
    F32Frame f;
    const float m = fmaxf(fmaxx - fminx, fmaxy - fminy) * 1.000001f + 1.1e-5f;
    f.qx = (float)(px - (double)fminx);
    f.qy = (float)(py - (double)fminy);
    f.tol = m * 3.0e-7f;          // 5 u M
    f.bound = m * m * 3.2e-6f;    // 52 u M^2
    return f;
}

// 1: interior, 0: not, 2: undecided (an edge whose decisions the bounds cannot certify: the
// point near a vertex's y, an edge's x, or an edge's line).  JTS's walk with p1 = v[i], p2 = v[i-1]:
// an edge with both ends certainly left of the point, or both certainly above / below its y, is
// skipped (as there, where such an edge changes nothing); a certainly straddling edge with a
// certain orientation counts a crossing as there; any other edge leaves the answer undecided
// (which covers every boundary case: vertex, horizontal edge, point on an edge).
MOSAIC_HD int ring_interior_f32(const float* v, uint32_t n, const F32Frame& f) {
    bool amb = false;
    uint32_t cross = 0;
    float x2 = v[0] - f.qx, y2 = v[1] - f.qy;
    for (uint32_t i = 1; i < n; i++) {
        const float x1 = v[2 * i] - f.qx, y1 = v[2 * i + 1] - f.qy;
        const bool a1 = y1 > f.tol, b1 = y1 < -f.tol, a2 = y2 > f.tol, b2 = y2 < -f.tol;
        const bool skip = (x1 < -f.tol && x2 < -f.tol) || (a1 && a2) || (b1 && b2);
        const bool strad = (a1 && b2) || (b1 && a2);
        const float det = x1 * y2 - y1 * x2;
        const bool pos = det > f.bound, neg = det < -f.bound;
        amb |= !skip && !(strad && (pos || neg));
        // orientation sign(det), negated when p2.y < p1.y (p1 above): a crossing when the result is 1
        cross += (!skip && strad && (a1 ? neg : pos)) ? 1u : 0u;
        x2 = x1;
        y2 = y1;
    }
    return amb ? 2 : (int)(cross & 1u);
}
// ring_interior_f32 as a rolled loop that reads the next vertex one step ahead (the walk the tile join
// inlines: the unrolled form's registers made k_join_tiles spill, 152 bytes of scratch per lane).
// Same decisions edge by edge; v must hold n >= 1 vertices.
MOSAIC_HD int ring_interior_f32_rolled(const float* v, uint32_t n, const F32Frame& f) {
    bool amb = false;
    uint32_t cross = 0;
    float x2 = v[0] - f.qx, y2 = v[1] - f.qy;
    float nx = n > 1 ? v[2] : 0.0f, ny = n > 1 ? v[3] : 0.0f;
#pragma unroll 1
    for (uint32_t i = 1; i < n; i++) {
        const float x1 = nx - f.qx, y1 = ny - f.qy;
        const uint32_t j = i + 1 < n ? i + 1 : i;
        nx = v[2 * j];
        ny = v[2 * j + 1];
        const bool a1 = y1 > f.tol, b1 = y1 < -f.tol, a2 = y2 > f.tol, b2 = y2 < -f.tol;
        const bool skip = (x1 < -f.tol && x2 < -f.tol) || (a1 && a2) || (b1 && b2);
        const bool strad = (a1 && b2) || (b1 && a2);
        const float det = x1 * y2 - y1 * x2;
        const bool pos = det > f.bound, neg = det < -f.bound;
        amb |= !skip && !(strad && (pos || neg));
        cross += (!skip && strad && (a1 ? neg : pos)) ? 1u : 0u;
        x2 = x1;
        y2 = y1;
    }
    return amb ? 2 : (int)(cross & 1u);
}

}  // namespace ringwalk
}  // namespace mosaic
