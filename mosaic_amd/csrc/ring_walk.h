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

}  // namespace ringwalk
}  // namespace mosaic
