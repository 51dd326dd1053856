// H3 grid arithmetic shared by the neighbour traversal (h3_neighbors.h), the cell geometry
// (h3_geom.h) and polyfill (h3_polyfill.h): coordijk.c's aperture-7 steps and rotations, faceijk.c's
// Class II dimension tables, and the face-adjacency table (h3_face_tables.h, tools/h3gen_faces.py).
// Integer-only, device and host.
#pragma once
#include <stdint.h>

#include "h3_device.h"

namespace mosaic {
namespace h3grid {

#if defined(__HIPCC__)
#define H3_TABLE static __constant__ const
#else
#define H3_TABLE static const
#endif
#include "h3_face_tables.h"
#undef H3_TABLE

using h3::IJK;

// faceijk.c maxDimByCIIres / unitScaleByCIIres (Class II resolutions 0, 2, ..., 16)
MOSAIC_HD int max_dim_c2(int res) {
    int m = 2;
    for (int r = 0; r < res; r += 2) m *= 7;
    return m;
}
MOSAIC_HD int unit_scale_c2(int res) {
    int m = 1;
    for (int r = 0; r < res; r += 2) m *= 7;
    return m;
}

MOSAIC_HD IJK add(IJK a, IJK b) { return IJK{a.i + b.i, a.j + b.j, a.k + b.k}; }
// coordijk.c _ijkRotate60ccw: i -> (1, 1, 0), j -> (0, 1, 1), k -> (1, 0, 1)
MOSAIC_HD void rotate60ccw(IJK& c) {
    IJK r{c.i + c.k, c.i + c.j, c.j + c.k};
    h3::ijk_normalize(r);
    c = r;
}
// coordijk.c _downAp7 / _downAp7r / _upAp7r
MOSAIC_HD void down_ap7(IJK& c) {
    IJK r{3 * c.i + c.j, 3 * c.j + c.k, c.i + 3 * c.k};
    h3::ijk_normalize(r);
    c = r;
}
MOSAIC_HD void down_ap7r(IJK& c) {
    IJK r{3 * c.i + c.k, c.i + 3 * c.j, c.j + 3 * c.k};
    h3::ijk_normalize(r);
    c = r;
}
MOSAIC_HD void up_ap7r(IJK& c) {
    const int i = c.i - c.k, j = c.j - c.k;
    c.i = h3::round_div7(2 * i + j);  // lround((2 i + j) / 7.0): no ties
    c.j = h3::round_div7(3 * j - i);
    c.k = 0;
    h3::ijk_normalize(c);
}
// UNIT_VECS[digit] = (digit >> 2 & 1, digit >> 1 & 1, digit & 1)
MOSAIC_HD IJK unit(int digit) { return IJK{(digit >> 2) & 1, (digit >> 1) & 1, digit & 1}; }

}  // namespace h3grid
}  // namespace mosaic
