// H3 grid rings (grid_cellkring / grid_cellkloop over H3 cells) on the device and the host: the
// reference's H3IndexSystem.kRing = h3.kRing(index, n) and kLoop = h3.hexRing(index, n)
// (core/index/H3IndexSystem.scala:154-177), i.e. H3 v3.7 hexRangeDistances / hexRing (algos.c).
//
// Integer-only.  H3's traversal (h3NeighborRotations with its base-cell neighbour and rotation
// tables) walks the ring in directions that it keeps geometrically fixed in the origin's frame by
// counting 60-degree rotations across base cells.  The same walk is taken here directly in that
// frame: the origin's FaceIJK before any overage adjustment (h3Index.c
// _h3ToFaceIjkWithInitializedFijk on the base cell's home face), stepped by the unit vectors of the
// direction digits, with every visited position turned into an index as H3 does for a cell centre
// (Class III: _downAp7r to the Class II substrate; _adjustOverageClassII onto the face that holds
// it; _upAp7r back; _faceIjkToH3).  Order: hexRange's (origin, then ring r = 1..k: one step along
// I without output, then r steps each along J, JK, K, IK, I, IJ) and hexRing's (the ring's start
// first, the walk without its closing step).
//
// Scope: hexRange / hexRing succeed exactly when no visited cell is a pentagon; otherwise H3
// falls back to _kRingInternal, whose output order is a hash-table order.  A row whose walk
// reaches a pentagon base cell, or a position needing more than one face change (only possible
// around an icosahedron vertex, i.e. a pentagon), is reported as unsupported (count -2), never
// answered approximately.  NYC / London / any region away from the 12 icosahedron vertices is
// fully covered.
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

// faceijk.c _adjustOverageClassII (substrate 0, pentLeading4 0): 0 no overage, 1 moved to a new face
MOSAIC_HD int adjust_overage(int& face, IJK& ijk, int res) {
    const int max_dim = max_dim_c2(res);
    if (ijk.i + ijk.j + ijk.k <= max_dim) return 0;
    int q;
    if (ijk.k > 0) q = ijk.j > 0 ? 3 : 2;  // JK : KI
    else q = 1;                            // IJ
    const int* o = kH3FaceNeighbors[face][q];
    face = o[0];
    for (int r = 0; r < o[4]; r++) rotate60ccw(ijk);
    const int s = unit_scale_c2(res);
    ijk = add(ijk, IJK{o[1] * s, o[2] * s, o[3] * s});
    h3::ijk_normalize(ijk);
    return 1;
}

// The index of the cell at `ijk` (res-`res` coordinates in face `face`'s frame, possibly beyond
// the face); 0 when it is unsupported (see the header).
MOSAIC_HD uint64_t cell_at(int face, IJK ijk, int res) {
    const bool c3 = (res & 1) != 0;
    int r2 = res;
    if (c3) {
        down_ap7r(ijk);
        r2++;
    }
    if (adjust_overage(face, ijk, r2) && adjust_overage(face, ijk, r2)) return 0;  // two face changes
    if (c3) up_ap7r(ijk);
    const uint64_t h = h3::face_ijk_to_h3(face, ijk, res);
    if (h == 0) return 0;
    const int bc = (int)((h >> 45) & 127);
    return h3::kH3BaseCellData[bc][4] ? 0 : h;
}

// Origin frame: the base cell's home FaceIJK plus the digits (_h3ToFaceIjkWithInitializedFijk).
// false for invalid cells and pentagon base cells.
MOSAIC_HD bool origin_frame(uint64_t h, int* face, IJK* ijk, int* res) {
    if (((h >> 59) & 15) != 1) return false;
    const int r = (int)((h >> 52) & 15), bc = (int)((h >> 45) & 127);
    if (bc >= 122 || h3::kH3BaseCellData[bc][4]) return false;
    IJK c{h3::kH3BaseCellData[bc][1], h3::kH3BaseCellData[bc][2], h3::kH3BaseCellData[bc][3]};
    for (int q = 1; q <= r; q++) {
        const int d = h3::get_digit(h, q);
        if (d == 7) return false;
        if (q & 1) down_ap7(c);  // Class III: ccw aperture 7
        else down_ap7r(c);
        if (d) {
            c = add(c, unit(d));
            h3::ijk_normalize(c);
        }
    }
    *face = h3::kH3BaseCellData[bc][0];
    *ijk = c;
    *res = r;
    return true;
}

// hexRange directions (algos.c DIRECTIONS) and NEXT_RING_DIRECTION (I)
MOSAIC_HD int ring_dir(int d) {
    const int t[6] = {2, 3, 1, 5, 4, 6};  // J, JK, K, IK, I, IJ
    return t[d];
}

// kRing (loop = 0: origin then rings 1..k, hexRangeDistances order; max 1 + 3k(k + 1) cells) or
// kLoop (loop = 1: hexRing order, 6k cells; k = 0: the origin).  Returns the cell count, or -2 when
// the row is unsupported (pentagon / vertex region) or the index is invalid.
MOSAIC_HD int kring(uint64_t origin, int k, int loop, int64_t* out) {
    int face, res;
    IJK p;
    if (!origin_frame(origin, &face, &p, &res)) return -2;
    if (loop && k == 0) {
        out[0] = (int64_t)origin;
        return 1;
    }
    int n = 0;
    if (!loop) out[n++] = (int64_t)origin;
    // hexRange walks every ring; hexRing only steps k times along I, then walks ring k
    for (int ring = loop ? k : 1; ring <= k; ring++) {
        for (int s = 0; s < (loop ? k : 1); s++) {
            p = add(p, unit(4));  // NEXT_RING_DIRECTION: I
            h3::ijk_normalize(p);
            if (!cell_at(face, p, res)) return -2;
        }
        if (loop) out[n++] = (int64_t)cell_at(face, p, res);
        for (int d = 0; d < 6; d++)
            for (int i = 0; i < ring; i++) {
                p = add(p, unit(ring_dir(d)));
                h3::ijk_normalize(p);
                const uint64_t c = cell_at(face, p, res);
                if (!c) return -2;
                if (!(loop && d == 5 && i == ring - 1)) out[n++] = (int64_t)c;
            }
    }
    return n;
}

}  // namespace h3grid
}  // namespace mosaic
