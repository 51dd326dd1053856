// Tile directory: the point side of the H3 chip join without the per-point H3 index arithmetic
// or the hash probe.
//
// The chip join needs, per point, the chips whose index_id equals the point's H3 cell
// (grid_pointascellid -> H3IndexSystem.pointToIndex, core/index/H3IndexSystem.scala:140-142, then
// the Quickstart equi-join, notebooks/examples/python/QuickstartNotebook.py:205-219).  The fast
// path (h3_device.h) certifies the hexagon (face, axial a, b) of a point; turning that into a
// 64-bit index (15 digit levels) and probing the chip hash is most of its integer work.  Here the
// lon/lat region around the chip cells is cut into tiles of ~4 hexagons a side.  Per tile the
// host proves (below) that every point of the tile lies on one icosahedron face, and records the
// window of axial coordinates its points can round to, with the chip-table slot of every hexagon
// in the window.  A point then costs: tile lookup, projection, rounding, one window read.
//
// Why it is exact (every condition is checked on the host while building; any doubt marks the
// tile kFull, which runs the unchanged h3_fast + probe path).  The map of a tile's points to its
// face plane, F(lon, lat) = S (EI.p, EP.p) / (FC.p) (hex units; p the unit vector, FC the face
// centre, EI / EP the plane's orthonormal axes), has derivatives bounded over the tile in closed
// form (TileCurv below).  From them:
//  * face: the 4 corners of the tile have the same closest face, with a dot-product gap >= 1e-4
//    to every other face.  Each gap (FC_f - FC_g).p has second derivatives <= |FC_f - FC_g| |p''|
//    <= 2 rad^-2 along lon and lat lines, so over a tile of <= 0.25 degrees it stays within
//    2 k^2 (tw^2 + th^2) / 8 < 1e-5 of the bilinear interpolant of its corner values (k = pi / 180),
//    which is >= the smallest corner gap: the whole tile is on the face.
//  * window: every image point lies within rect_tol(tile) <= 0.25 hex units of the bilinear patch
//    through the corner images, which lies in their convex hull; 0.25 hex units are < 0.29 in each
//    axial coordinate, and a point's hexagon centre is within 2/3 of its fractional axial
//    coordinates (the Voronoi hexagon's vertices are at axial offsets (2/3, 1/3) and rotations),
//    so the window [floor(min) - 1, floor(max) + 1] per axis (min / max over the samples) contains
//    every hexagon a tile point can have, under H3 or the fast path (their images differ by
//    < 1e-9 hex units).  A certified point outside the window (impossible by this argument)
//    still takes the index + probe path.
//  * skip: a tile whose window holds no chip cell is kSkip: none of its points can join.
//  * outside the grid: the grid is the region of the chip cells (from a rough cell -> lon/lat
//    inverse, placement only) widened by k tile rings, and every chip cell must be found in the
//    window of a tile T at least k rings inside the grid, with its hexagon at least 2/sqrt(3) hex
//    units inside the territory of T's face (the bisector lines with every other face in T's
//    plane).  A point P of such a cell whose closest face is T's rounds to that hexagon, so F(P)
//    lies within 1/sqrt(3) of its centre and within 2.5 hex units of T's image; F is expanding by
//    at least S k cos(lat_max) per degree (the gnomonic map expands the sphere, 1 / D >= 1, and
//    lon / lat -> sphere has singular values cos(lat) and 1), and k rings are >= 1.5 x 2.5 hex
//    units under that bound, so P is inside the grid.  P cannot have another closest face: H3's
//    grids of adjacent faces continue each other across the shared edge (the faceNeighbors ijk
//    transforms), so the cell's position on another face's grid is outside that face's triangle by
//    more than a rounding radius.  So a finite point outside the grid joins nothing.
//    Non-finite points take the full path (H3 returns 0 for them, which a chip could carry).
//
// HBM layout (per chip table): tile_idx u32[nx * ny] (kSkip, kFull or record + 2), TileRec 16 B
// per non-empty tile, u32 window entries (chip-hash slot + 1, 0 = no chips), row-major (a, b).
#pragma once
#include <math.h>
#include <stdint.h>

#include "h3_device.h"
#include "raster.h"
#include "raster_build.h"

#include <algorithm>
#include <atomic>
#include <functional>
#include <thread>
#include <vector>

namespace mosaic {
namespace tiles {

static const uint32_t kSkip = 0;  // no point of the tile can join
static const uint32_t kFull = 1;  // run the generic fast path + probe

// point raster codes (uint16): 0 = no pair, k + 1 = one pair with polygon key k (k + 1 < kSubBlock),
// kMixed = the points of the cell take the tile path.  Sub-block entries (uint16) are a code,
// kMixed, kSubBlock | n (n < kLineBit): the C x C leaf block at blocks[tile_base[tile] + n C^2],
// or kSubBlock | kLineBit | n: the line record at blocks[tile_base[tile] - 8 (n + 1)] (a tile's
// line records precede its leaf blocks, last first; tile_base counts uint16 elements and is a
// multiple of 8).  Sub-block line records are in the tile frame (rbuild::line_slack_tile): u, v
// are the point's offsets from the TILE's corner in leaf cells, and the sub-blocks one edge splits
// share one record.
static const uint16_t kMixed = 0xffffu;
static const uint16_t kSubBlock = 0x8000u;
static const uint16_t kLineBit = 0x4000u;
static const int32_t kMaxRasterKeys = 0x7ffd;  // polygon keys 0 .. kMaxRasterKeys - 1

// A sub-block split by one straight feature (a chip edge: a zone boundary or a hexagon side):
// s = a u + b v + c with (u, v) the point's offset from the tile's lower-left corner in leaf cells
// (0 <= u, v < S C; leaf lines: from the sub-block's corner, 0 <= u, v < C), (a, b) scaled to
// 1 / (margin C), so points with s >= 1 get code pos,
// s <= -1 code neg and the band of half-width `margin` (sub-block units, chosen per record)
// between is mixed.  The host certifies the two half-planes widened by kLineSlack sub-block units,
// far more than the float evaluation's error.
struct LineRec {
    float a, b, c;
    uint16_t pos, neg;
};
static_assert(sizeof(LineRec) == 16, "LineRec is one 16-byte record");
static const double kLineSlack = 5e-5;
MOSAIC_HD uint16_t line_code(const LineRec& l, float u, float v) {
    const float sv = fmaf(l.a, u, fmaf(l.b, v, l.c));
    return sv >= 1.0f ? l.pos : (sv <= -1.0f ? l.neg : kMixed);
}

struct PointRaster {
    const uint16_t* sub;        // (nx) x (ny) sub-block entries (S x S per tile), then the compact
                                // copies of the non-uniform quads; nullptr: no raster
    const uint32_t* tile_base;  // per tile (tnx per row): first leaf-block element of the tile
    const uint16_t* blocks;     // per tile: line records (8 elements each), C x C leaf blocks
    double sx, sy;              // sub-blocks per degree
    int32_t nx, ny, C, sshift, tnx;  // S = 1 << sshift sub-blocks per tile side
    int32_t cshift;             // C = 1 << cshift leaf cells per sub-block side
    // quad level: one uint16 per 2^qshift x 2^qshift sub-blocks: the code they all share (< 0x8000)
    // or kSubBlock | r (= look at the sub-block's copy in compact quad r,
    // sub[nx * ny + (r << 2 qshift) + local]); small enough (<= kQuadMax entries) to live in LDS
    const uint16_t* quad;       // nullptr: no quad level
    int32_t qnx, qny, qshift;
    // quad records (LDS-resident beside the quad level): for compact quad r < n_qrec, 8 x 8
    // sub-quads of 2^qrec_shift sub-blocks a side (qrec_shift = qshift - 3); bit
    // (sy & 7) 8 + (sx & 7) of qrec_mask[2 r], [2 r + 1] (sx, sy = sub-block >> qrec_shift) set
    // when every sub-block of that sub-quad holds the code qrec_code[r] -- the quad's most common
    // uniform sub-quad code -- so such points need no sub-block lookup
    const uint32_t* qrec_mask;
    const uint16_t* qrec_code;
    int32_t n_qrec, qrec_shift;
    // leaf lines (leaf code kSubBlock | kLineBit | n): LineRec llines[tile_lbase[tile] + n], apart from
    // `blocks` so that the stream kernels' line records and leaf blocks keep their layout; nullptr: none
    const uint32_t* tile_lbase;
    const LineRec* llines;
};
static const int kQuadMax = 32768;    // default quad-level entry budget
static const int kQuadRefMax = 0x7ffe;  // quad entries kSubBlock | r, r <= kQuadRefMax: compact sub-blocks
static const int kQuadLimit = 65536;  // option raster_quad: largest entry budget

MOSAIC_HD bool sub_is_block(uint32_t e) { return (e & kSubBlock) && e != kMixed; }
// Leaf codes are 0, key + 1, kMixed or -- a leaf line -- kSubBlock | kLineBit | n: the cell is split
// by one straight chip edge, the tile's leaf line n (PointRaster::llines, sub-block frame, as the
// line sub-blocks' records).
// Every consumer that does not evaluate leaf lines treats codes >= kSubBlock as kMixed.
MOSAIC_HD bool leaf_is_line(uint32_t c) { return (c & 0xC000u) == 0xC000u && c != kMixed; }
static const int kLeafLineMargins = 3;  // leaf lines try line_margin(0 .. 2): at most 1/128 sub-block

// The point raster's code of (x, y), grid origin (x0, y0) shared with the tile grid; the kernel
// k_join_stream computes exactly this, lane-parallel.  Fine-cell coordinates g = (x - x0) sx C
// (C a power of two, so g is the sub-block coordinate scaled exactly) are clamped to the grid:
// a finite point outside lands on an edge sub-block, whose entry the builder has checked to be 0
// (no pair; every chip cell lies well inside the grid) or kMixed.  Non-finite points: kMixed.
// With use_quad the sub-block entry is read through the quad level and its compact copies, as the
// kernel does; the answer is the same.
MOSAIC_HD uint16_t raster_code(const PointRaster& r, double x0, double y0, double x, double y, bool use_quad = false) {
    if (!isfinite(x + y)) return kMixed;
    const int C = 1 << r.cshift, cm = C - 1;
    double gx = (x - x0) * (r.sx * (double)C), gy = (y - y0) * (r.sy * (double)C);
    gx = fmin(fmax(gx, 0.0), (double)r.nx * C - 1.0);
    gy = fmin(fmax(gy, 0.0), (double)r.ny * C - 1.0);
    const int ixC = (int)gx, iyC = (int)gy, ix = ixC >> r.cshift, iy = iyC >> r.cshift;
    uint32_t e;
    if (use_quad && r.quad) {
        uint32_t q = r.quad[(uint32_t)(iy >> r.qshift) * (uint32_t)r.qnx + (uint32_t)(ix >> r.qshift)];
        if (q >= kSubBlock && (q & 0x7fffu) < (uint32_t)r.n_qrec) {
            const uint32_t rr = q & 0x7fffu;
            const uint32_t b = (uint32_t)((((iy >> r.qrec_shift) & 7) << 3) | ((ix >> r.qrec_shift) & 7));
            if ((r.qrec_mask[2 * rr + (b >> 5)] >> (b & 31)) & 1u) q = r.qrec_code[rr];
        }
        const int qm = (1 << r.qshift) - 1;
        e = q < kSubBlock ? q
                          : r.sub[(size_t)r.nx * r.ny + ((size_t)(q & 0x7fffu) << (2 * r.qshift)) +
                                  (size_t)(((iy & qm) << r.qshift) | (ix & qm))];
    } else {
        e = r.sub[(size_t)iy * r.nx + ix];
    }
    if (!sub_is_block(e)) return (uint16_t)e;
    const size_t base = r.tile_base[(iy >> r.sshift) * r.tnx + (ix >> r.sshift)];
    const uint32_t n = e & 0x3fffu;
    if (e & kLineBit) {  // tile frame
        const int tm = (1 << (r.sshift + r.cshift)) - 1;
        return line_code(*(const LineRec*)(r.blocks + base - 8 * (size_t)(n + 1)), (float)(gx - (double)(ixC & ~tm)),
                         (float)(gy - (double)(iyC & ~tm)));
    }
    const uint16_t lc = r.blocks[base + ((size_t)n << (2 * r.cshift)) + (size_t)(((iyC & cm) << r.cshift) | (ixC & cm))];
    if (leaf_is_line(lc) && r.llines)
        return line_code(r.llines[r.tile_lbase[(iy >> r.sshift) * r.tnx + (ix >> r.sshift)] + (lc & 0x3fffu)],
                         (float)(gx - (double)(ixC & ~cm)), (float)(gy - (double)(iyC & ~cm)));
    return leaf_is_line(lc) ? kMixed : lc;
}

// Fixed-point fine-cell coordinates (k_join_stream_pipe): gi = floor(g 2^kFixBits) with g the
// fine-cell coordinate, computed as the saturating conversion of fma(x, sxC 2^F, -x0 sxC 2^F) (a
// power-of-two scaling of the kernel's fma(x, sxC, -x0 sxC): the same rounding, so floor(gi / 2^F)
// is the same leaf cell; negative and NaN -> 0) clamped to gmax 2^F.  The line test then sees the point's offset
// truncated to 2^-F leaf cells (< 2^-16 sub-blocks per axis with C = 16): far inside the
// kLineSlack sub-block units the line records are certified with.  Needs (N C) 2^F < 2^31.
static const int kFixBits = 12;
MOSAIC_HD uint32_t fix_cvt(double v) {  // v_cvt_u32_f64: saturating (negative and NaN -> 0)
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    __asm__("v_cvt_u32_f64 %0, %1" : "=v"(r) : "v"(v));
    return r;
#else
    if (!(v > 0.0)) return 0u;
    if (v >= 4294967295.0) return 4294967295u;
    return (uint32_t)v;
#endif
}
// the host statement of k_join_stream_pipe's lookup (quad level, compact copies, leaf blocks and line
// records with fixed-point offsets); ax = sxC 2^F, bx = -x0 sxC 2^F (likewise y), gmax = (N C - 1) 2^F
MOSAIC_HD uint16_t raster_code_fixed(const PointRaster& r, double ax, double bx, double ay, double by, uint32_t gxmax,
                                     uint32_t gymax, double x, double y) {
    const int F = kFixBits;
    uint32_t gix = fix_cvt(fma(x, ax, bx)), giy = fix_cvt(fma(y, ay, by));
    gix = gix > gxmax ? gxmax : gix;
    giy = giy > gymax ? gymax : giy;
    const int cm = (1 << r.cshift) - 1;
    const int ixC = gix >> F, iyC = giy >> F, ix = ixC >> r.cshift, iy = iyC >> r.cshift;
    uint32_t q = r.quad[(uint32_t)(iy >> r.qshift) * (uint32_t)r.qnx + (uint32_t)(ix >> r.qshift)];
    if (q >= kSubBlock && (q & 0x7fffu) < (uint32_t)r.n_qrec) {
        const uint32_t rr = q & 0x7fffu;
        const uint32_t b = (uint32_t)((((iy >> r.qrec_shift) & 7) << 3) | ((ix >> r.qrec_shift) & 7));
        if ((r.qrec_mask[2 * rr + (b >> 5)] >> (b & 31)) & 1u) q = r.qrec_code[rr];
    }
    const int qm = (1 << r.qshift) - 1;
    const uint32_t e = q < kSubBlock ? q
                                     : r.sub[(size_t)r.nx * r.ny + ((size_t)(q & 0x7fffu) << (2 * r.qshift)) +
                                             (size_t)(((iy & qm) << r.qshift) | (ix & qm))];
    if (!sub_is_block(e)) return (uint16_t)e;
    const size_t base = r.tile_base[(iy >> r.sshift) * r.tnx + (ix >> r.sshift)];
    const uint32_t n = e & 0x3fffu;
    if (e & kLineBit) {  // tile frame
        const uint32_t fm = (1u << (r.sshift + r.cshift + F)) - 1u;
        const float sc = 1.0f / (float)(1 << F);
        return line_code(*(const LineRec*)(r.blocks + base - 8 * (size_t)(n + 1)), (float)((uint32_t)gix & fm) * sc,
                         (float)((uint32_t)giy & fm) * sc);
    }
    const uint16_t lc = r.blocks[base + ((size_t)n << (2 * r.cshift)) + (size_t)(((iyC & cm) << r.cshift) | (ixC & cm))];
    if (leaf_is_line(lc) && r.llines) {
        const uint32_t fm = (1u << (r.cshift + F)) - 1u;
        const float sc = 1.0f / (float)(1 << F);
        return line_code(r.llines[r.tile_lbase[(iy >> r.sshift) * r.tnx + (ix >> r.sshift)] + (lc & 0x3fffu)],
                         (float)((uint32_t)gix & fm) * sc, (float)((uint32_t)giy & fm) * sc);
    }
    return leaf_is_line(lc) ? kMixed : lc;
}

// std::vector allocator whose resize() leaves trivial elements uninitialised (host builders only)
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept {
        ::new ((void*)p) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new ((void*)p) U(std::forward<A>(a)...);
    }
};

struct TileRec {
    int32_t a0, b0;  // window origin (axial)
    uint32_t off;    // first window entry
    uint32_t dims;   // face | wa << 8 | wb << 20
};
static_assert(sizeof(TileRec) == 16, "TileRec is one 16-byte record");

struct Grid {
    double x0, y0;  // lon, lat of the grid origin
    double sx, sy;  // tiles per degree
    int32_t nx, ny;
};

// Bounds of F (above) over one tile, for paths of unit speed in (lon, lat) degrees.  With D = FC.p
// >= D_min and s = |p - D FC| = sin(angle to FC) <= s_max over the tile, S = kH3FastScale[res] and
// k = pi / 180 (F = S M p / D, M = (EI; EP) of norm 1, |M p| = s, D' = FC.p' with |D'| <= s |p'| as
// p' is tangent, and |p'| <= 1; |p''| <= 1 along lon / lat lines, <= 2 along any straight line):
//   |F'|  <= jac  = S k (1 / D + s^2 / D^2)
//   |F''| <= kax  = S k^2 (1 / D + 3 s / D^2 + 2 s^3 / D^3)   (lon / lat lines)
//   |F''| <= kdir = S k^2 (2 / D + 4 s / D^2 + 2 s^3 / D^3)   (any straight line)
// from F'' = S (M p'' / D - 2 M p' D' / D^2 - M p D'' / D^2 + 2 M p D'^2 / D^3).
struct TileCurv {
    double kax, kdir, jac;
};
// A rectangle w x h (degrees) widened by e per side: every point's image lies within this distance
// (hex units) of the quadrilateral of its corner images -- the bilinear interpolant maps the
// rectangle onto that quadrilateral and differs from F by <= (w^2 + h^2) kax / 8 (its error along
// each axis is <= length^2 / 8 times the second derivative; bilinear interpolation is the two in
// turn, each non-expanding), the widening moves an image by <= sqrt(2) e jac, and 1e-7 covers the
// corner images' rounding.
MOSAIC_HD double rect_tol(const TileCurv& c, double w, double h, double e) {
    return 0.125 * c.kax * (w * w + h * h) + 1.5 * c.jac * e + 1e-7;
}
// A convex polygon with bounding box w x h (degrees), widened by e: within this distance of the
// polygon of its vertex images -- F differs from its first-order Taylor polynomial A at the box
// centre by <= kdir r^2 / 2 (r^2 <= (w^2 + h^2) / 4), and A(polygon) = hull(A(vertices)) is within
// that of hull(F(vertices)), hence twice that.
MOSAIC_HD double poly_tol(const TileCurv& c, double w, double h, double e) {
    return 0.25 * c.kdir * (w * w + h * h) + 1.5 * c.jac * e + 1e-7;
}

// Tile code of (x = lon, y = lat): kSkip outside the grid (finite points), kFull for non-finite.
MOSAIC_HD uint32_t tile_of(const Grid& g, const uint32_t* idx, double x, double y) {
    double fx = (x - g.x0) * g.sx, fy = (y - g.y0) * g.sy;
    if (!(fx >= 0.0 && fx < (double)g.nx && fy >= 0.0 && fy < (double)g.ny))
        return (isfinite(x) && isfinite(y)) ? kSkip : kFull;
    return idx[(int64_t)(int)fy * g.nx + (int)fx];
}

// ---- host-side construction -------------------------------------------------------------------
// The builder reads the H3 tables as host constants, so its code is compiled by the host compiler
// only (tiles_build.cpp, g++): hipcc's host pass sees __constant__ tables as uninitialised
// shadows.  mosaic_hip.hip calls Builder::build across that boundary.
#if !defined(__HIPCC__)
// Approximate lon/lat centre of an H3 cell (on its base cell's home face) and its hex-unit scale;
// used only to place the grid, whose coverage is then verified by the forward path.
inline bool cell_center(uint64_t h, int res, double* lon, double* lat) {
    if (((h >> 59) & 15) != 1 || (int)((h >> 52) & 15) != res) return false;
    int bc = (int)((h >> 45) & 127);
    if (bc >= 122) return false;
    const int* bd = h3::kH3BaseCellData[bc];
    if (bd[4] && h3::leading_nonzero_digit(h, res) == 5) h = h3::rotate_all(h, res, false);
    int face = bd[0];
    int a = bd[1] - bd[3], b = bd[2] - bd[3];
    for (int r = 1; r <= res; r++) {
        int na, nb;
        if (r & 1) {
            na = 2 * a + b;
            nb = 3 * b - a;
        } else {
            na = 3 * a - b;
            nb = a + 2 * b;
        }
        int d = h3::get_digit(h, r);
        if (d == 7) return false;
        a = na + (((d >> 2) & 1) - (d & 1));
        b = nb + (((d >> 1) & 1) - (d & 1));
    }
    const double s60 = 0.86602540378443864676;
    double vx = (double)a - 0.5 * (double)b, vy = (double)b * s60;
    const double* fb = h3::kH3FastBasis[face];
    const double* ei = fb + ((res & 1) ? 9 : 3);
    const double* ep = fb + ((res & 1) ? 12 : 6);
    double t = vx / h3::kH3FastScale[res], u = vy / h3::kH3FastScale[res];
    double px = fb[0] + t * ei[0] + u * ep[0], py = fb[1] + t * ei[1] + u * ep[1], pz = fb[2] + t * ei[2] + u * ep[2];
    double nrm = sqrt(px * px + py * py + pz * pz);
    *lat = asin(pz / nrm) * 57.29577951308232;
    *lon = atan2(py, px) * 57.29577951308232;
    return isfinite(*lat) && isfinite(*lon);
}

#endif  // !__HIPCC__

struct Builder {
    Grid grid{};
    std::vector<uint32_t> tile_idx;
    std::vector<TileRec> recs;
    std::vector<uint32_t> entries;
    int rings = 0;
    int64_t n_full = 0, n_skip = 0;
    const char* why = nullptr;  // reason the directory was not built
    int res_ = 0;
    std::vector<TileCurv> rec_curv;  // per record: the bounds of F over the tile

    // ---- point raster (second stage, optional): per sub-block of a tile (S x S per tile, S a power
    // of two) a uint16 entry: a code, kMixed, kSubBlock | tile-local leaf block, or kSubBlock |
    // kLineBit | tile-local line record; leaf blocks are C x C uint16 codes, a tile's first at
    // element tile_base[tile], its line records (LineRec, 8 elements) just below it, last first.
    // Codes: 0 = the point joins nothing, k + 1 = exactly one pair with polygon key k, kMixed =
    // run the tile path.
    int S = 0, C = 0, sshift = 0, cshift = 0;
    bool edge_ok = false;  // every edge sub-block is 0 or kMixed (raster_code clamps onto them)
    // (sub and blocks are resized without value-initialisation: assemble_raster writes every
    // element, in parallel, so the pages are first touched by the threads that fill them)
    std::vector<uint16_t, NoInitAlloc<uint16_t>> sub;
    std::vector<uint32_t> tile_base;
    std::vector<uint32_t> tile_lbase;  // leaf lines: per tile the first of its records in llines
    std::vector<LineRec> llines;
    std::vector<uint16_t, NoInitAlloc<uint16_t>> blocks;
    std::vector<uint16_t> quad;  // quad level (empty: none)
    int qshift = 0, qnx = 0, qny = 0;
    int quad_max = kQuadMax;  // quad-level entry budget (set before build_raster)
    // quad records (PointRaster::qrec_*): LDS bytes for the quad level and the records together
    // (0: no records); set before build_raster
    size_t quad_lds_bytes = 0;
    std::vector<uint32_t> qrec_mask;
    std::vector<uint16_t> qrec_code;
    int qrec_shift = 0;
    int64_t n_sub_pure = 0, n_sub_mixed = 0, n_cell_mixed = 0, n_sub_line = 0, n_cell_line = 0;
    bool lines = true;  // split single-feature sub-blocks by a line (set before build_raster)
    bool leaf_lines = false;  // and single-feature leaf cells of the other mixed sub-blocks
    // Chip access for the raster classification (host memory)
    struct ChipSource {
        const uint32_t* slot_first;  // per hash slot: first chip, chip count (0 for empty slots)
        const uint32_t* slot_count;
        const uint32_t* meta;        // (polygon_key << 1) | is_core
        pip::GeomStore store;        // chip geometry (border chips), host pointers
        int32_t n_polygons;
    };
    bool build_raster(const ChipSource& src, int S_, int C_, int threads);
    // build_raster in two phases, so the classification can run on the GPU (k_raster_* in
    // mosaic_hip.hip) and the assembly on the host:
    //   phase 1: every sub-block's code (kMixed for mixed ones); per mixed sub-block (in record,
    //            then scan order) a line record (kind 1) or its C x C cell codes (kind 0);
    //   phase 2: sub-block entries, per-tile line records and leaf blocks, quad level.
    struct RasterClass {
        // (code and cells are filled by device-to-host copies: not value-initialised)
        std::vector<uint16_t, NoInitAlloc<uint16_t>> code;  // records x S x S (scan order sj S + si)
        std::vector<uint8_t> kind;      // per mixed sub-block
        std::vector<LineRec> line;      // per mixed sub-block (kind 1)
        std::vector<uint32_t> cell_at;  // per mixed sub-block (kind 0): its block of C x C codes in cells
        std::vector<uint16_t, NoInitAlloc<uint16_t>> cells;
        // leaf lines: the kMixed leaf cells (index into cells, ascending) that one straight chip edge
        // splits, and their line records (sub-block frame, as the sub-block line records)
        std::vector<uint32_t> cline_at;
        std::vector<LineRec> cline;
    };
    std::vector<int> tile_of_rec;  // record -> tile (raster_setup)
    bool raster_setup(const ChipSource& src, int S_, int C_);
    void classify_raster_host(const ChipSource& src, int threads, RasterClass& rc);
    bool assemble_raster(const RasterClass& rc, int threads = 1);
    static rbuild::HexTable hex_table_values();

    // cells: distinct chip cells; slot_of(cell) -> chip hash slot or -1.  Defined for the host
    // compiler only (tiles_build.cpp); false (with `why`) when the directory is not built.
    bool build(int res, const std::vector<int64_t>& cells, const std::function<int64_t(int64_t)>& slot_of);

#if !defined(__HIPCC__)
    // Sample geometry of one tile: face (or -1) and axial coordinates of the 3 x 3 samples.
    struct Samples {
        int face;
        double a[9], b[9];
    };
    static bool sample(double lon0, double lat0, double tw, double th, int res, Samples* s) {
        s->face = -1;
        for (int k = 0; k < 9; k++) {
            double lon = lon0 + 0.5 * (k % 3) * tw, lat = lat0 + 0.5 * (k / 3) * th;
            double px, py, pz, best, gap;
            h3::fast_unit(lat, lon, &px, &py, &pz);
            int f = h3::face_search(px, py, pz, &best, &gap);
            if (gap < 1e-4 || (s->face >= 0 && f != s->face)) return false;
            s->face = f;
            double vx, vy, b;
            h3::fast_plane(px, py, pz, f, res, &vx, &vy, &b);
            const double inv_s60 = 1.1547005383792515;
            s->b[k] = vy * inv_s60;
            s->a[k] = vx + 0.5 * s->b[k];
        }
        return true;
    }

    bool build_impl(int res, const std::vector<int64_t>& cells, const std::function<int64_t(int64_t)>& slot_of) {
        why = nullptr;
        if (cells.empty()) return fail("no chip cells");
        if (res < 0 || res > 15) return fail("resolution");
        // region of the chip cells: centres widened by ~3 hex units (measured at the centre)
        double x0 = INFINITY, y0 = INFINITY, x1 = -INFINITY, y1 = -INFINITY;
        std::vector<double> cx(cells.size()), cy(cells.size());
        for (size_t k = 0; k < cells.size(); k++) {
            if (!cell_center((uint64_t)cells[k], res, &cx[k], &cy[k])) return fail("cell outside the supported set");
            x0 = std::min(x0, cx[k]);
            x1 = std::max(x1, cx[k]);
            y0 = std::min(y0, cy[k]);
            y1 = std::max(y1, cy[k]);
        }
        // hex units per degree at the region centre (lon and lat directions): placement only
        double mx = 0.5 * (x0 + x1), my = 0.5 * (y0 + y1);
        Samples c0;
        double dd = 1e-4;
        if (!sample(mx - dd, my - dd, 2 * dd, 2 * dd, res, &c0)) return fail("region centre near a face edge");
        double slon = axis_scale(c0, 3, 5, 2 * dd), slat = axis_scale(c0, 1, 7, 2 * dd);
        if (!(slon > 0 && slat > 0)) return fail("degenerate scale");
        // pad by 3 hex units (cells are ~0.6 hex units around their centres)
        x0 -= 6.0 / slon;
        x1 += 6.0 / slon;
        y0 -= 6.0 / slat;
        y1 += 6.0 / slat;
        if (y0 < -80.0 || y1 > 80.0) return fail("polar region");
        if (x1 - x0 > 90.0 || y1 - y0 > 60.0) return fail("region too large");
        double tw = std::min(0.25, 4.0 / slon), th = std::min(0.25, 4.0 / slat);
        // tile budget: at most 2^24 tiles and 2^26 window entries
        double ntiles = ((x1 - x0) / tw + 4) * ((y1 - y0) / th + 4);
        if (ntiles > (double)(1 << 24)) return fail("too many tiles");
        // rings: 1.5x the cell reach (2.5 hex units) under the lower bound S k cos(lat_max) on F's
        // expansion per degree, lat_max over the grid (<= 64 rings past the padded region)
        const double kdeg = 3.141592653589793 / 180.0;
        const double lat_max = std::min(89.0, std::max(fabs(y0), fabs(y1)) + 64.0 * th);
        const double sig_lo = h3::kH3FastScale[res] * kdeg * cos(lat_max * kdeg) * (1.0 - 1e-9);
        int k = std::max(2, (int)ceil(3.75 / (std::min(tw, th) * sig_lo)));
        if (k > 64) return fail("ring count");
        rings = k;
        int nx = (int)ceil((x1 - x0) / tw) + 2 * k, ny = (int)ceil((y1 - y0) / th) + 2 * k;
        grid.x0 = x0 - k * tw;
        grid.y0 = y0 - k * th;
        grid.sx = 1.0 / tw;
        grid.sy = 1.0 / th;
        grid.nx = nx;
        grid.ny = ny;
        tile_idx.assign((size_t)nx * ny, kSkip);
        recs.clear();
        entries.clear();
        rec_curv.clear();
        res_ = res;
        std::vector<uint8_t> found(cells.size(), 0);
        // slot -> position in cells (for the found flags)
        std::vector<int64_t> slot_cell;
        {
            int64_t mx = -1;
            for (size_t q = 0; q < cells.size(); q++) mx = std::max(mx, slot_of(cells[q]));
            slot_cell.assign((size_t)std::max<int64_t>(mx + 1, 0), -1);
            for (size_t q = 0; q < cells.size(); q++) {
                const int64_t sl = slot_of(cells[q]);
                if (sl >= 0) slot_cell[(size_t)sl] = (int64_t)q;
            }
        }
        n_full = n_skip = 0;
        // tile rows on host threads (each tile is independent; found flags are only ever set to 1),
        // then merged in row order: records and window entries exactly as a sequential scan
        struct RowOut {
            std::vector<uint32_t> code;  // per tile: kFull, kSkip, or 2 + the row-local record
            std::vector<TileRec> recs;
            std::vector<TileCurv> curv;
            std::vector<uint32_t> entries;
        };
        std::vector<RowOut> rows((size_t)ny);
        auto do_row = [&](int j) {
            RowOut& ro = rows[(size_t)j];
            ro.code.assign((size_t)nx, kFull);
            std::vector<uint32_t> win;
            for (int i = 0; i < nx; i++) {
                // tile bounds exactly as the kernel's index computes them (to rounding)
                double lon0 = grid.x0 + i * tw, lat0 = grid.y0 + j * th;
                Samples s;
                uint32_t code = kFull;
                TileCurv cv;
                if (sample(lon0, lat0, tw, th, res, &s) && tile_curv(s.face, lon0, lat0, tw, th, res, &cv) &&
                    rect_tol(cv, tw, th, 0.0) <= 0.25) {
                    double amin = INFINITY, amax = -INFINITY, bmin = INFINITY, bmax = -INFINITY;
                    for (int q = 0; q < 9; q++) {
                        amin = std::min(amin, s.a[q]);
                        amax = std::max(amax, s.a[q]);
                        bmin = std::min(bmin, s.b[q]);
                        bmax = std::max(bmax, s.b[q]);
                    }
                    int a0 = (int)floor(amin) - 1, a1 = (int)floor(amax) + 1;
                    int b0 = (int)floor(bmin) - 1, b1 = (int)floor(bmax) + 1;
                    int wa = a1 - a0 + 1, wb = b1 - b0 + 1;
                    if (wa <= 255 && wb <= 4095 && wa * wb <= 4096) {
                        win.assign((size_t)wa * wb, 0);
                        bool any = false;
                        bool inner = i >= k && j >= k && i < nx - k && j < ny - k;
                        for (int ra = 0; ra < wa; ra++) {
                            for (int rb = 0; rb < wb; rb++) {
                                int64_t h = (int64_t)h3::face_axial_to_h3(s.face, a0 + ra, b0 + rb, res);
                                int64_t slot = slot_of(h);
                                if (slot < 0) continue;
                                win[(size_t)ra * wb + rb] = (uint32_t)slot + 1;
                                any = true;
                                if (inner && slot < (int64_t)slot_cell.size() && slot_cell[(size_t)slot] >= 0) {
                                    uint8_t& fd = found[(size_t)slot_cell[(size_t)slot]];
                                    if (!fd && deep_inside(s.face, a0 + ra, b0 + rb, res)) fd = 1;
                                }
                            }
                        }
                        if (!any) {
                            code = kSkip;
                        } else {
                            TileRec r;
                            r.a0 = a0;
                            r.b0 = b0;
                            r.off = (uint32_t)ro.entries.size();  // row-local until the merge
                            r.dims = (uint32_t)s.face | ((uint32_t)wa << 8) | ((uint32_t)wb << 20);
                            ro.entries.insert(ro.entries.end(), win.begin(), win.end());
                            code = (uint32_t)ro.recs.size() + 2;
                            ro.recs.push_back(r);
                            ro.curv.push_back(cv);
                        }
                    }
                }
                ro.code[(size_t)i] = code;
            }
        };
        {
            const int nt = (int)std::max(1, std::min({16, (int)std::max(1u, std::thread::hardware_concurrency()), ny}));
            std::atomic<int> next(0);
            auto work = [&]() {
                for (int j; (j = next.fetch_add(1)) < ny;) do_row(j);
            };
            std::vector<std::thread> pool;
            for (int t = 1; t < nt; t++) pool.emplace_back(work);
            work();
            for (auto& th : pool) th.join();
        }
        for (int j = 0; j < ny; j++) {
            RowOut& ro = rows[(size_t)j];
            const uint32_t rec0 = (uint32_t)recs.size();
            const size_t ent0 = entries.size();
            if (ent0 + ro.entries.size() >= ((size_t)1 << 26)) return fail("window entries");
            for (TileRec r : ro.recs) {
                r.off += (uint32_t)ent0;
                recs.push_back(r);
            }
            rec_curv.insert(rec_curv.end(), ro.curv.begin(), ro.curv.end());
            entries.insert(entries.end(), ro.entries.begin(), ro.entries.end());
            for (int i = 0; i < nx; i++) {
                uint32_t code = ro.code[(size_t)i];
                if (code == kFull) n_full++;
                else if (code == kSkip) n_skip++;
                else code += rec0;
                tile_idx[(size_t)j * nx + i] = code;
            }
            std::vector<uint32_t>().swap(ro.entries);
        }
        // coverage: every chip cell found in an inner tile, deep inside its face, and k rings span
        // 1.5x the cell reach under the expansion bound over the whole grid
        for (size_t q = 0; q < cells.size(); q++)
            if (!found[q]) return fail("a chip cell was not found inside the grid, away from face edges");
        const double glat = std::max(fabs(grid.y0), fabs(grid.y0 + ny * th));
        if (!(glat <= lat_max && k * std::min(tw, th) * sig_lo >= 3.75)) return fail("ring margin below the cell reach");
        if (recs.empty()) recs.push_back(TileRec{0, 0, 0, 0});
        if (entries.empty()) entries.push_back(0);
        return true;
    }

  private:
    // Euclidean hex units per degree along one sample pair (k0 -> k1 spans `span` degrees)
    static double axis_scale(const Samples& s, int k0, int k1, double span) {
        const double s60 = 0.86602540378443864676;
        double da = s.a[k1] - s.a[k0], db = s.b[k1] - s.b[k0];
        return hypot(da - 0.5 * db, s60 * db) / span;
    }
    bool fail(const char* w) {
        why = w;
        tile_idx.clear();
        recs.clear();
        entries.clear();
        return false;
    }
#endif  // !__HIPCC__

  public:
#if !defined(__HIPCC__)
    // TileCurv of tile [lon0, lon0 + tw] x [lat0, lat0 + th] on `face`: D and s at the centre, moved
    // by at most the tile's angular radius rho <= (tw + th) / 2 degrees (a meridian then a parallel
    // path; D and s are 1-Lipschitz in angle); false when D_min <= 0.5 (never on a face's own tile)
    static bool tile_curv(int face, double lon0, double lat0, double tw, double th, int res, TileCurv* c) {
        const double k = 3.141592653589793 / 180.0;
        double px, py, pz;
        h3::fast_unit(lat0 + 0.5 * th, lon0 + 0.5 * tw, &px, &py, &pz);
        const double* fc = h3::kH3FastBasis[face];
        const double dc = fc[0] * px + fc[1] * py + fc[2] * pz;
        const double rho = 0.5 * (tw + th) * k * (1.0 + 1e-9) + 1e-12;
        const double D = dc - rho, s = std::min(1.0, sqrt(std::max(0.0, 1.0 - dc * dc)) + rho);
        if (!(D > 0.5)) return false;
        const double S = h3::kH3FastScale[res] * (1.0 + 1e-12), up = 1.0 + 1e-9;
        const double D2 = D * D, D3 = D2 * D, s3 = s * s * s;
        c->kax = S * k * k * (1.0 / D + 3.0 * s / D2 + 2.0 * s3 / D3) * up;
        c->kdir = S * k * k * (2.0 / D + 4.0 * s / D2 + 2.0 * s3 / D3) * up;
        c->jac = S * k * (1.0 / D + s * s / D2) * up;
        return true;
    }
    // the hexagon at axial (a, b) on `face` (resolution res) lies at least 2 / sqrt(3) hex units
    // inside the face's territory: its centre's distance (face plane, hex units) from the line
    // (FC_f - FC_g).(FC_f + (x EI + y EP) / S) = 0 of every other face g
    static bool deep_inside(int face, int a, int b, int res) {
        const double* fb = h3::kH3FastBasis[face];
        const double* ei = fb + ((res & 1) ? 9 : 3);
        const double* ep = fb + ((res & 1) ? 12 : 6);
        const double S = h3::kH3FastScale[res];
        const double x = (double)a - 0.5 * (double)b, y = (double)b * 0.86602540378443864676;
        for (int g = 0; g < 20; g++) {
            if (g == face) continue;
            const double* gc = h3::kH3FastBasis[g];
            const double n[3] = {fb[0] - gc[0], fb[1] - gc[1], fb[2] - gc[2]};
            const double c0 = n[0] * fb[0] + n[1] * fb[1] + n[2] * fb[2];
            const double gx = (n[0] * ei[0] + n[1] * ei[1] + n[2] * ei[2]) / S;
            const double gy = (n[0] * ep[0] + n[1] * ep[1] + n[2] * ep[2]) / S;
            const double gn = sqrt(gx * gx + gy * gy);
            if (gn == 0.0) continue;  // (the opposite face: its bisector plane misses the face's plane)
            if (!((c0 + gx * x + gy * y) / gn >= 1.1547005383792515 + 1e-6)) return false;
        }
        return true;
    }
#endif  // !__HIPCC__
};


// BNG leaf blocks (tiles_build.cpp): for each border cell (lower-left corner x0, y0 in metres,
// side `side`, chips at hash slot `slot`), C x C uint16 codes over the cell, same codes and same
// rule as the H3 point raster (the cell is the only candidate: BNG cells are squares in the
// points' own coordinates).  Host compiler only.
struct BngBorderCell {
    double x0, y0;
    uint32_t slot;
};
// BNG border cells (k_join_stream_bng): per cell a C x C block of sub-cell entries -- a code,
// kMixed, or kSubBlock | kLineBit | n for a sub-cell split by one straight chip edge (LineRec n of
// the cell, evaluated at the point's offset in the sub-cell in sub-cell units, stored at
// blocks[base - 8 (n + 1)]); base[k] = element offset of cell k's block (a multiple of 8).
// The cells' sub-block levels (BngStreamArgs::lvl): per border cell, per 4 x 4 group of sub-cells
// (bng_level_side(C) groups per row, row-major, bng_level_stride(C) entries per cell) the group's
// code when all its sub-cells carry the same code that is not a line code, else kSubBlock ("read the
// sub-cell's own code").  k_join_stream_bng_cpt gathers the level beside the cell entry and the leaf
// code only for kSubBlock groups, so the rows of uniform groups touch one 128-byte line per border
// cell (L2-resident) instead of a line of the cell's 2 KB leaf block.
#ifndef MOSAIC_BNG_LVL_SHIFT
#define MOSAIC_BNG_LVL_SHIFT 2  // groups of 4 x 4 sub-cells
#endif
static const int kBngLvlShift = MOSAIC_BNG_LVL_SHIFT, kBngLvlG = 1 << MOSAIC_BNG_LVL_SHIFT;
inline int bng_level_side(int C) { return (C + kBngLvlG - 1) / kBngLvlG; }
inline int bng_level_stride(int C) { return ((bng_level_side(C) * bng_level_side(C) + 63) / 64) * 64; }
inline uint16_t bng_level_code(const uint16_t* e, int C, int bi, int bj) {
    const int G = kBngLvlG;
    const uint16_t v = e[(size_t)(G * bj) * C + G * bi];
    if (v != kMixed && (v & 0xC000u) == 0xC000u) return kSubBlock;  // a line code: per sub-cell
    for (int j = G * bj; j < std::min(C, G * bj + G); j++)
        for (int i = G * bi; i < std::min(C, G * bi + G); i++)
            if (e[(size_t)j * C + i] != v) return kSubBlock;
    return v;
}
// glines (optional): per border cell bng_level_side(C)^2 group codes -- a line code kSubBlock |
// kLineBit | n where the cell's line record n (cell frame) is certified over the whole group (every
// line sub-cell of the group names n, none is kMixed, and both half-planes of the record clipped to
// the widened group square classify to its pos / neg), else kSubBlock.  The level then carries that
// line code, so k_join_stream_bng_cpt gathers the record without the leaf code (a level code is a
// valid answer for every point of its group, as before).
// wedges: a sub-cell split by two chip segments that share a vertex gets the leaf code
// kSubBlock | n (no line bit): records n and n + 1 (cell frame) are the two segments' lines, oriented
// so that the convex wedge is s >= 1 on both; its code is record n's pos, the reflex side's (s <= -1
// on either line) its neg; both regions certified like a line record's sides.  The stream kernels
// send such rows to the mixed queue and k_join_mixed_bng answers them from the two records when the
// point lies outside both bands (bng_wedge_code), before any chip test.
bool bng_leaf_blocks(const Builder::ChipSource& src, const std::vector<BngBorderCell>& cells, double side, int C,
                     bool lines, int threads, std::vector<uint16_t>& blocks, std::vector<uint32_t>& base,
                     std::vector<uint16_t>* glines = nullptr, bool wedges = false);
MOSAIC_HD uint32_t bng_wedge_code(const LineRec& r1, const LineRec& r2, float u, float v) {
    const float s1 = fmaf(r1.a, u, fmaf(r1.b, v, r1.c)), s2 = fmaf(r2.a, u, fmaf(r2.b, v, r2.c));
    if (s1 >= 1.0f && s2 >= 1.0f) return r1.pos;
    if (s1 <= -1.0f || s2 <= -1.0f) return r1.neg;
    return kMixed;
}

}  // namespace tiles
}  // namespace mosaic
