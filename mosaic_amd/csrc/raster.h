// Ray-parity raster of a border chip: answers JTS contains(chip, point) for most points with one
// table lookup, and for the rest with the few segment records that can still change the answer.
//
// Why it is exact.  For a one-ring chip JTS contains(p) = "p on no segment" && "the rightward ray
// from p crosses an odd number of segments" (RayCrossingCounter over (ring[i], ring[i-1]) with the
// half-open straddle rule (p1.y > p.y) != (p2.y > p.y) and an exact orientation; reference path
// ST_Contains.scala:34-42 -> MosaicGeometryJTS.scala:101 -> JTS PointLocation.locateInRing).
// The chip envelope is cut into rows x cols cells.  For a cell C (widened by mu to absorb the
// rounding of the kernel's cell index) every segment s of the ring falls in one class:
//   touching  s meets C widened by another mu          -> listed: evaluated per point
//   outside   s lies entirely above / below C's rows     -> never straddles p.y: contributes 0
//   left      s's part inside C's rows is left of C      -> p is right of it: contributes 0
//   right     s's part inside C's rows is right of C:
//     spans   one end below and one above C's rows      -> straddles every p.y, p left of it: 1
//     partial otherwise                                  -> listed: evaluated per point
// and a point on a segment lies in a cell the segment touches, so "on" is decided by the list.
// The cell stores parity(#right-spanning) and its list; a cell with an empty list ("pure") is
// decided by the parity alone.  Any doubt in the (double precision, host side) classification
// lists the segment, which is always safe: listed segments run the exact JTS step.
//
// HBM layout (per chip table, chips in table order):
//   ChipHdr  64 B per chip       envelope, cell scales, first cell, dims
//   CellRec  8 B per cell        (first record << 1 | parity, record count), row-major per chip
//   Edge     32 B per record     {p1, p2} segment records, one run per listed cell
#pragma once
#include <math.h>
#include <stdint.h>

#include "pip_device.h"

#include <algorithm>
#include <vector>

namespace mosaic {
namespace raster {

static const uint32_t kNoRaster = 0xffffffffu;  // ChipHdr.cell_base of chips on the general path

struct ChipHdr {
    pip::Box box;        // the chip envelope (JTS envelope pre-check)
    double sx, sy;       // cols / width, rows / height (0 for a single column / row)
    uint32_t cell_base;  // first CellRec, or kNoRaster
    uint32_t cols, rows;
    uint32_t pad;
};
static_assert(sizeof(ChipHdr) == 64, "ChipHdr is one 64-byte record");

struct CellRec {
    uint32_t word;  // first record << 1 | parity of the right-spanning segments
    uint32_t m;     // listed records
};

MOSAIC_HD uint32_t cell_index(const ChipHdr& h, double x, double y) {
    int c = (int)floor((x - h.box.minx) * h.sx);
    int r = (int)floor((y - h.box.miny) * h.sy);
    c = c < 0 ? 0 : (c >= (int)h.cols ? (int)h.cols - 1 : c);
    r = r < 0 ? 0 : (r >= (int)h.rows ? (int)h.rows - 1 : r);
    return h.cell_base + (uint32_t)r * h.cols + (uint32_t)c;
}

// contains(chip, (x, y)) for a point inside the chip envelope, evaluated from the cell's list.
MOSAIC_HD bool cell_contains(const CellRec& rec, const pip::Edge* edges, double x, double y) {
    bool on = false;
    uint32_t par = rec.word & 1u;
    const pip::Edge* e = edges + (rec.word >> 1);
    for (uint32_t k = 0; k < rec.m; k++) {
        bool o, c;
        pip::edge_rec_flags(e[k], x, y, o, c);
        on |= o;
        par ^= (uint32_t)c;
    }
    return !on && par;
}

// ---- host-side construction -------------------------------------------------------------------
// Closed-segment vs closed-rectangle test (Liang-Barsky), double precision.
MOSAIC_HD bool seg_meets_rect(double ax, double ay, double bx, double by, double x0, double y0, double x1, double y1) {
    double t0 = 0.0, t1 = 1.0;
    const double dx = bx - ax, dy = by - ay;
    auto clip = [&](double p, double q) -> bool {  // constraint p * t <= q
        if (p == 0.0) return q >= 0.0;
        double r = q / p;
        if (p < 0.0) {
            if (r > t1) return false;
            if (r > t0) t0 = r;
        } else {
            if (r < t0) return false;
            if (r < t1) t1 = r;
        }
        return true;
    };
    return clip(-dx, ax - x0) && clip(dx, x1 - ax) && clip(-dy, ay - y0) && clip(dy, y1 - ay) && t0 <= t1;
}

enum SegClass { SEG_IGNORE = 0, SEG_SPAN = 1, SEG_LIST = 2 };

// Class of segment (a, b) for the cell whose possible points are [x0, x1] x [y0, y1] (already
// widened by mu); mx / my: the extra safety margins.
inline int classify(const pip::Edge& e, double x0, double y0, double x1, double y1, double mx, double my) {
    const double X0 = x0 - mx, X1 = x1 + mx, Y0 = y0 - my, Y1 = y1 + my;
    if (seg_meets_rect(e.p1x, e.p1y, e.p2x, e.p2y, X0, Y0, X1, Y1)) return SEG_LIST;
    const double ylo = std::min(e.p1y, e.p2y), yhi = std::max(e.p1y, e.p2y);
    if (yhi < Y0 || ylo > Y1) return SEG_IGNORE;
    // x-range of the segment's part within the band [Y0, Y1]
    double xa, xb;
    if (e.p1y == e.p2y) {
        xa = std::min(e.p1x, e.p2x);
        xb = std::max(e.p1x, e.p2x);
    } else {
        double ta = (Y0 - e.p1y) / (e.p2y - e.p1y), tb = (Y1 - e.p1y) / (e.p2y - e.p1y);
        ta = std::min(1.0, std::max(0.0, ta));
        tb = std::min(1.0, std::max(0.0, tb));
        double pa = e.p1x + ta * (e.p2x - e.p1x), pb = e.p1x + tb * (e.p2x - e.p1x);
        xa = std::min(pa, pb);
        xb = std::max(pa, pb);
    }
    if (xb < X0) return SEG_IGNORE;  // left of the cell: never to the right of its points
    if (xa > X1) return (ylo < Y0 && yhi > Y1) ? SEG_SPAN : SEG_LIST;
    return SEG_LIST;  // numerically inconsistent with "does not meet": keep it exact
}

struct Builder {
    std::vector<ChipHdr> hdr;
    std::vector<CellRec> cells;
    std::vector<pip::Edge> edges;
    int64_t pure_cells = 0;

    // Ring v[0..n) (closed: v[n-1] == v[0]) of one-ring chip `h`'s geometry; dims <= 0: no raster.
    void add_ring(ChipHdr& h, const pip::Vec2* v, uint32_t n, int dims) {
        h.cell_base = kNoRaster;
        h.cols = h.rows = 0;
        h.sx = h.sy = 0.0;
        if (dims <= 0 || n < 2) return;
        const pip::Box& b = h.box;
        const double W = b.maxx - b.minx, H = b.maxy - b.miny;
        const uint32_t cols = W > 0 ? (uint32_t)dims : 1u, rows = H > 0 ? (uint32_t)dims : 1u;
        h.cols = cols;
        h.rows = rows;
        h.sx = cols > 1 ? (double)cols / W : 0.0;
        h.sy = rows > 1 ? (double)rows / H : 0.0;
        h.cell_base = (uint32_t)cells.size();
        const double mx = 1e-7 * W + 1e-12 * std::max(std::fabs(b.minx), std::fabs(b.maxx)) + 1e-300;
        const double my = 1e-7 * H + 1e-12 * std::max(std::fabs(b.miny), std::fabs(b.maxy)) + 1e-300;
        std::vector<pip::Edge> segs;
        segs.reserve(n - 1);
        for (uint32_t k = 1; k < n; k++) segs.push_back(pip::Edge{v[k].x, v[k].y, v[k - 1].x, v[k - 1].y});
        std::vector<uint32_t> band;
        for (uint32_t r = 0; r < rows; r++) {
            const double y0 = (r == 0 ? b.miny : b.miny + H * r / rows) - my;
            const double y1 = (r + 1 == rows ? b.maxy : b.miny + H * (r + 1) / rows) + my;
            band.clear();
            for (uint32_t k = 0; k < segs.size(); k++) {
                const double ylo = std::min(segs[k].p1y, segs[k].p2y), yhi = std::max(segs[k].p1y, segs[k].p2y);
                if (!(yhi < y0 - my || ylo > y1 + my)) band.push_back(k);
            }
            for (uint32_t c = 0; c < cols; c++) {
                const double x0 = (c == 0 ? b.minx : b.minx + W * c / cols) - mx;
                const double x1 = (c + 1 == cols ? b.maxx : b.minx + W * (c + 1) / cols) + mx;
                uint32_t par = 0, first = (uint32_t)edges.size();
                for (uint32_t k : band) {
                    int cl = classify(segs[k], x0, y0, x1, y1, mx, my);
                    if (cl == SEG_SPAN) par ^= 1u;
                    else if (cl == SEG_LIST) edges.push_back(segs[k]);
                }
                uint32_t m = (uint32_t)edges.size() - first;
                if (m == 0) {
                    first = 0;
                    pure_cells++;
                }
                cells.push_back(CellRec{(first << 1) | par, m});
            }
        }
    }
};

}  // namespace raster
}  // namespace mosaic
