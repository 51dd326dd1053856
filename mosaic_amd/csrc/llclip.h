// Border chips the way the reference builds them: geometry n indexToGeometry(cell), clipped in the
// plane of the coordinates (lon / lat degrees for H3, metres for BNG) -- shared by the host producer
// (tessellate.cpp, g++) and the device producer (k_tess_clip_ll, hipcc), so both write the same bytes.
//
// Reference: IndexSystem.getBorderChips (src/main/scala/com/databricks/labs/mosaic/core/index/
// IndexSystem.scala:152-168): `geometry.intersection(indexToGeometry(index))`, isCore =
// `intersect.equals(indexGeom)`, empty chips dropped; indexToGeometry = the h3ToGeoBoundary ring in
// degrees with straight chords (H3IndexSystem.scala:93-100) or the BNG square
// (BNGIndexSystem.scala indexToGeometry); MosaicGeometryJTS.intersection (core/geometry/
// MosaicGeometryJTS.scala:75-80) -> JTS 1.19 overlay.  The arithmetic that fixes the bits of a chip is
// restated from JTS 1.19 [third party, absent from the reference]:
//   * crossing points: RobustLineIntersector.computeIntersect -- orientation signs by
//     CGAlgorithmsDD (pip_device.h), endpoint rules for touching / collinear segments, and for a
//     proper crossing Intersection.intersection (homogeneous coordinates conditioned by the midpoint
//     of the two envelopes' intersection), checked against both segment envelopes with
//     nearestEndpoint as the fallback;
//   * ring orientation: Orientation.isCCW (highest point, cap orientation).
// Original vertices of the geometry and of the cell are copied, never recomputed.
//
// Algorithm (Weiler-Atherton against a simple counter-clockwise cell polygon C): every ring is walked
// with the interior on its left (shells counter-clockwise, holes clockwise); each edge is split at the
// points where it meets C's boundary and each piece labelled inside / not inside C (a piece on C's
// boundary counts as not inside: the boundary walk below supplies it); maximal inside runs are chains
// from an entry point to an exit point on C's boundary; from each exit the result follows C's
// boundary counter-clockwise to the next entry (positions on the boundary are (side, parameter)
// pairs compared exactly).  Rings wholly inside C are kept; C itself is a result shell when no ring
// crosses it and it lies in the polygon.  Each result ring is written counter-clockwise (holes
// clockwise) from its lowest vertex (least y, then least x), polygons ordered by that vertex: the
// order of the reference's rendered chips (docs notebooks, 164 border chips: tests/golden).
#pragma once
#include <math.h>
#include <stdint.h>

#include "pip_device.h"

namespace mosaic {
namespace llclip {

struct Pt {
    double x, y;
};

// a position on C's boundary: side index and parameter in [0, 1) along it, ordered lexicographically
struct Pos {
    int32_t side;
    double s;
};
MOSAIC_HD bool pos_less(Pos a, Pos b) { return a.side != b.side ? a.side < b.side : a.s < b.s; }
MOSAIC_HD bool pos_eq(Pos a, Pos b) { return a.side == b.side && a.s == b.s; }

MOSAIC_HD bool same(Pt a, Pt b) { return a.x == b.x && a.y == b.y; }
MOSAIC_HD double mn(double a, double b) { return a < b ? a : b; }
MOSAIC_HD double mx(double a, double b) { return a > b ? a : b; }
MOSAIC_HD int orient(Pt a, Pt b, Pt c) { return pip::orientation_index(a.x, a.y, b.x, b.y, c.x, c.y); }
// Envelope(a, b).contains(r), inclusive
MOSAIC_HD bool in_env(Pt r, Pt a, Pt b) {
    return r.x >= mn(a.x, b.x) && r.x <= mx(a.x, b.x) && r.y >= mn(a.y, b.y) && r.y <= mx(a.y, b.y);
}
MOSAIC_HD bool env_meet(Pt a, Pt b, Pt c, Pt d) {
    return !(mx(a.x, b.x) < mn(c.x, d.x) || mn(a.x, b.x) > mx(c.x, d.x) || mx(a.y, b.y) < mn(c.y, d.y) ||
             mn(a.y, b.y) > mx(c.y, d.y));
}

// JTS Distance.pointToSegment
MOSAIC_HD double pt_dist(Pt p, Pt a) {
    const double dx = p.x - a.x, dy = p.y - a.y;
    return sqrt(dx * dx + dy * dy);
}
MOSAIC_HD double point_to_segment(Pt p, Pt a, Pt b) {
    if (a.x == b.x && a.y == b.y) return pt_dist(p, a);
    const double len2 = (b.x - a.x) * (b.x - a.x) + (b.y - a.y) * (b.y - a.y);
    const double r = ((p.x - a.x) * (b.x - a.x) + (p.y - a.y) * (b.y - a.y)) / len2;
    if (r <= 0.0) return pt_dist(p, a);
    if (r >= 1.0) return pt_dist(p, b);
    const double s = ((a.y - p.y) * (b.x - a.x) - (a.x - p.x) * (b.y - a.y)) / len2;
    return fabs(s) * sqrt(len2);
}
// RobustLineIntersector.nearestEndpoint
MOSAIC_HD Pt nearest_endpoint(Pt p1, Pt p2, Pt q1, Pt q2) {
    Pt best = p1;
    double md = point_to_segment(p1, q1, q2), d = point_to_segment(p2, q1, q2);
    if (d < md) md = d, best = p2;
    d = point_to_segment(q1, p1, p2);
    if (d < md) md = d, best = q1;
    d = point_to_segment(q2, p1, p2);
    if (d < md) md = d, best = q2;
    return best;
}
// Intersection.intersection (JTS 1.19) + RobustLineIntersector.intersection's envelope check
MOSAIC_HD Pt intersection(Pt p1, Pt p2, Pt q1, Pt q2) {
    const double int_min_x = mx(mn(p1.x, p2.x), mn(q1.x, q2.x)), int_max_x = mn(mx(p1.x, p2.x), mx(q1.x, q2.x));
    const double int_min_y = mx(mn(p1.y, p2.y), mn(q1.y, q2.y)), int_max_y = mn(mx(p1.y, p2.y), mx(q1.y, q2.y));
    const double midx = (int_min_x + int_max_x) / 2.0, midy = (int_min_y + int_max_y) / 2.0;
    const double p1x = p1.x - midx, p1y = p1.y - midy, p2x = p2.x - midx, p2y = p2.y - midy;
    const double q1x = q1.x - midx, q1y = q1.y - midy, q2x = q2.x - midx, q2y = q2.y - midy;
    const double px = p1y - p2y, py = p2x - p1x, pw = p1x * p2y - p2x * p1y;
    const double qx = q1y - q2y, qy = q2x - q1x, qw = q1x * q2y - q2x * q1y;
    const double x = py * qw - qy * pw, y = qx * pw - px * qw, w = px * qy - qx * py;
    const double xi = x / w, yi = y / w;
    Pt r;
    if (isnan(xi) || isinf(xi) || isnan(yi) || isinf(yi)) {
        r = nearest_endpoint(p1, p2, q1, q2);
    } else {
        r = Pt{xi + midx, yi + midy};
    }
    if (!(in_env(r, p1, p2) && in_env(r, q1, q2))) r = nearest_endpoint(p1, p2, q1, q2);
    return r;
}

// RobustLineIntersector.computeIntersect of segment a-b with c-d: the points where they meet (0-2)
MOSAIC_HD int meet(Pt a, Pt b, Pt c, Pt d, Pt out[2]) {
    if (!env_meet(a, b, c, d)) return 0;
    const int pq1 = orient(a, b, c), pq2 = orient(a, b, d);
    if ((pq1 > 0 && pq2 > 0) || (pq1 < 0 && pq2 < 0)) return 0;
    const int qp1 = orient(c, d, a), qp2 = orient(c, d, b);
    if ((qp1 > 0 && qp2 > 0) || (qp1 < 0 && qp2 < 0)) return 0;
    if (pq1 == 0 && pq2 == 0 && qp1 == 0 && qp2 == 0) {  // collinear: computeCollinearIntersection
        const bool c_in = in_env(c, a, b), d_in = in_env(d, a, b), a_in = in_env(a, c, d), b_in = in_env(b, c, d);
        int n = 0;
        if (c_in && d_in) {
            out[n++] = c;
            out[n++] = d;
        } else if (a_in && b_in) {
            out[n++] = a;
            out[n++] = b;
        } else if (c_in && a_in) {
            out[n++] = c;
            if (!same(c, a) || !d_in) out[n++] = a;
        } else if (c_in && b_in) {
            out[n++] = c;
            if (!same(c, b) || !d_in) out[n++] = b;
        } else if (d_in && a_in) {
            out[n++] = d;
            if (!same(d, a) || !c_in) out[n++] = a;
        } else if (d_in && b_in) {
            out[n++] = d;
            if (!same(d, b) || !c_in) out[n++] = b;
        }
        if (n == 2 && same(out[0], out[1])) n = 1;
        return n;
    }
    if (pq1 == 0 || pq2 == 0 || qp1 == 0 || qp2 == 0) {
        if (same(a, c) || same(a, d)) out[0] = a;
        else if (same(b, c) || same(b, d)) out[0] = b;
        else if (pq1 == 0) out[0] = c;
        else if (pq2 == 0) out[0] = d;
        else if (qp1 == 0) out[0] = a;
        else out[0] = b;
        return 1;
    }
    out[0] = intersection(a, b, c, d);
    return 1;
}

// The cell polygon: nc vertices, counter-clockwise, open; its envelope.
struct Cell {
    Pt v[16];
    int nc;
    double x0, y0, x1, y1;
};
MOSAIC_HD void cell_init(Cell& C) {
    C.x0 = C.x1 = C.v[0].x;
    C.y0 = C.y1 = C.v[0].y;
    for (int i = 1; i < C.nc; i++) {
        C.x0 = mn(C.x0, C.v[i].x);
        C.x1 = mx(C.x1, C.v[i].x);
        C.y0 = mn(C.y0, C.v[i].y);
        C.y1 = mx(C.y1, C.v[i].y);
    }
}
MOSAIC_HD Pt cv(const Cell& C, int i) { return C.v[i >= C.nc ? i - C.nc : i]; }
// true when C can be clipped in the plane: >= 3 vertices, counter-clockwise, no side spanning more
// than 180 degrees of longitude (cells over the antimeridian or a pole are not planar polygons there)
MOSAIC_HD bool cell_ok(const Cell& C, bool lonlat) {
    if (C.nc < 3 || C.nc > 16) return false;
    double a = 0;
    for (int i = 0; i < C.nc; i++) {
        const Pt p = C.v[i], q = cv(C, i + 1);
        a += (p.x - C.v[0].x) * (q.y - C.v[0].y) - (q.x - C.v[0].x) * (p.y - C.v[0].y);
        if (lonlat && fabs(q.x - p.x) > 180.0) return false;
    }
    return a > 0;
}

// twice C's area (relative to its first vertex); result rings below 1e-12 of it are dropped
MOSAIC_HD double cell_area2(const Cell& C) {
    double a = 0;
    for (int i = 0; i < C.nc; i++) {
        const Pt p = C.v[i], q = cv(C, i + 1);
        a += (p.x - C.v[0].x) * (q.y - C.v[0].y) - (q.x - C.v[0].x) * (p.y - C.v[0].y);
    }
    return a;
}

// location of p against C: 0 exterior, 1 boundary, 2 interior (PointLocation / RayCrossingCounter)
MOSAIC_HD int locate_cell(Pt p, const Cell& C) {
    if (p.x < C.x0 || p.x > C.x1 || p.y < C.y0 || p.y > C.y1) return 0;
    bool odd = false;
    for (int i = 0; i < C.nc; i++) {
        const Pt a = C.v[i], b = cv(C, i + 1);
        if (orient(a, b, p) == 0 && in_env(p, a, b)) return 1;
        if ((a.y > p.y) != (b.y > p.y)) {
            const int o = orient(a, b, p);
            if ((o > 0) == (b.y > a.y)) odd = !odd;
        }
    }
    return odd ? 2 : 0;
}
// position on C's boundary of a point known to lie on side j (a computed crossing, or an original
// point on it): the parameter along the side's dominant axis (monotone in that coordinate, so two
// points of one side compare exactly); C's vertices get (index, 0)
MOSAIC_HD Pos pos_on(const Cell& C, int j, Pt q) {
    const Pt c = C.v[j], d = cv(C, j + 1);
    if (same(q, c)) return Pos{j, 0.0};
    if (same(q, d)) return Pos{j + 1 == C.nc ? 0 : j + 1, 0.0};
    const double dx = d.x - c.x, dy = d.y - c.y;
    double s = fabs(dx) >= fabs(dy) ? (q.x - c.x) / dx : (q.y - c.y) / dy;
    if (!(s > 0.0)) s = 0.0;
    if (s >= 1.0) s = 0.99999999999999989;  // (the largest double below 1)
    return Pos{j, s};
}
// the position of an original point on C's boundary; false if it is not on it
MOSAIC_HD bool pos_of(const Cell& C, Pt q, Pos* out) {
    for (int j = 0; j < C.nc; j++)
        if (same(q, C.v[j])) {
            *out = Pos{j, 0.0};
            return true;
        }
    for (int j = 0; j < C.nc; j++) {
        const Pt c = C.v[j], d = cv(C, j + 1);
        if (in_env(q, c, d) && orient(c, d, q) == 0) {
            *out = pos_on(C, j, q);
            return true;
        }
    }
    return false;
}

// ---- the geometry: closed rings as in the chip producer's flat arrays
// Optional ring indexes (ring_blocks below; null: none): per ring, the envelopes of its stored edges
// in blocks of kBlk -- the walks skip a block whose envelope cannot meet C (ring_chains) or the ray of
// a point (locate_part), with the same comparisons the skipped edges would make, so the result does
// not depend on them -- and Orientation.isCCW of every ring.
static constexpr int kBlk = 16;
struct Geom {
    const double* xy;             // interleaved vertices
    const int64_t* ring_offsets;  // ring r = vertices [ring_offsets[r], ring_offsets[r + 1]) (closed)
    const int64_t* part_rings;    // part p = rings [part_rings[p], part_rings[p + 1]); first = shell
    int64_t p0, p1;               // the geometry's parts
    const double* blk = nullptr;        // block envelopes (x0, y0, x1, y1), ring r's from ring_blk[r]
    const int64_t* ring_blk = nullptr;
    const uint8_t* ring_ccw = nullptr;  // isCCW per ring
};
MOSAIC_HD Pt gv(const Geom& g, int64_t v) { return Pt{g.xy[2 * v], g.xy[2 * v + 1]}; }

// Orientation.isCCW (JTS 1.19) of closed ring [vb, vb + n + 1)
MOSAIC_HD bool ring_is_ccw(const Geom& g, int64_t vb, int n) {
    if (n < 3) return false;
    Pt up_hi = gv(g, vb), up_low = up_hi;
    double prev_y = up_hi.y;
    int i_up_hi = 0;
    for (int i = 1; i <= n; i++) {
        const Pt p = gv(g, vb + i);
        if (p.y > prev_y && p.y >= up_hi.y) {
            up_hi = p;
            i_up_hi = i;
            up_low = gv(g, vb + i - 1);
        }
        prev_y = p.y;
    }
    if (i_up_hi == 0) return false;
    int i_down_low = i_up_hi;
    do {
        i_down_low = (i_down_low + 1) % n;
    } while (i_down_low != i_up_hi && gv(g, vb + i_down_low).y == up_hi.y);
    const Pt down_low = gv(g, vb + i_down_low);
    const int i_down_hi = i_down_low > 0 ? i_down_low - 1 : n - 1;
    const Pt down_hi = gv(g, vb + i_down_hi);
    if (same(up_hi, down_hi)) {
        if (same(up_low, up_hi) || same(down_low, up_hi) || same(up_low, down_low)) return false;
        return orient(up_low, up_hi, down_low) == 1;
    }
    return down_hi.x - up_hi.x < 0;
}

// The ring indexes of Geom: per ring its number of blocks; then per ring (host loop or one device lane
// per ring) its block envelopes from blk = Geom::blk + 4 ring_blk[r] and its orientation.
MOSAIC_HD int64_t ring_block_count(const int64_t* ro, int64_t r) {
    const int64_t n = ro[r + 1] - ro[r] - 1;
    return n > 0 ? (n + kBlk - 1) / kBlk : 0;
}
MOSAIC_HD void ring_blocks_one(const int64_t* ro, const double* xy, int64_t r, double* blk, uint8_t* ccw) {
    const Geom g{xy, ro, nullptr, 0, 0};
    const int64_t vb = ro[r], n = ro[r + 1] - vb - 1;
    *ccw = n >= 3 && n <= 0x7fffffff && ring_is_ccw(g, vb, (int)n) ? 1 : 0;
    for (int64_t j = 0; n > 0 && j * kBlk < n; j++) {
        double x0 = xy[2 * (vb + j * kBlk)], y0 = xy[2 * (vb + j * kBlk) + 1], x1 = x0, y1 = y0;
        const int64_t e = j * kBlk + kBlk < n ? j * kBlk + kBlk : n;
        for (int64_t v = vb + j * kBlk + 1; v <= vb + e; v++) {
            const double x = xy[2 * v], y = xy[2 * v + 1];
            x0 = x < x0 ? x : x0, x1 = x > x1 ? x : x1, y0 = y < y0 ? y : y0, y1 = y > y1 ? y : y1;
        }
        blk[4 * j] = x0, blk[4 * j + 1] = y0, blk[4 * j + 2] = x1, blk[4 * j + 3] = y1;
    }
}

// one ring walked with the interior on its left: oriented vertex k -> the stored vertex
struct RingRef {
    int64_t vb;  // first stored vertex
    int32_t n;   // open vertex count
    int32_t rev; // walk reversed
    int64_t blk = -1;  // the ring's first block envelope (Geom::blk), -1 without
};
MOSAIC_HD Pt rv(const Geom& g, const RingRef& r, int32_t k) {
    k %= r.n;
    return gv(g, r.vb + (r.rev ? (k == 0 ? 0 : r.n - k) : k));
}

struct Chain {   // one inside run of a ring
    Pt in, out;  // entry / exit points (on C's boundary)
    Pos pin, pout;
    RingRef ring;
    int32_t vstart, vcount;  // oriented vertices strictly inside the run
    int32_t next;            // the chain the boundary walk from `out` reaches
    int32_t part;
};
struct Out {     // one result ring
    int32_t kind;   // 0 linked chains (first chain a), 1 whole ring `ring`, 2 the cell
    int32_t a;
    RingRef ring;
    int32_t part;
    int32_t hole;   // 1: a hole (whole ring walked clockwise)
    int32_t npts, start;
    int32_t shell;  // holes: their shell's index in the result list
    Pt sp;          // the ring's lowest point (where it is written from)
    int32_t order;  // holes: rank within their shell (shells 0)
    int32_t skey;   // output group: a shell's own rank, a hole its shell's
};

// Scratch: caller-owned arrays (device: per-lane private arrays; host: vectors).
struct Work {
    Chain* ch;
    int32_t ch_cap;
    Out* out;
    int32_t out_cap;
    int32_t n_ch, n_out;
};

enum Status : int { kOk = 0, kOverflow = 1, kInconsistent = 2, kBadCell = 3 };

// the points of a result ring, in walk order, duplicates next to each other removed (f(Pt))
template <class F>
MOSAIC_HD void ring_points(const Geom& g, const Cell& C, const Work& w, const Out& o, F f) {
    bool have = false;
    Pt first = Pt{0, 0}, last = Pt{0, 0};
    auto emit = [&](Pt p) {
        if (have && same(p, last)) return;
        if (!have) first = p;
        have = true;
        last = p;
        f(p, false);
    };
    if (o.kind == 2) {
        for (int m = 0; m < C.nc; m++) emit(C.v[m]);
    } else if (o.kind == 1) {
        for (int32_t k = 0; k < o.ring.n; k++) emit(rv(g, o.ring, k));
    } else {
        int32_t c = o.a;
        for (int guard = 0; guard <= w.n_ch; guard++) {
            const Chain& h = w.ch[c];
            emit(h.in);
            for (int32_t i = 0; i < h.vcount; i++) emit(rv(g, h.ring, h.vstart + i));
            emit(h.out);
            const Chain& nx = w.ch[h.next];
            // C's vertices strictly between h.out and nx.in, counter-clockwise
            const bool wrap = pos_less(nx.pin, h.pout);
            int32_t m = h.pout.side + 1;
            for (int step = 0; step < C.nc; step++, m++) {
                if (m == C.nc) {
                    if (!wrap) break;
                    m = 0;
                }
                const Pos pm = Pos{m, 0.0};
                if (wrap && m > h.pout.side) {
                    emit(C.v[m]);
                    continue;
                }
                if (!pos_less(pm, nx.pin)) break;
                emit(C.v[m]);
            }
            c = h.next;
            if (c == o.a) break;
        }
    }
    if (have && same(first, last)) f(last, true);  // the closing duplicate: callers drop it
}

// ring statistics: point count, lowest point and its index, twice the signed area (relative to the
// first point), all over the deduplicated sequence (a final point equal to the first is dropped)
MOSAIC_HD void ring_stats(const Geom& g, const Cell& C, const Work& w, Out& o, double* area2) {
    int32_t n = 0, lo = 0;
    Pt low = Pt{0, 0}, p0 = Pt{0, 0}, prev = Pt{0, 0};
    double a = 0;
    bool drop_last = false;
    ring_points(g, C, w, o, [&](Pt p, bool closing) {
        if (closing) {
            drop_last = true;
            return;
        }
        if (n == 0) {
            p0 = p;
            low = p;
        } else {
            a += (prev.x - p0.x) * (p.y - p0.y) - (p.x - p0.x) * (prev.y - p0.y);
            if (p.y < low.y || (p.y == low.y && p.x < low.x)) {
                low = p;
                lo = n;
            }
        }
        prev = p;
        n++;
    });
    if (drop_last) {
        // the sequence ended on its first point: that point was counted twice
        n--;
        if (lo == n) lo = 0;
    }
    o.npts = n;
    o.start = lo;
    o.sp = low;
    *area2 = a;
}

// location of p against a result ring (0 exterior, 1 boundary, 2 interior)
MOSAIC_HD int locate_out(Pt p, const Geom& g, const Cell& C, const Work& w, const Out& o) {
    bool odd = false, on = false, have = false;
    Pt first = Pt{0, 0}, prev = Pt{0, 0};
    auto seg = [&](Pt a, Pt b) {
        if (on) return;
        if (orient(a, b, p) == 0 && in_env(p, a, b)) {
            on = true;
            return;
        }
        if ((a.y > p.y) != (b.y > p.y)) {
            const int s = orient(a, b, p);
            if ((s > 0) == (b.y > a.y)) odd = !odd;
        }
    };
    ring_points(g, C, w, o, [&](Pt q, bool closing) {
        if (closing) return;
        if (!have) {
            first = q;
            have = true;
        } else {
            seg(prev, q);
        }
        prev = q;
    });
    if (have) seg(prev, first);
    return on ? 1 : (odd ? 2 : 0);
}

// location of p against the rings of part p (shell minus holes): 0 / 1 / 2
MOSAIC_HD int locate_part(Pt p, const Geom& g, int64_t part) {
    bool in_shell = false;
    for (int64_t r = g.part_rings[part]; r < g.part_rings[part + 1]; r++) {
        const int64_t vb = g.ring_offsets[r], n = g.ring_offsets[r + 1] - vb - 1;
        if (n < 3) continue;
        bool odd = false;
        for (int64_t i = 0; i < n; i++) {
            if (g.blk && i % kBlk == 0) {
                // a block wholly above or below p: no edge of it holds p or crosses its ray
                const double* b = g.blk + 4 * (g.ring_blk[r] + i / kBlk);
                if (b[1] > p.y || b[3] < p.y) {
                    i += kBlk - 1;
                    continue;
                }
            }
            const Pt a = gv(g, vb + i), b = gv(g, vb + i + 1);
            if (orient(a, b, p) == 0 && in_env(p, a, b)) return 1;
            if ((a.y > p.y) != (b.y > p.y)) {
                const int s = orient(a, b, p);
                if ((s > 0) == (b.y > a.y)) odd = !odd;
            }
        }
        if (r == g.part_rings[part]) {
            if (!odd) return 0;
            in_shell = true;
        } else if (odd) {
            return 0;
        }
    }
    return in_shell ? 2 : 0;
}

// The chains of one ring: returns kOk or kOverflow.  whole: 0 no inside piece, 1 wholly inside,
// 2 chains were added.
MOSAIC_HD int ring_chains(const Geom& g, const Cell& C, const RingRef& R, int32_t part, Work& w, int* whole) {
    const int32_t n = R.n;
    *whole = 0;
    // C's envelope misses the ring's vertices and edges entirely: nothing inside
    int cur = -1;       // label of the current piece (1 inside, 0 not), -1 before the first piece
    int first_lab = -1;
    int32_t open0 = -1; // a chain begun before the walk reached its first entry (the walk starts inside)
    int32_t start_ch = w.n_ch;
    bool any_in = false, any_out = false;
    Pt ev[40];
    Pos evp[40];
    double evt[40];
    for (int32_t k = 0; k < n; k++) {
        if (R.blk >= 0 && cur != 1) {
            // a stored block of edges starting at oriented edge k whose envelope misses C's: each of
            // its edges is a single piece outside C (the walk cannot be inside at its first vertex,
            // which lies outside C's envelope)
            int32_t j = -1, m = 0;
            if (!R.rev) {
                if (k % kBlk == 0) j = k / kBlk, m = n - k < kBlk ? n - k : kBlk;
            } else if ((n - k) % kBlk == 0) {
                j = (n - k) / kBlk - 1, m = kBlk;  // stored edges n - k - kBlk .. n - k - 1
            }
            if (j >= 0) {
                const double* e = g.blk + 4 * (R.blk + j);
                if (e[2] < C.x0 || e[0] > C.x1 || e[3] < C.y0 || e[1] > C.y1) {
                    any_out = true;
                    if (cur == -1) first_lab = 0;
                    cur = 0;
                    k += m - 1;
                    continue;
                }
            }
        }
        const Pt a = rv(g, R, k), b = rv(g, R, k + 1);
        if (same(a, b)) continue;
        int ne = 0;
        const bool touch = !(mx(a.x, b.x) < C.x0 || mn(a.x, b.x) > C.x1 || mx(a.y, b.y) < C.y0 || mn(a.y, b.y) > C.y1);
        if (touch) {
            for (int j = 0; j < C.nc; j++) {
                Pt q[2];
                const int m = meet(a, b, C.v[j], cv(C, j + 1), q);
                for (int t = 0; t < m; t++) {
                    if (same(q[t], a) || same(q[t], b)) continue;
                    const double dx = b.x - a.x, dy = b.y - a.y;
                    const double tt = fabs(dx) >= fabs(dy) ? (q[t].x - a.x) / dx : (q[t].y - a.y) / dy;
                    // insert sorted by the parameter along a -> b; drop exact duplicates
                    bool dup = false;
                    for (int u = 0; u < ne; u++)
                        if (same(ev[u], q[t])) dup = true;
                    if (dup) continue;
                    if (ne == 40) return kOverflow;
                    int u = ne++;
                    while (u > 0 && evt[u - 1] > tt) {
                        ev[u] = ev[u - 1];
                        evp[u] = evp[u - 1];
                        evt[u] = evt[u - 1];
                        u--;
                    }
                    ev[u] = q[t];
                    evp[u] = pos_on(C, j, q[t]);
                    evt[u] = tt;
                }
            }
        }
        const int la = touch ? locate_cell(a, C) : 0, lb = touch ? locate_cell(b, C) : 0;
        // pieces a -> ev[0] -> ... -> ev[ne-1] -> b
        for (int i = 0; i <= ne; i++) {
            const Pt p0 = i == 0 ? a : ev[i - 1], p1 = i == ne ? b : ev[i];
            int lab;
            if (!touch) {
                lab = 0;
            } else if (i == 0 && la != 1) {
                lab = la == 2;
            } else if (i == ne && lb != 1) {
                lab = lb == 2;
            } else {
                lab = locate_cell(Pt{(p0.x + p1.x) / 2, (p0.y + p1.y) / 2}, C) == 2;
            }
            if (lab) any_in = true;
            else any_out = true;
            if (cur == -1) {
                first_lab = lab;
                if (lab) {
                    // the walk starts inside: an open chain whose entry is found at the end
                    if (w.n_ch >= w.ch_cap) return kOverflow;
                    open0 = w.n_ch++;
                    Chain& h = w.ch[open0];
                    h.ring = R;
                    h.part = part;
                    h.vstart = 0;
                    h.vcount = 0;
                    h.next = -1;
                }
            } else if (lab != cur) {
                // transition at p0 (a vertex when i == 0, else an event point)
                Pos ps;
                if (i == 0) {
                    if (!pos_of(C, p0, &ps)) return kInconsistent;
                } else {
                    ps = evp[i - 1];
                }
                if (lab) {  // entry
                    if (w.n_ch >= w.ch_cap) return kOverflow;
                    Chain& h = w.ch[w.n_ch++];
                    h.in = p0;
                    h.pin = ps;
                    h.ring = R;
                    h.part = part;
                    h.vstart = k + 1;
                    h.vcount = 0;
                    h.next = -1;
                } else {  // exit: closes the last chain
                    Chain& h = w.ch[w.n_ch - 1];
                    h.out = p0;
                    h.pout = ps;
                    // the chain's inside vertices: from vstart to the vertex before p0
                    const int32_t last = i == 0 ? k - 1 : k;  // oriented index of the last inside vertex
                    int32_t cnt = last - h.vstart + 1;
                    if (w.n_ch - 1 == open0) cnt = last + 1;  // (the open chain starts at vertex 0)
                    h.vcount = cnt < 0 ? 0 : cnt;
                }
            }
            cur = lab;
            // a vertex strictly inside a run: counted when the run closes (vstart..last)
        }
    }
    if (cur == -1) return kOk;  // (a ring of one repeated point)
    if (!any_out) {
        w.n_ch = start_ch;
        *whole = 1;
        return kOk;
    }
    if (!any_in) return kOk;
    // the walk ends where it began: the label change (if any) between the last piece and the first
    // is at vertex 0
    const Pt w0 = rv(g, R, 0);
    if (first_lab == 1 && cur == 1) {
        // the last chain (entered, never exited) continues into the open chain
        if (w.n_ch - 1 == open0) return kInconsistent;
        Chain& last = w.ch[w.n_ch - 1];
        Chain& op = w.ch[open0];
        last.out = op.out;
        last.pout = op.pout;
        last.vcount = (n - last.vstart) + op.vcount;
        op = last;  // the open chain was the last one's tail
        w.n_ch--;
    } else if (first_lab == 1) {
        // entry at vertex 0: the open chain's inside vertices start after it
        Pos ps;
        if (!pos_of(C, w0, &ps)) return kInconsistent;
        Chain& op = w.ch[open0];
        op.in = w0;
        op.pin = ps;
        op.vstart = 1;
        op.vcount = op.vcount > 0 ? op.vcount - 1 : 0;
    } else if (cur == 1) {
        // exit at vertex 0
        Pos ps;
        if (!pos_of(C, w0, &ps)) return kInconsistent;
        Chain& h = w.ch[w.n_ch - 1];
        h.out = w0;
        h.pout = ps;
        h.vcount = n - h.vstart;
    }
    *whole = 2;
    return kOk;
}

// Clip the geometry against C.  On kOk, w.out[0 .. n_out) are the result rings with npts / start /
// sp set, shells first in output order, each followed by its holes; *polys = number of shells;
// *is_cell = the result is exactly C (one shell, no holes, the same vertices).
MOSAIC_HD int clip(const Geom& g, const Cell& C, Work& w, double area_eps2, int32_t* polys, bool* is_cell) {
    w.n_ch = 0;
    w.n_out = 0;
    *polys = 0;
    *is_cell = false;
    for (int64_t p = g.p0; p < g.p1; p++) {
        const int32_t ch0 = w.n_ch, out0 = w.n_out;
        bool shell_inside = false;
        for (int64_t r = g.part_rings[p]; r < g.part_rings[p + 1]; r++) {
            const int64_t vb = g.ring_offsets[r];
            const int32_t n = (int32_t)(g.ring_offsets[r + 1] - vb - 1);
            if (n < 3) continue;
            const bool shell = r == g.part_rings[p];
            const bool ccw = g.ring_ccw ? g.ring_ccw[r] != 0 : ring_is_ccw(g, vb, n);
            RingRef R{vb, n, (int32_t)(ccw != shell), g.blk ? g.ring_blk[r] : -1};
            int whole = 0;
            const int st = ring_chains(g, C, R, (int32_t)p, w, &whole);
            if (st) return st;
            if (whole == 1) {
                if (w.n_out >= w.out_cap) return kOverflow;
                Out& o = w.out[w.n_out++];
                o.kind = 1;
                o.a = -1;
                o.ring = R;
                o.part = (int32_t)p;
                o.hole = shell ? 0 : 1;
                o.shell = -1;
                if (shell) shell_inside = true;
            }
        }
        // link the part's chains: from each exit to the next entry counter-clockwise
        for (int32_t c = ch0; c < w.n_ch; c++) {
            int32_t best = -1, best_wrap = -1;
            for (int32_t e = ch0; e < w.n_ch; e++) {
                const Pos pe = w.ch[e].pin;
                if (!pos_less(pe, w.ch[c].pout)) {
                    if (best < 0 || pos_less(pe, w.ch[best].pin)) best = e;
                } else if (best_wrap < 0 || pos_less(pe, w.ch[best_wrap].pin)) {
                    best_wrap = e;
                }
            }
            w.ch[c].next = best >= 0 ? best : best_wrap;
        }
        // every entry must be reached by exactly one exit (a permutation)
        for (int32_t c = ch0; c < w.n_ch; c++) {
            int32_t hits = 0;
            for (int32_t e = ch0; e < w.n_ch; e++) hits += w.ch[e].next == c;
            if (hits != 1) return kInconsistent;
        }
        // the cycles of the permutation are the linked shells
        for (int32_t c = ch0; c < w.n_ch; c++) {
            bool seen = false;
            for (int32_t o = out0; o < w.n_out; o++)
                if (w.out[o].kind == 0) {
                    int32_t x = w.out[o].a;
                    for (int guard = 0; guard <= w.n_ch; guard++) {
                        if (x == c) seen = true;
                        x = w.ch[x].next;
                        if (x == w.out[o].a) break;
                    }
                }
            if (seen) continue;
            if (w.n_out >= w.out_cap) return kOverflow;
            Out& o = w.out[w.n_out++];
            o.kind = 0;
            o.a = c;
            o.ring = w.ch[c].ring;
            o.part = (int32_t)p;
            o.hole = 0;
            o.shell = -1;
        }
        // no ring crosses C and the shell is not inside it: C is a shell of the result when it lies in
        // the part (tested at a vertex of C on no ring, else at C's vertex mean)
        if (ch0 == w.n_ch && !shell_inside) {
            int loc = 1;
            for (int m = 0; m < C.nc && loc == 1; m++) loc = locate_part(C.v[m], g, p);
            if (loc == 1) {
                double sx = 0, sy = 0;
                for (int m = 0; m < C.nc; m++) sx += C.v[m].x, sy += C.v[m].y;
                loc = locate_part(Pt{sx / C.nc, sy / C.nc}, g, p);
            }
            if (loc == 2) {
                if (w.n_out >= w.out_cap) return kOverflow;
                Out& o = w.out[w.n_out++];
                o.kind = 2;
                o.a = -1;
                o.ring = RingRef{0, 0, 0};
                o.part = (int32_t)p;
                o.hole = 0;
                o.shell = -1;
            }
        }
    }
    // statistics; drop rings without area
    int32_t k = 0;
    for (int32_t o = 0; o < w.n_out; o++) {
        double a2;
        ring_stats(g, C, w, w.out[o], &a2);
        if (w.out[o].npts < 3 || !(fabs(a2) > area_eps2)) continue;
        w.out[k++] = w.out[o];
    }
    w.n_out = k;
    // shells in output order (lowest point: y, then x), then holes to the shell of their part that
    // holds them, in the same order
    int32_t ns = 0;
    for (int32_t o = 0; o < w.n_out; o++)
        if (!w.out[o].hole) {
            Out t = w.out[o];
            int32_t u = o;
            while (u > ns) {
                w.out[u] = w.out[u - 1];
                u--;
            }
            w.out[ns++] = t;
        }
    for (int32_t a = 1; a < ns; a++) {  // insertion sort of the shells by lowest point
        Out t = w.out[a];
        int32_t u = a;
        while (u > 0 && (w.out[u - 1].sp.y > t.sp.y || (w.out[u - 1].sp.y == t.sp.y && w.out[u - 1].sp.x > t.sp.x))) {
            w.out[u] = w.out[u - 1];
            u--;
        }
        w.out[u] = t;
    }
    for (int32_t h = ns; h < w.n_out; h++) {
        Out& o = w.out[h];
        o.shell = -1;
        const Pt q = o.sp;
        for (int32_t s = 0; s < ns && o.shell < 0; s++)
            if (w.out[s].part == o.part && locate_out(q, g, C, w, w.out[s]) == 2) o.shell = s;
        if (o.shell < 0)
            for (int32_t s = 0; s < ns && o.shell < 0; s++)
                if (w.out[s].part == o.part) o.shell = s;
        if (o.shell < 0) o.shell = 0;
    }
    // final order: each shell followed by its holes (by lowest point)
    for (int32_t s = 0; s < ns; s++) {
        w.out[s].skey = s;
        w.out[s].order = 0;
    }
    for (int32_t h = ns; h < w.n_out; h++) {
        int32_t rank = 0;
        const Out& o = w.out[h];
        for (int32_t q = ns; q < w.n_out; q++) {
            const Out& v = w.out[q];
            if (q == h || v.shell != o.shell) continue;
            if (v.sp.y < o.sp.y || (v.sp.y == o.sp.y && (v.sp.x < o.sp.x || (v.sp.x == o.sp.x && q < h)))) rank++;
        }
        w.out[h].skey = o.shell;
        w.out[h].order = rank + 1;
    }
    for (int32_t a = 1; a < w.n_out; a++) {  // stable insertion sort by (skey, order)
        Out t = w.out[a];
        int32_t u = a;
        while (u > 0 && (w.out[u - 1].skey > t.skey || (w.out[u - 1].skey == t.skey && w.out[u - 1].order > t.order))) {
            w.out[u] = w.out[u - 1];
            u--;
        }
        w.out[u] = t;
    }
    *polys = ns;
    if (ns == 1 && w.n_out == 1 && w.out[0].npts == C.nc) {
        // exactly C: the points are C's vertices
        bool all = true;
        ring_points(g, C, w, w.out[0], [&](Pt p, bool closing) {
            if (closing) return;
            bool f = false;
            for (int m = 0; m < C.nc; m++) f = f || same(p, C.v[m]);
            all = all && f;
        });
        *is_cell = all;
    }
    return kOk;
}

// Write result ring o from its lowest point, closed: npts + 1 points into dst (interleaved).
MOSAIC_HD void write_ring(const Geom& g, const Cell& C, const Work& w, const Out& o, double* dst) {
    int32_t i = 0;
    const int32_t n = o.npts;
    ring_points(g, C, w, o, [&](Pt p, bool closing) {
        if (closing || i >= n) return;
        int32_t k = i - o.start;
        if (k < 0) k += n;
        dst[2 * k] = p.x;
        dst[2 * k + 1] = p.y;
        i++;
    });
    dst[2 * n] = dst[0];
    dst[2 * n + 1] = dst[1];
}

}  // namespace llclip
}  // namespace mosaic
