// Host-compiled (g++) half of the H3 tile directory and point raster (tiles.h): the builders read
// the H3 tables as host constants.  Linked into libmosaic_hip.so next to mosaic_hip.o.
//
// Point raster.  Each non-empty tile is cut into S x S sub-blocks and, where needed, each
// sub-block into C x C cells.  A rectangle R (sub-block or cell, widened by eps) gets a code
// valid for EVERY point of R:
//   * the hexagons R can reach: R's image on the tile's face is the quadrilateral of its corner
//     images to within rect_tol (tiles.h: the tile's closed-form bound on the map's second
//     derivatives, scaled by R's size, plus R's widening); every window
//     hexagon (exact Voronoi hexagon of the face lattice, H3's _hex2dToCoordIJK rounding) that the
//     quadrilateral meets within a tolerance (separating-axis test) is a candidate.  H3 assigns
//     each point of R one of them.
//   * per candidate hexagon h, the answer of its points in R: the keys of h's core chips plus the
//     keys of h's border chips containing the point.  When no segment of any border chip of h
//     meets R, each border chip's contains() is constant on R (R is connected and misses the
//     chip's boundary), so it is evaluated once, at R's centre, with the JTS restatement.
//   * R's code is that answer if all candidates agree and it is empty or one key; otherwise
//     kMixed (sub-blocks: split into cells; cells: the tile path runs for their points).
// Reference semantics followed: the chip join = H3 cell equality (H3IndexSystem.scala:140-142) +
// is_core || st_contains (QuickstartNotebook.py:205-219, ST_Contains.scala:34-42).
#include "tiles.h"
#include "raster_build.h"

#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>

namespace mosaic {
namespace tiles {

bool Builder::build(int res, const std::vector<int64_t>& cells, const std::function<int64_t(int64_t)>& slot_of) {
    return build_impl(res, cells, slot_of);
}

namespace {

using rbuild::clip_half;
using rbuild::clip_seg;
using rbuild::kS60;
using rbuild::P2;
using rbuild::seg_meets_poly;

struct Seg {
    double ax, ay, bx, by;
};

struct Rect {
    double x0, y0, x1, y1;
};

void chip_segments(const pip::GeomStore& s, uint32_t g, std::vector<Seg>& out) {
    out.clear();
    for (uint32_t p = s.geom_part[g]; p < s.geom_part[g + 1]; p++)
        for (uint32_t r = s.part_ring[p]; r < s.part_ring[p + 1]; r++)
            for (uint32_t v = s.ring_start[r] + 1; v < s.ring_start[r + 1]; v++)
                out.push_back(Seg{s.verts[v - 1].x, s.verts[v - 1].y, s.verts[v].x, s.verts[v].y});
}

bool any_seg_meets(const std::vector<Seg>& segs, const Rect& r) {
    for (const Seg& e : segs)
        if (raster::seg_meets_rect(e.ax, e.ay, e.bx, e.by, r.x0, r.y0, r.x1, r.y1)) return true;
    return false;
}

// One window hexagon's chips, prepared for classification.
struct Hex {
    P2 c;                       // lattice centre (face plane, hex units)
    std::vector<int32_t> core;  // keys of core chips
    std::vector<uint32_t> border;
    std::vector<int32_t> border_key;
    std::vector<std::vector<Seg>> segs;  // per border chip
    std::vector<pip::Box> bbox;
};

const rbuild::HexTable& hex_table() {
    static const rbuild::HexTable t = rbuild::hex_table();
    return t;
}

}  // namespace

rbuild::HexTable Builder::hex_table_values() { return hex_table(); }

bool Builder::raster_setup(const ChipSource& src, int S_, int C_) {
    S = S_;
    C = C_;
    sub.clear();
    tile_base.clear();
    tile_lbase.clear();
    llines.clear();
    blocks.clear();
    quad.clear();
    qrec_mask.clear();
    qrec_code.clear();
    qrec_shift = 0;
    n_sub_pure = n_sub_mixed = n_cell_mixed = n_sub_line = n_cell_line = 0;
    if (tile_idx.empty() || S < 1 || S > 128 || (S & (S - 1)) || C < 1 || (C & (C - 1)) || S * C > 1024) return false;
    if (src.n_polygons > (int32_t)kMaxRasterKeys) return false;  // codes must stay below kSubBlock
    sshift = 0;
    while ((1 << sshift) < S) sshift++;
    cshift = 0;
    while ((1 << cshift) < C) cshift++;
    if ((int64_t)grid.nx * S * grid.ny * S > ((int64_t)1 << 28)) return false;
    tile_of_rec.assign(recs.size(), -1);
    for (int64_t t = 0; t < (int64_t)grid.nx * grid.ny; t++)
        if (tile_idx[(size_t)t] >= 2) tile_of_rec[tile_idx[(size_t)t] - 2] = (int)t;
    return true;
}

bool Builder::build_raster(const ChipSource& src, int S_, int C_, int threads) {
    if (!raster_setup(src, S_, C_)) return false;
    RasterClass rc;
    classify_raster_host(src, threads, rc);
    return assemble_raster(rc, threads);
}

// Phase 1 on the host: every sub-block's code (kMixed for mixed ones), and for the mixed ones a
// line record or their C x C cell codes.
void Builder::classify_raster_host(const ChipSource& src, int threads, RasterClass& rc) {
    const int nx = grid.nx, N = S * C;
    const double tw = 1.0 / grid.sx, th = 1.0 / grid.sy;
    const rbuild::HexTable& ht = hex_table();
    const size_t SS = (size_t)S * S;
    rc.code.assign(recs.size() * SS, (uint16_t)0);
    // per record: its mixed sub-blocks' results (concatenated in record order afterwards)
    std::vector<std::vector<uint8_t>> r_kind(recs.size());
    std::vector<std::vector<LineRec>> r_line(recs.size());
    std::vector<std::vector<uint16_t>> r_cells(recs.size());
    std::vector<std::vector<uint32_t>> r_cline_at(recs.size());  // leaf lines: cell (record-local) ...
    std::vector<std::vector<LineRec>> r_cline(recs.size());      // ... and its record
    std::atomic<int64_t> next(0);

    auto work = [&]() {
        std::vector<P2> lat;  // (S + 1)^2 sub-block corner images
        std::vector<Hex> hexes;
        std::vector<int> cand, cand2;
        std::vector<int32_t> ans, ah;
        std::vector<Seg> segs_tmp;
        while (true) {
            int64_t ri = next.fetch_add(1);
            if (ri >= (int64_t)recs.size()) break;
            const TileRec& tr = recs[(size_t)ri];
            int t = tile_of_rec[(size_t)ri];
            if (t < 0 || tr.dims == 0) continue;
            const int ti = t % nx, tj = t / nx;
            const int face = (int)(tr.dims & 0xffu), wa = (int)((tr.dims >> 8) & 0xfffu), wb = (int)(tr.dims >> 20);
            const double lon0 = grid.x0 + ti * tw, lat0 = grid.y0 + tj * th;
            // lattice images on the tile's face: sub-block corners now, cell corners of a
            // sub-block only when it needs its cells
            auto image = [&](double i, double j) -> P2 {
                double px, py, pz, vx, vy, b;
                h3::fast_unit(lat0 + th * j / N, lon0 + tw * i / N, &px, &py, &pz);
                h3::fast_plane(px, py, pz, face, res_, &vx, &vy, &b);
                return P2{vx, vy};
            };
            lat.resize((size_t)(S + 1) * (S + 1));
            for (int j = 0; j <= S; j++)
                for (int i = 0; i <= S; i++) lat[(size_t)j * (S + 1) + i] = image(i * C, j * C);
            std::vector<P2> clat((size_t)(C + 1) * (C + 1));
            // window hexagons
            hexes.assign((size_t)wa * wb, Hex());
            for (int ra = 0; ra < wa; ra++)
                for (int rb = 0; rb < wb; rb++) {
                    Hex& h = hexes[(size_t)ra * wb + rb];
                    int a = tr.a0 + ra, bb = tr.b0 + rb;
                    h.c = P2{(double)a - 0.5 * (double)bb, (double)bb * kS60};
                    uint32_t e = entries[tr.off + (uint32_t)(ra * wb + rb)];
                    if (!e) continue;
                    uint32_t f0 = src.slot_first[e - 1], n0 = src.slot_count[e - 1];
                    for (uint32_t cidx = f0; cidx < f0 + n0; cidx++) {
                        uint32_t m = src.meta[cidx];
                        if (m & 1u) {
                            h.core.push_back((int32_t)(m >> 1));
                        } else {
                            h.border.push_back(cidx);
                            h.border_key.push_back((int32_t)(m >> 1));
                            chip_segments(src.store, cidx, segs_tmp);
                            h.segs.push_back(segs_tmp);
                            h.bbox.push_back(src.store.geom_bbox[cidx]);
                        }
                    }
                    std::sort(h.core.begin(), h.core.end());
                }
            const TileCurv cv = rec_curv[(size_t)ri];
            const double cell_deg_x = tw / N, cell_deg_y = th / N;
            // classification of the fine-lattice rectangle [i0, i1] x [j0, j1] whose corner images
            // are q (counter-clockwise), with candidate hexagons `cin` -> code; `cout` receives the
            // candidates it meets
            auto classify = [&](int i0, int j0, int i1, int j1, const P2* q, const std::vector<int>& cin,
                                std::vector<int>& cout) -> uint16_t {
                double ex = 1e-6 * cell_deg_x + 1e-12 * (fabs(lon0) + 1.0);
                double ey = 1e-6 * cell_deg_y + 1e-12 * (fabs(lat0) + 1.0);
                const double tol = rect_tol(cv, cell_deg_x * (i1 - i0), cell_deg_y * (j1 - j0), std::max(ex, ey));
                cout.clear();
                for (int k : cin)
                    if (rbuild::poly_meets_hex(q, 4, hexes[(size_t)k].c, tol, ht)) cout.push_back(k);
                Rect r;
                r.x0 = lon0 + tw * i0 / N - ex;
                r.x1 = lon0 + tw * i1 / N + ex;
                r.y0 = lat0 + th * j0 / N - ey;
                r.y1 = lat0 + th * j1 / N + ey;
                double cxm = lon0 + tw * (i0 + i1) / (2.0 * N), cym = lat0 + th * (j0 + j1) / (2.0 * N);
                bool first = true;
                bool mixed_ans = false;
                for (int k : cout) {
                    const Hex& h = hexes[(size_t)k];
                    ah = h.core;
                    for (size_t b = 0; b < h.border.size(); b++) {
                        const pip::Box& bx = h.bbox[b];
                        if (!(bx.maxx < r.x0 || bx.minx > r.x1 || bx.maxy < r.y0 || bx.miny > r.y1) &&
                            any_seg_meets(h.segs[b], r))
                            return kMixed;
                        if (pip::contains(src.store, h.border[b], cxm, cym)) ah.push_back(h.border_key[b]);
                    }
                    std::sort(ah.begin(), ah.end());
                    if (first) {
                        ans = ah;
                        first = false;
                    } else if (ah != ans) {
                        mixed_ans = true;
                    }
                }
                if (mixed_ans || cout.empty()) return kMixed;  // no candidate: cannot happen; stay safe
                if (ans.empty()) return 0;
                if (ans.size() == 1) return (uint16_t)(ans[0] + 1);
                return kMixed;
            };
            // classification of the convex region uv[n] (sub-block units, counter-clockwise) of
            // sub-block (si, sj) with candidate hexagons `cin` (those of the whole sub-block) -> code
            const double exd = 1e-6 * cell_deg_x + 1e-12 * (fabs(lon0) + 1.0);
            const double eyd = 1e-6 * cell_deg_y + 1e-12 * (fabs(lat0) + 1.0);
            auto classify_poly = [&](int si, int sj, const P2* uv, int n, const std::vector<int>& cin) -> uint16_t {
                P2 img[8], ll[8];
                double u0 = INFINITY, u1 = -INFINITY, v0 = INFINITY, v1 = -INFINITY;
                double x0 = INFINITY, x1 = -INFINITY, y0 = INFINITY, y1 = -INFINITY, mx = 0.0, my = 0.0;
                for (int v = 0; v < n; v++) {
                    img[v] = image((si + uv[v].x) * C, (sj + uv[v].y) * C);
                    ll[v] = P2{lon0 + tw * (si + uv[v].x) / S, lat0 + th * (sj + uv[v].y) / S};
                    u0 = std::min(u0, uv[v].x);
                    u1 = std::max(u1, uv[v].x);
                    v0 = std::min(v0, uv[v].y);
                    v1 = std::max(v1, uv[v].y);
                    x0 = std::min(x0, ll[v].x);
                    x1 = std::max(x1, ll[v].x);
                    y0 = std::min(y0, ll[v].y);
                    y1 = std::max(y1, ll[v].y);
                    mx += ll[v].x;
                    my += ll[v].y;
                }
                mx /= n;  // a point inside the (convex) region
                my /= n;
                const double eps = std::max(exd, eyd);
                const double tol = poly_tol(cv, tw * (u1 - u0) / S, th * (v1 - v0) / S, eps);
                bool first = true, mixed_ans = false, any = false;
                for (int k : cin) {
                    const Hex& h = hexes[(size_t)k];
                    if (!rbuild::poly_meets_hex(img, n, h.c, tol, ht)) continue;
                    any = true;
                    ah = h.core;
                    for (size_t b = 0; b < h.border.size(); b++) {
                        const pip::Box& bx = h.bbox[b];
                        if (!(bx.maxx < x0 - eps || bx.minx > x1 + eps || bx.maxy < y0 - eps || bx.miny > y1 + eps))
                            for (const Seg& e : h.segs[b])
                                if (seg_meets_poly(P2{e.ax, e.ay}, P2{e.bx, e.by}, ll, n, eps)) return kMixed;
                        if (pip::contains(src.store, h.border[b], mx, my)) ah.push_back(h.border_key[b]);
                    }
                    std::sort(ah.begin(), ah.end());
                    if (first) {
                        ans = ah;
                        first = false;
                    } else if (ah != ans) {
                        mixed_ans = true;
                    }
                }
                if (mixed_ans || !any) return kMixed;
                if (ans.empty()) return 0;
                if (ans.size() == 1) return (uint16_t)(ans[0] + 1);
                return kMixed;
            };
            // a mixed sub-block whose chip edges all lie along one line: the line through the
            // longest clipped edge; both sides (beyond a margin, less the slack) must classify
            // The box is [u0, u1] x [v0, v1] in sub-block units: the whole sub-block, or one leaf cell
            // (a leaf line, tried margins 0 .. mk_end - 1) in the sub-block's frame.
            // tf: a sub-block line, in the tile frame (rbuild::line_slack_tile); else a leaf line in
            // the sub-block frame
            std::vector<P2> ends;
            auto try_line = [&](int si, int sj, double u0, double v0, double u1, double v1, int mk_end,
                                const std::vector<int>& cin, LineRec& out, bool tf) -> bool {
                const double wR = tw / S, hR = th / S;
                const double lonR0 = lon0 + tw * si / S, latR0 = lat0 + th * sj / S;
                const double exu = exd / wR, eyv = eyd / hR;
                const double bx0 = lonR0 + wR * u0 - exd, bx1 = lonR0 + wR * u1 + exd, by0 = latR0 + hR * v0 - eyd,
                             by1 = latR0 + hR * v1 + eyd;
                double best = 0.0;
                P2 pa{0, 0}, pb{0, 0}, ta{0, 0}, tb{0, 0};
                ends.clear();
                for (int k : cin) {
                    const Hex& h = hexes[(size_t)k];
                    for (size_t b = 0; b < h.border.size(); b++) {
                        const pip::Box& bx = h.bbox[b];
                        if (bx.maxx < bx0 || bx.minx > bx1 || bx.maxy < by0 || bx.miny > by1) continue;
                        for (const Seg& e : h.segs[b]) {
                            double ax = (e.ax - lonR0) / wR, ay = (e.ay - latR0) / hR;
                            double qx = (e.bx - lonR0) / wR, qy = (e.by - latR0) / hR;
                            if (!clip_seg(ax, ay, qx, qy, u0 - exu, v0 - eyv, u1 + exu, v1 + eyv)) continue;
                            ends.push_back(P2{ax, ay});
                            ends.push_back(P2{qx, qy});
                            const double l2 = (qx - ax) * (qx - ax) + (qy - ay) * (qy - ay);
                            if (l2 > best) {
                                best = l2;
                                pa = P2{ax, ay};
                                pb = P2{qx, qy};
                                ta = P2{(e.ax - lon0) / wR, (e.ay - lat0) / hR};
                                tb = P2{(e.bx - lon0) / wR, (e.by - lat0) / hR};
                            }
                        }
                    }
                }
                if (!(best > 1e-6)) return false;
                double a, b, c, dev_max = 0.0;
                if (tf) {  // the whole segment's line, tile frame
                    const double lt = sqrt((tb.x - ta.x) * (tb.x - ta.x) + (tb.y - ta.y) * (tb.y - ta.y));
                    a = -(tb.y - ta.y) / lt;
                    b = (tb.x - ta.x) / lt;
                    c = -(a * 0.5 * (ta.x + tb.x) + b * 0.5 * (ta.y + tb.y));
                    for (const P2& p : ends) dev_max = std::max(dev_max, fabs(a * (p.x + si) + b * (p.y + sj) + c));
                } else {
                    const double l = sqrt(best);
                    a = -(pb.y - pa.y) / l;
                    b = (pb.x - pa.x) / l;
                    c = -(a * 0.5 * (pa.x + pb.x) + b * 0.5 * (pa.y + pb.y));
                    for (const P2& p : ends) dev_max = std::max(dev_max, fabs(a * p.x + b * p.y + c));
                }
                const P2 sq[4] = {{u0 - exu, v0 - eyv}, {u1 + exu, v0 - eyv}, {u1 + exu, v1 + eyv}, {u0 - exu, v1 + eyv}};
                // the narrowest band (fewest rows to the mixed kernel) whose two sides certify
                for (int mk = 0; mk < mk_end; mk++) {
                    const double margin = rbuild::line_margin(mk);
                    if (dev_max > margin - 2.0 * kLineSlack) continue;
                    out.a = (float)(a / margin);
                    out.b = (float)(b / margin);
                    out.c = (float)(c / margin);
                    // certify with the coefficients the device uses: device side + implies
                    // A u + B v + C >= 1 - (float error) >= 1 - kLineSlack / margin (tile frame:
                    // the sub-block's own C = Ct + A si + B sj, and line_slack_tile)
                    const double A = out.a, B = out.b;
                    const double Cf = tf ? (double)out.c + A * si + B * sj : (double)out.c;
                    const double m = 1.0 - (tf ? rbuild::line_slack_tile(A, B, out.c, S, kLineSlack) : kLineSlack / margin);
                    P2 hp[8], hn[8];
                    const int np = clip_half(sq, 4, A, B, Cf - m, hp), nn = clip_half(sq, 4, -A, -B, -Cf - m, hn);
                    const uint16_t cp = np >= 3 ? classify_poly(si, sj, hp, np, cin) : 0;
                    if (cp == kMixed) continue;
                    const uint16_t cn = nn >= 3 ? classify_poly(si, sj, hn, nn, cin) : 0;
                    if (cn == kMixed) continue;
                    out.pos = cp;
                    out.neg = cn;
                    // the device evaluates the line at leaf-cell offsets u C, v C: a / C, b / C
                    // (C a power of two: the same products, bit for bit)
                    out.a = (float)((double)out.a / C);
                    out.b = (float)((double)out.b / C);
                    return true;
                }
                return false;
            };
            std::vector<int> all((size_t)wa * wb);
            for (size_t k = 0; k < all.size(); k++) all[k] = (int)k;
            uint16_t* rcode = rc.code.data() + (size_t)ri * SS;
            std::vector<uint16_t> cellc((size_t)C * C);
            for (int sj = 0; sj < S; sj++)
                for (int si = 0; si < S; si++) {
                    const P2 qs[4] = {lat[(size_t)sj * (S + 1) + si], lat[(size_t)sj * (S + 1) + si + 1],
                                      lat[(size_t)(sj + 1) * (S + 1) + si + 1], lat[(size_t)(sj + 1) * (S + 1) + si]};
                    uint16_t code = classify(si * C, sj * C, (si + 1) * C, (sj + 1) * C, qs, all, cand);
                    rcode[(size_t)sj * S + si] = code;
                    if (code != kMixed) continue;
                    LineRec lr;
                    if (lines && try_line(si, sj, 0.0, 0.0, 1.0, 1.0, 4, cand, lr, true)) {
                        r_kind[(size_t)ri].push_back(1);
                        r_line[(size_t)ri].push_back(lr);
                        continue;
                    }
                    for (int cj = 0; cj <= C; cj++)
                        for (int ci = 0; ci <= C; ci++)
                            clat[(size_t)cj * (C + 1) + ci] =
                                (ci % C == 0 && cj % C == 0) ? lat[(size_t)(sj + cj / C) * (S + 1) + si + ci / C]
                                                             : image(si * C + ci, sj * C + cj);
                    for (int cj = 0; cj < C; cj++)
                        for (int ci = 0; ci < C; ci++) {
                            int i0 = si * C + ci, j0 = sj * C + cj;
                            const P2 qc[4] = {clat[(size_t)cj * (C + 1) + ci], clat[(size_t)cj * (C + 1) + ci + 1],
                                              clat[(size_t)(cj + 1) * (C + 1) + ci + 1], clat[(size_t)(cj + 1) * (C + 1) + ci]};
                            uint16_t cc = classify(i0, j0, i0 + 1, j0 + 1, qc, cand, cand2);
                            if (cc == kMixed && leaf_lines &&
                                try_line(si, sj, (double)ci / C, (double)cj / C, (double)(ci + 1) / C, (double)(cj + 1) / C,
                                         kLeafLineMargins, cand2, lr, false)) {
                                r_cline_at[(size_t)ri].push_back((uint32_t)(r_cells[(size_t)ri].size() + (size_t)cj * C + ci));
                                r_cline[(size_t)ri].push_back(lr);
                            }
                            cellc[(size_t)cj * C + ci] = cc;
                        }
                    r_kind[(size_t)ri].push_back(0);
                    r_line[(size_t)ri].push_back(LineRec{0, 0, 0, 0, 0});
                    r_cells[(size_t)ri].insert(r_cells[(size_t)ri].end(), cellc.begin(), cellc.end());
                }
        }
    };
    int nt = std::max(1, threads);
    std::vector<std::thread> pool;
    for (int k = 1; k < nt; k++) pool.emplace_back(work);
    work();
    for (auto& th_ : pool) th_.join();
    rc.kind.clear();
    rc.line.clear();
    rc.cell_at.clear();
    rc.cells.clear();
    rc.cline_at.clear();
    rc.cline.clear();
    for (size_t r = 0; r < recs.size(); r++) {
        size_t c0 = 0;
        for (size_t k = 0; k < r_cline_at[r].size(); k++) {
            rc.cline_at.push_back((uint32_t)(rc.cells.size() + r_cline_at[r][k]));
            rc.cline.push_back(r_cline[r][k]);
        }
        for (size_t k = 0; k < r_kind[r].size(); k++) {
            rc.kind.push_back(r_kind[r][k]);
            rc.line.push_back(r_line[r][k]);
            if (r_kind[r][k]) {
                rc.cell_at.push_back(0);
            } else {
                rc.cell_at.push_back((uint32_t)(rc.cells.size() / ((size_t)C * C)));
                rc.cells.insert(rc.cells.end(), r_cells[r].begin() + (ptrdiff_t)c0, r_cells[r].begin() + (ptrdiff_t)(c0 + (size_t)C * C));
                c0 += (size_t)C * C;
            }
        }
    }
}

// Phase 2 (host, either classification): sub-block entries, per-tile line records and leaf blocks,
// the quad level with its compact copies.
namespace {
// fn(begin, end) over [0, n) in contiguous chunks on up to `threads` threads
template <class F>
void parallel_for(int64_t n, int threads, F fn) {
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(threads, n / 64));
    if (nt <= 1) {
        if (n > 0) fn((int64_t)0, n);
        return;
    }
    std::vector<std::thread> pool;
    for (int k = 0; k < nt; k++) pool.emplace_back([=, &fn]() { fn(n * k / nt, n * (k + 1) / nt); });
    for (auto& t : pool) t.join();
}
}  // namespace

// phase trace of the assembly (measurement only): MOSAIC_BUILD_TRACE=1
namespace {
struct AsmTrace {
    bool on = getenv("MOSAIC_BUILD_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(const char* what) {
        if (!on) return;
        fprintf(stderr, "[asm]   %-26s %8.3f ms\n", what,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count());
        t = std::chrono::steady_clock::now();
    }
};
}  // namespace

bool Builder::assemble_raster(const RasterClass& rc, int threads) {
    AsmTrace trace;
    const int nx = grid.nx, ny = grid.ny;
    const int64_t NX = (int64_t)nx * S, NY = (int64_t)ny * S;
    const size_t SS = (size_t)S * S, CC = (size_t)C * C;
    sub.clear();
    {
        // room for the quad level's compact copies too (appended below), so that growing the table
        // neither moves it nor faults its pages in on one thread
        int qs = 0;
        while (qs < 16 && ((NX + (1 << qs) - 1) >> qs) * ((NY + (1 << qs) - 1) >> qs) > quad_max) qs++;
        int64_t extra = 0;
        if (qs <= 6) {
            const int64_t nq = ((NX + (1 << qs) - 1) >> qs) * ((NY + (1 << qs) - 1) >> qs);
            extra = std::min<int64_t>(nq, kQuadRefMax + 1) << (2 * qs);
        }
        sub.reserve((size_t)(NX * NY + extra));
    }
    sub.resize((size_t)(NX * NY));  // (uninitialised: every tile's entries are written below)
    tile_base.assign((size_t)nx * ny, 0u);
    std::vector<std::vector<uint16_t>> tile_blocks(recs.size());
    std::vector<std::vector<LineRec>> tile_lines(recs.size());
    std::vector<std::vector<LineRec>> tile_llines(recs.size());
    // each record's first mixed sub-block (records are independent after that)
    const int64_t nrec = (int64_t)recs.size();
    std::vector<size_t> mk0((size_t)nrec + 1, 0);
    auto rec_ok = [&](int64_t ri) { return tile_of_rec[(size_t)ri] >= 0 && recs[(size_t)ri].dims != 0; };
    parallel_for(nrec, threads, [&](int64_t b, int64_t e) {
        for (int64_t ri = b; ri < e; ri++) {
            size_t m = 0;
            if (rec_ok(ri)) {
                const uint16_t* rcode = rc.code.data() + (size_t)ri * SS;
                for (size_t k = 0; k < SS; k++) m += rcode[k] == kMixed;
            }
            mk0[(size_t)ri + 1] = m;
        }
    });
    for (int64_t ri = 0; ri < nrec; ri++) mk0[(size_t)ri + 1] += mk0[(size_t)ri];
    if (mk0[(size_t)nrec] > rc.kind.size()) return false;
    trace.mark("alloc + mixed counts");
    std::atomic<int64_t> pure(0), mixed(0), cmixed(0), nline(0), ncline(0);
    parallel_for(nrec, threads, [&](int64_t b, int64_t e) {
        int64_t l_pure = 0, l_mixed = 0, l_cmixed = 0, l_line = 0, l_cline = 0;
        for (int64_t ri = b; ri < e; ri++) {
            if (!rec_ok(ri)) continue;
            const int t = tile_of_rec[(size_t)ri];
            const int ti = t % nx, tj = t / nx;
            const uint16_t* rcode = rc.code.data() + (size_t)ri * SS;
            std::vector<uint16_t>& outb = tile_blocks[(size_t)ri];
            std::vector<LineRec>& outl = tile_lines[(size_t)ri];
            std::vector<LineRec>& outll = tile_llines[(size_t)ri];
            size_t mk = mk0[(size_t)ri];  // next mixed sub-block
            // the tile's distinct line records (tile frame: every sub-block one edge splits with
            // the same margin and sides shares its record), first occurrence first
            std::unordered_map<std::string, uint32_t> lidx;
            for (int sj = 0; sj < S; sj++)
                for (int si = 0; si < S; si++) {
                    const uint16_t code = rcode[(size_t)sj * S + si];
                    uint16_t entry;
                    if (code != kMixed) {
                        entry = code;
                        l_pure++;
                    } else {
                        l_mixed++;
                        if (rc.kind[mk]) {
                            // tile-local line record number (< S * S <= kLineBit)
                            const auto ins = lidx.emplace(std::string((const char*)&rc.line[mk], sizeof(LineRec)),
                                                          (uint32_t)outl.size());
                            if (ins.second) outl.push_back(rc.line[mk]);
                            entry = (uint16_t)(kSubBlock | kLineBit | ins.first->second);
                            l_line++;
                        } else {
                            const uint16_t* cellc = rc.cells.data() + (size_t)rc.cell_at[mk] * CC;
                            bool same = true;
                            for (size_t q = 0; q < CC; q++) {
                                if (cellc[q] == kMixed) l_cmixed++;
                                same = same && cellc[q] == cellc[0];
                            }
                            if (same && cellc[0] != kMixed) {
                                entry = cellc[0];
                            } else {
                                // tile-local leaf block number (< S * S <= kLineBit)
                                entry = (uint16_t)(kSubBlock | (uint32_t)(outb.size() / CC));
                                const size_t b0 = outb.size();
                                outb.insert(outb.end(), cellc, cellc + CC);
                                // leaf lines: kSubBlock | kLineBit | n, n the tile's leaf line
                                // (while n fits 14 bits; the others stay kMixed)
                                const uint32_t g0 = rc.cell_at[mk] * (uint32_t)CC;
                                for (auto it = std::lower_bound(rc.cline_at.begin(), rc.cline_at.end(), g0);
                                     it != rc.cline_at.end() && *it < g0 + (uint32_t)CC && outll.size() < kLineBit; ++it) {
                                    outb[b0 + (*it - g0)] = (uint16_t)(kSubBlock | kLineBit | (uint32_t)outll.size());
                                    outll.push_back(rc.cline[(size_t)(it - rc.cline_at.begin())]);
                                    l_cline++;
                                    l_cmixed--;
                                }
                            }
                        }
                        mk++;
                    }
                    sub[(size_t)((int64_t)(tj * S + sj) * NX + (ti * S + si))] = entry;
                }
        }
        pure += l_pure;
        mixed += l_mixed;
        cmixed += l_cmixed;
        nline += l_line;
        ncline += l_cline;
    });
    trace.mark("sub entries");
    // tiles without a record: kFull (every point takes the tile path) or kSkip (no pair: 0)
    std::vector<uint8_t> has_rec((size_t)nx * ny, 0);
    for (int64_t ri = 0; ri < nrec; ri++)
        if (rec_ok(ri)) has_rec[(size_t)tile_of_rec[(size_t)ri]] = 1;
    parallel_for((int64_t)nx * ny, threads, [&](int64_t b, int64_t e) {
        for (int64_t t = b; t < e; t++) {
            if (has_rec[(size_t)t]) continue;
            const uint16_t v = tile_idx[(size_t)t] == kFull ? kMixed : (uint16_t)0;
            int ti = (int)(t % nx), tj = (int)(t / nx);
            for (int sj = 0; sj < S; sj++)
                std::fill_n(sub.data() + (size_t)((int64_t)(tj * S + sj) * NX + ti * S), S, v);
        }
    });
    // merge: per tile [line records, last first][leaf blocks], 16-byte aligned; tile_base = the
    // element of the tile's first leaf block
    size_t total = 0;
    std::vector<size_t> at(recs.size());
    for (size_t r = 0; r < recs.size(); r++) {
        at[r] = total + 8 * tile_lines[r].size();
        if (tile_of_rec[r] >= 0) tile_base[(size_t)tile_of_rec[r]] = (uint32_t)at[r];
        total = (at[r] + tile_blocks[r].size() + 7) & ~(size_t)7;
    }
    if (total >= ((size_t)1 << 32)) {
        sub.clear();
        return false;
    }
    const size_t nblocks = std::max<size_t>(total, std::max<size_t>(CC, 8));
    blocks.clear();
    blocks.resize(nblocks);  // (uninitialised: each record's span and the padding are written below)
    parallel_for(nrec, threads, [&](int64_t b, int64_t e) {
        for (int64_t r = b; r < e; r++) {
            // [span start, line records, leaf blocks, padding to the next record's span)
            const size_t lo = at[(size_t)r] - 8 * tile_lines[(size_t)r].size();
            const size_t hi = (size_t)r + 1 < recs.size() ? at[(size_t)r + 1] - 8 * tile_lines[(size_t)r + 1].size() : nblocks;
            for (size_t n = 0; n < tile_lines[(size_t)r].size(); n++)
                memcpy(blocks.data() + at[(size_t)r] - 8 * (n + 1), &tile_lines[(size_t)r][n], sizeof(LineRec));
            std::copy(tile_blocks[(size_t)r].begin(), tile_blocks[(size_t)r].end(), blocks.begin() + (ptrdiff_t)at[(size_t)r]);
            std::fill(blocks.begin() + (ptrdiff_t)(at[(size_t)r] + tile_blocks[(size_t)r].size()), blocks.begin() + (ptrdiff_t)hi,
                      kMixed);
            if (r == 0) std::fill(blocks.begin(), blocks.begin() + (ptrdiff_t)lo, kMixed);
        }
    });
    if (nrec == 0) std::fill(blocks.begin(), blocks.end(), kMixed);
    // leaf lines, per tile in record order
    tile_lbase.assign((size_t)nx * ny, 0u);
    llines.clear();
    for (size_t r = 0; r < recs.size(); r++) {
        if (tile_of_rec[r] >= 0) tile_lbase[(size_t)tile_of_rec[r]] = (uint32_t)llines.size();
        llines.insert(llines.end(), tile_llines[r].begin(), tile_llines[r].end());
    }
    trace.mark("full tiles + merge blocks");
    // clamping (raster_code, k_join_stream): a finite point outside the grid is looked up at the
    // nearest edge sub-block, so every edge sub-block must answer "no pair" (0) or kMixed (the
    // tile path, which finds no chip outside the grid); chip cells lie >= k tile rings inside
    edge_ok = true;
    for (int64_t i = 0; i < NX && edge_ok; i++)
        for (int64_t j : {(int64_t)0, NY - 1}) {
            const uint16_t e = sub[(size_t)(j * NX + i)];
            if (e != 0 && e != kMixed) edge_ok = false;
        }
    for (int64_t j = 0; j < NY && edge_ok; j++)
        for (int64_t i : {(int64_t)0, NX - 1}) {
            const uint16_t e = sub[(size_t)(j * NX + i)];
            if (e != 0 && e != kMixed) edge_ok = false;
        }
    n_sub_line = nline.load();
    n_sub_pure = pure.load();
    n_sub_mixed = mixed.load();
    n_cell_mixed = cmixed.load();
    n_cell_line = ncline.load();
    // quad level: the smallest power-of-two group of sub-blocks whose table fits quad_max entries
    qshift = 0;
    while (qshift < 16 && ((NX + (1 << qshift) - 1) >> qshift) * ((NY + (1 << qshift) - 1) >> qshift) > quad_max)
        qshift++;
    if (qshift < 16) {
        qnx = (int)((NX + (1 << qshift) - 1) >> qshift);
        qny = (int)((NY + (1 << qshift) - 1) >> qshift);
        quad.assign((size_t)qnx * qny, kMixed);
        // per quad: the code all its (in-grid) sub-blocks share, else kMixed (blocks and kMixed alike)
        parallel_for((int64_t)qnx * qny, threads, [&](int64_t qb, int64_t qe) {
            for (int64_t q = qb; q < qe; q++) {
                const int64_t i0 = (q % qnx) << qshift, j0 = (q / qnx) << qshift;
                const int64_t i1 = std::min<int64_t>(NX, i0 + ((int64_t)1 << qshift));
                const int64_t j1 = std::min<int64_t>(NY, j0 + ((int64_t)1 << qshift));
                const uint16_t first = sub[(size_t)(j0 * NX + i0)];
                uint16_t code = (first & kSubBlock) ? kMixed : first;
                for (int64_t j = j0; j < j1 && code != kMixed; j++) {
                    const uint16_t* row = sub.data() + (size_t)(j * NX);
                    for (int64_t i = i0; i < i1; i++)
                        if (row[i] != code) {
                            code = kMixed;
                            break;
                        }
                }
                quad[(size_t)q] = code;
            }
        });
        trace.mark("edge check + quad level");
        // compact copies of the non-uniform quads' sub-block entries behind the grid's own
        // (quad entry kSubBlock | r: quad r's 2^qshift x 2^qshift entries, row-major, from
        // sub[nx * ny + (r << 2 qshift)]), so the sub-block lookups that pass the quad level
        // gather from a table the size of the mixed quads rather than of the grid
        const int64_t QS = (int64_t)1 << qshift, QQ = QS * QS;
        int64_t nref = 0;
        for (uint16_t e : quad) nref += e == kMixed;
        if (qshift <= 6 && nref <= kQuadRefMax + 1 && NX * NY + nref * QQ < ((int64_t)1 << 31)) {
            const size_t base = sub.size();
            sub.resize(base + (size_t)(nref * QQ));  // (uninitialised: every entry is written below)
            std::vector<int64_t> refq;  // compact quad r -> quad (row-major order)
            refq.reserve((size_t)nref);
            for (int64_t q = 0; q < (int64_t)quad.size(); q++)
                if (quad[(size_t)q] == kMixed) refq.push_back(q);
            parallel_for(nref, threads, [&](int64_t b, int64_t e) {
                for (int64_t r = b; r < e; r++) {
                    const int64_t qj = refq[(size_t)r] / qnx, qi = refq[(size_t)r] % qnx;
                    uint16_t* dst = sub.data() + base + (size_t)(r * QQ);
                    for (int64_t dj = 0; dj < QS; dj++)
                        for (int64_t di = 0; di < QS; di++) {
                            const int64_t j = qj * QS + dj, i = qi * QS + di;
                            dst[dj * QS + di] = j < NY && i < NX ? sub[(size_t)(j * NX + i)] : (uint16_t)0;
                        }
                    quad[(size_t)refq[(size_t)r]] = (uint16_t)(kSubBlock | r);
                }
            });
            trace.mark("compact copies");
            // quad records for as many compact quads as the LDS budget holds (10 bytes each)
            qrec_mask.clear();
            qrec_code.clear();
            qrec_shift = 0;
            const int64_t qbytes = ((int64_t)quad.size() + 1) / 2 * 4;
            const int64_t nrec = qshift >= 3 && (int64_t)quad_lds_bytes > qbytes + 16
                                     ? std::min<int64_t>(nref, ((int64_t)quad_lds_bytes - qbytes - 16) / 10)
                                     : 0;
            if (nrec > 0) {
                qrec_shift = qshift - 3;
                const int64_t G = (int64_t)1 << qrec_shift;
                qrec_mask.assign((size_t)(2 * nrec), 0u);
                qrec_code.assign((size_t)nrec, 0);
                parallel_for(nrec, threads, [&](int64_t rb, int64_t re) {
                for (int64_t rr = rb; rr < re; rr++) {
                    // the compact copy (out-of-grid entries are 0 there; points never reach them, and a
                    // sub-quad counts as uniform only if they agree too)
                    const uint16_t* src = sub.data() + base + (size_t)(rr * QQ);
                    uint16_t code[64];
                    bool uni[64];
                    for (int b = 0; b < 64; b++) {
                        const int64_t i0 = (b & 7) * G, j0 = (b >> 3) * G;
                        const uint16_t c = src[j0 * QS + i0];
                        bool u = !(c & kSubBlock);
                        for (int64_t dj = 0; dj < G && u; dj++)
                            for (int64_t di = 0; di < G; di++)
                                if (src[(j0 + dj) * QS + i0 + di] != c) {
                                    u = false;
                                    break;
                                }
                        code[b] = c;
                        uni[b] = u;
                    }
                    // the most common uniform code (ties: the smallest)
                    int best_n = 0;
                    uint16_t best = 0;
                    for (int b = 0; b < 64; b++) {
                        if (!uni[b]) continue;
                        int cnt = 0;
                        for (int b2 = 0; b2 < 64; b2++) cnt += uni[b2] && code[b2] == code[b];
                        if (cnt > best_n || (cnt == best_n && code[b] < best)) {
                            best_n = cnt;
                            best = code[b];
                        }
                    }
                    qrec_code[(size_t)rr] = best;
                    for (int b = 0; b < 64; b++)
                        if (uni[b] && code[b] == best) qrec_mask[(size_t)(2 * rr + (b >> 5))] |= 1u << (b & 31);
                }
                });
            }
            trace.mark("quad records");
        } else {
            quad.clear();  // no quad level: k_join_stream needs one (the tile path serves)
        }
    }
    return true;
}

bool bng_leaf_blocks(const Builder::ChipSource& src, const std::vector<BngBorderCell>& cells, double side, int C,
                     bool lines, int threads, std::vector<uint16_t>& blocks, std::vector<uint32_t>& base,
                     std::vector<uint16_t>* glines, bool wedges) {
    if (C < 1 || C > 64) return false;
    const int CB = bng_level_side(C), G = kBngLvlG;
    if (glines) glines->assign(cells.size() * (size_t)CB * CB, kSubBlock);
    const size_t CC = (size_t)C * C, CCp = (CC + 7) & ~(size_t)7;  // leaf block padded to 16 bytes
    std::vector<std::vector<uint16_t>> ent(cells.size());
    std::vector<std::vector<LineRec>> lrec(cells.size());
    std::atomic<int64_t> next(0);
    auto work = [&]() {
        std::vector<Seg> segs;
        std::vector<std::vector<Seg>> csegs;
        std::vector<int32_t> ans;
        std::vector<P2> ends;
        while (true) {
            const int64_t k = next.fetch_add(1);
            if (k >= (int64_t)cells.size()) break;
            const BngBorderCell& bc = cells[(size_t)k];
            const uint32_t f0 = src.slot_first[bc.slot], n0 = src.slot_count[bc.slot];
            std::vector<int32_t> core;
            std::vector<uint32_t> border;
            csegs.clear();
            for (uint32_t c = f0; c < f0 + n0; c++) {
                if (src.meta[c] & 1u) {
                    core.push_back((int32_t)(src.meta[c] >> 1));
                } else {
                    border.push_back(c);
                    chip_segments(src.store, c, segs);
                    csegs.push_back(segs);
                }
            }
            const double h = side / C;
            // the sub-rectangles are widened past the kernel's index rounding
            const double ex = 1e-6 * h + 1e-9 * (fabs(bc.x0) + side);
            const double ey = 1e-6 * h + 1e-9 * (fabs(bc.y0) + side);
            // answer of the convex polygon q[n] (metres): kMixed when a border chip's segment comes
            // within ex of it, else the keys containing its vertex mean (contains() is constant on it)
            auto classify_poly = [&](const P2* q, int n) -> uint16_t {
                double mx = 0, my = 0, x0 = INFINITY, y0 = INFINITY, x1 = -INFINITY, y1 = -INFINITY;
                for (int v = 0; v < n; v++) {
                    mx += q[v].x;
                    my += q[v].y;
                    x0 = rbuild::dmin(x0, q[v].x);
                    y0 = rbuild::dmin(y0, q[v].y);
                    x1 = rbuild::dmax(x1, q[v].x);
                    y1 = rbuild::dmax(y1, q[v].y);
                }
                mx /= n;
                my /= n;
                ans = core;
                for (size_t b = 0; b < border.size(); b++) {
                    const pip::Box& bx = src.store.geom_bbox[border[b]];
                    if (!(bx.maxx < x0 - ex || bx.minx > x1 + ex || bx.maxy < y0 - ey || bx.miny > y1 + ey))
                        for (const Seg& e : csegs[b])
                            if (seg_meets_poly(P2{e.ax, e.ay}, P2{e.bx, e.by}, q, n, ex)) return kMixed;
                    if (pip::contains(src.store, border[b], mx, my)) ans.push_back((int32_t)(src.meta[border[b]] >> 1));
                }
                return ans.empty() ? (uint16_t)0 : (ans.size() == 1 ? (uint16_t)(ans[0] + 1) : kMixed);
            };
            // a mixed sub-cell whose chip edges all lie along one line (tiles_build try_line, in
            // sub-cell units): the line through the chip segment holding the longest clipped piece,
            // in the CELL frame (offsets from the cell's corner, 0 <= u, v <= C: the sub-cells one
            // edge splits share the record; rbuild::line_slack_tile), both sides certified
            auto try_line = [&](int i, int j, LineRec& out) -> bool {
                const double rx0 = bc.x0 + h * i, ry0 = bc.y0 + h * j;
                const double exu = ex / h, eyv = ey / h;
                const double bx0 = rx0 - ex, bx1 = rx0 + h + ex, by0 = ry0 - ey, by1 = ry0 + h + ey;
                double best = 0.0;
                P2 ta{0, 0}, tb{0, 0};
                ends.clear();
                for (size_t b = 0; b < border.size(); b++) {
                    const pip::Box& bx = src.store.geom_bbox[border[b]];
                    if (bx.maxx < bx0 || bx.minx > bx1 || bx.maxy < by0 || bx.miny > by1) continue;
                    for (const Seg& e : csegs[b]) {
                        double ax = (e.ax - rx0) / h, ay = (e.ay - ry0) / h;
                        double qx = (e.bx - rx0) / h, qy = (e.by - ry0) / h;
                        if (!clip_seg(ax, ay, qx, qy, -exu, -eyv, 1.0 + exu, 1.0 + eyv)) continue;
                        ends.push_back(P2{ax, ay});
                        ends.push_back(P2{qx, qy});
                        const double l2 = (qx - ax) * (qx - ax) + (qy - ay) * (qy - ay);
                        if (l2 > best) {
                            best = l2;
                            ta = P2{(e.ax - bc.x0) / h, (e.ay - bc.y0) / h};
                            tb = P2{(e.bx - bc.x0) / h, (e.by - bc.y0) / h};
                        }
                    }
                }
                if (!(best > 1e-6)) return false;
                const double lt = sqrt((tb.x - ta.x) * (tb.x - ta.x) + (tb.y - ta.y) * (tb.y - ta.y));
                const double a = -(tb.y - ta.y) / lt, b = (tb.x - ta.x) / lt;
                const double c = -(a * 0.5 * (ta.x + tb.x) + b * 0.5 * (ta.y + tb.y));
                double dev_max = 0.0;
                for (const P2& p : ends) dev_max = std::max(dev_max, fabs(a * (p.x + i) + b * (p.y + j) + c));
                const P2 sq[4] = {{-exu, -eyv}, {1.0 + exu, -eyv}, {1.0 + exu, 1.0 + eyv}, {-exu, 1.0 + eyv}};
                for (int mk = 0; mk < 4; mk++) {
                    const double margin = rbuild::line_margin(mk);
                    if (dev_max > margin - 2.0 * kLineSlack) continue;
                    out.a = (float)(a / margin);
                    out.b = (float)(b / margin);
                    out.c = (float)(c / margin);
                    // certify with the coefficients the device uses (as try_line): the sub-cell's
                    // own C = Ct + A i + B j
                    const double A = out.a, B = out.b, Cf = (double)out.c + A * i + B * j;
                    const double m = 1.0 - rbuild::line_slack_tile(A, B, out.c, C, kLineSlack);
                    P2 hp[8], hn[8];
                    const int np = clip_half(sq, 4, A, B, Cf - m, hp), nn = clip_half(sq, 4, -A, -B, -Cf - m, hn);
                    for (int v = 0; v < np; v++) hp[v] = P2{rx0 + h * hp[v].x, ry0 + h * hp[v].y};
                    for (int v = 0; v < nn; v++) hn[v] = P2{rx0 + h * hn[v].x, ry0 + h * hn[v].y};
                    const uint16_t cp = np >= 3 ? classify_poly(hp, np) : 0;
                    if (cp == kMixed) continue;
                    const uint16_t cn = nn >= 3 ? classify_poly(hn, nn) : 0;
                    if (cn == kMixed) continue;
                    out.pos = cp;
                    out.neg = cn;
                    return true;
                }
                return false;
            };
            // a mixed sub-cell split by two segments sharing a vertex (tiles.h bng_leaf_blocks wedges):
            // the two longest clipped pieces' segments, their lines oriented so that the convex
            // wedge is s >= 0 on both, both regions certified
            auto try_wedge = [&](int i, int j, LineRec& o1, LineRec& o2) -> bool {
                const double rx0 = bc.x0 + h * i, ry0 = bc.y0 + h * j;
                const double exu = ex / h, eyv = ey / h;
                const double bx0 = rx0 - ex, bx1 = rx0 + h + ex, by0 = ry0 - ey, by1 = ry0 + h + ey;
                // the longest clipped piece's segment, then the longest piece of a different segment
                // (adjacent zones' chips carry the same boundary segment: equal ends either way round)
                double l1 = 0.0, l2 = 0.0;
                const Seg* s1 = nullptr;
                const Seg* s2 = nullptr;
                auto same = [](const Seg* p, const Seg& q) {
                    return (p->ax == q.ax && p->ay == q.ay && p->bx == q.bx && p->by == q.by) ||
                           (p->ax == q.bx && p->ay == q.by && p->bx == q.ax && p->by == q.ay);
                };
                for (int pass = 0; pass < 2; pass++) {
                    if (pass == 1 && !s1) return false;
                    for (size_t b = 0; b < border.size(); b++) {
                        const pip::Box& bx = src.store.geom_bbox[border[b]];
                        if (bx.maxx < bx0 || bx.minx > bx1 || bx.maxy < by0 || bx.miny > by1) continue;
                        for (const Seg& e : csegs[b]) {
                            if (pass == 1 && same(s1, e)) continue;
                            double ax = (e.ax - rx0) / h, ay = (e.ay - ry0) / h;
                            double qx = (e.bx - rx0) / h, qy = (e.by - ry0) / h;
                            if (!clip_seg(ax, ay, qx, qy, -exu, -eyv, 1.0 + exu, 1.0 + eyv)) continue;
                            const double l = (qx - ax) * (qx - ax) + (qy - ay) * (qy - ay);
                            if (pass == 0 && l > l1) {
                                l1 = l;
                                s1 = &e;
                            } else if (pass == 1 && l > l2) {
                                l2 = l;
                                s2 = &e;
                            }
                        }
                    }
                }
                if (!s1 || !s2 || !(l2 > 1e-6)) return false;
                P2 V, A1, A2;  // the shared vertex and the segments' other ends (metres)
                if (s1->bx == s2->ax && s1->by == s2->ay) {
                    V = P2{s1->bx, s1->by}; A1 = P2{s1->ax, s1->ay}; A2 = P2{s2->bx, s2->by};
                } else if (s1->ax == s2->bx && s1->ay == s2->by) {
                    V = P2{s1->ax, s1->ay}; A1 = P2{s1->bx, s1->by}; A2 = P2{s2->ax, s2->ay};
                } else if (s1->ax == s2->ax && s1->ay == s2->ay) {
                    V = P2{s1->ax, s1->ay}; A1 = P2{s1->bx, s1->by}; A2 = P2{s2->bx, s2->by};
                } else if (s1->bx == s2->bx && s1->by == s2->by) {
                    V = P2{s1->bx, s1->by}; A1 = P2{s1->ax, s1->ay}; A2 = P2{s2->ax, s2->ay};
                } else {
                    return false;
                }
                auto cf = [&](P2 p) { return P2{(p.x - bc.x0) / h, (p.y - bc.y0) / h}; };  // cell frame
                V = cf(V);
                A1 = cf(A1);
                A2 = cf(A2);
                auto line_of = [&](P2 A, P2 O, double* a, double* b, double* c) -> bool {  // through V, A; O on the + side
                    const double L = sqrt((A.x - V.x) * (A.x - V.x) + (A.y - V.y) * (A.y - V.y));
                    if (!(L > 0.0)) return false;
                    *a = -(A.y - V.y) / L;
                    *b = (A.x - V.x) / L;
                    *c = -(*a * V.x + *b * V.y);
                    const double so = *a * O.x + *b * O.y + *c;
                    if (so < 0) {
                        *a = -*a;
                        *b = -*b;
                        *c = -*c;
                    }
                    return fabs(so) > 1e-9;  // (collinear: a line record's case)
                };
                double a1, b1, c1, a2, b2, c2;
                if (!line_of(A1, A2, &a1, &b1, &c1) || !line_of(A2, A1, &a2, &b2, &c2)) return false;
                const P2 sq[4] = {{-exu, -eyv}, {1.0 + exu, -eyv}, {1.0 + exu, 1.0 + eyv}, {-exu, 1.0 + eyv}};
                for (int mk = 0; mk < 4; mk++) {
                    const double margin = rbuild::line_margin(mk);
                    o1 = LineRec{(float)(a1 / margin), (float)(b1 / margin), (float)(c1 / margin), 0, 0};
                    o2 = LineRec{(float)(a2 / margin), (float)(b2 / margin), (float)(c2 / margin), 0, 0};
                    const double A1c = o1.a, B1c = o1.b, C1 = (double)o1.c + A1c * i + B1c * j;
                    const double A2c = o2.a, B2c = o2.b, C2 = (double)o2.c + A2c * i + B2c * j;
                    const double m1 = 1.0 - rbuild::line_slack_tile(A1c, B1c, o1.c, C, kLineSlack);
                    const double m2 = 1.0 - rbuild::line_slack_tile(A2c, B2c, o2.c, C, kLineSlack);
                    P2 t[8], w[8], r1[8], r2[8];
                    const int nt = clip_half(sq, 4, A1c, B1c, C1 - m1, t);
                    const int nw = nt >= 3 ? clip_half(t, nt, A2c, B2c, C2 - m2, w) : 0;
                    const int n1 = clip_half(sq, 4, -A1c, -B1c, -C1 - m1, r1), n2 = clip_half(sq, 4, -A2c, -B2c, -C2 - m2, r2);
                    auto metres = [&](P2* q, int n) {
                        for (int v = 0; v < n; v++) q[v] = P2{rx0 + h * q[v].x, ry0 + h * q[v].y};
                    };
                    metres(w, nw);
                    metres(r1, n1);
                    metres(r2, n2);
                    const uint16_t cw = nw >= 3 ? classify_poly(w, nw) : 0;
                    if (cw == kMixed) continue;
                    const uint16_t cr1 = n1 >= 3 ? classify_poly(r1, n1) : kSubBlock;
                    if (cr1 == kMixed) continue;
                    const uint16_t cr2 = n2 >= 3 ? classify_poly(r2, n2) : kSubBlock;
                    if (cr2 == kMixed) continue;
                    if (cr1 != kSubBlock && cr2 != kSubBlock && cr1 != cr2) return false;
                    const uint16_t cr = cr1 != kSubBlock ? cr1 : (cr2 != kSubBlock ? cr2 : (uint16_t)0);
                    o1.pos = o2.pos = cw;
                    o1.neg = o2.neg = cr;
                    return true;
                }
                return false;
            };
            std::vector<uint16_t>& e = ent[(size_t)k];
            e.assign(CCp, 0);
            for (int j = 0; j < C; j++)
                for (int i = 0; i < C; i++) {
                    Rect r{bc.x0 + h * i - ex, bc.y0 + h * j - ey, bc.x0 + h * (i + 1) + ex, bc.y0 + h * (j + 1) + ey};
                    const double cxm = bc.x0 + h * (i + 0.5), cym = bc.y0 + h * (j + 0.5);
                    ans = core;
                    bool mixed = false;
                    for (size_t b = 0; b < border.size() && !mixed; b++) {
                        const pip::Box& bx = src.store.geom_bbox[border[b]];
                        if (!(bx.maxx < r.x0 || bx.minx > r.x1 || bx.maxy < r.y0 || bx.miny > r.y1) &&
                            any_seg_meets(csegs[b], r)) {
                            mixed = true;
                            break;
                        }
                        if (pip::contains(src.store, border[b], cxm, cym)) ans.push_back((int32_t)(src.meta[border[b]] >> 1));
                    }
                    uint16_t code = kMixed;
                    if (!mixed) code = ans.empty() ? (uint16_t)0 : (ans.size() == 1 ? (uint16_t)(ans[0] + 1) : kMixed);
                    LineRec lr;
                    if (code == kMixed && lines && try_line(i, j, lr)) {
                        // the cell's distinct records, first occurrence first
                        size_t n = 0;
                        while (n < lrec[(size_t)k].size() && memcmp(&lrec[(size_t)k][n], &lr, sizeof(LineRec))) n++;
                        code = (uint16_t)(kSubBlock | kLineBit | n);
                        if (n == lrec[(size_t)k].size()) lrec[(size_t)k].push_back(lr);
                    } else if (code == kMixed && lines && wedges && lrec[(size_t)k].size() + 2 <= 0x3fffu) {
                        LineRec w2;
                        if (try_wedge(i, j, lr, w2)) {
                            code = (uint16_t)(kSubBlock | lrec[(size_t)k].size());
                            lrec[(size_t)k].push_back(lr);
                            lrec[(size_t)k].push_back(w2);
                        }
                    }
                    e[(size_t)j * C + i] = code;
                }
            // group-level line codes (glines): a group whose line sub-cells all name record n and
            // whose other sub-cells are pure, with n certified over the whole widened group
            if (glines && lines && !lrec[(size_t)k].empty())
                for (int bj = 0; bj < CB; bj++)
                    for (int bi = 0; bi < CB; bi++) {
                        uint32_t n = ~0u;
                        bool ok = true;
                        for (int j = G * bj; ok && j < std::min(C, G * bj + G); j++)
                            for (int i = G * bi; ok && i < std::min(C, G * bi + G); i++) {
                                const uint16_t v = e[(size_t)j * C + i];
                                if (v == kMixed) ok = false;
                                else if ((v & 0xC000u) == 0xC000u) {
                                    if (n == ~0u) n = v & 0x3fffu;
                                    else if (n != (uint32_t)(v & 0x3fffu)) ok = false;
                                }
                            }
                        if (!ok || n == ~0u) continue;
                        const LineRec& lr = lrec[(size_t)k][n];
                        const double exu = ex / h, eyv = ey / h;
                        const double u0 = G * bi, v0 = G * bj, u1 = std::min(C, G * bi + G), v1 = std::min(C, G * bj + G);
                        const P2 sq[4] = {{u0 - exu, v0 - eyv}, {u1 + exu, v0 - eyv}, {u1 + exu, v1 + eyv}, {u0 - exu, v1 + eyv}};
                        const double A = lr.a, B = lr.b, Ct = lr.c;
                        const double m = 1.0 - rbuild::line_slack_tile(A, B, Ct, C, kLineSlack);
                        P2 hp[8], hn[8];
                        const int np = clip_half(sq, 4, A, B, Ct - m, hp), nn = clip_half(sq, 4, -A, -B, -Ct - m, hn);
                        for (int v = 0; v < np; v++) hp[v] = P2{bc.x0 + h * hp[v].x, bc.y0 + h * hp[v].y};
                        for (int v = 0; v < nn; v++) hn[v] = P2{bc.x0 + h * hn[v].x, bc.y0 + h * hn[v].y};
                        if (np >= 3 && classify_poly(hp, np) != lr.pos) continue;
                        if (nn >= 3 && classify_poly(hn, nn) != lr.neg) continue;
                        (*glines)[(size_t)k * CB * CB + (size_t)bj * CB + bi] = (uint16_t)(kSubBlock | kLineBit | n);
                    }
        }
    };
    const int nt = std::max(1, threads);
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; t++) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
    // layout per border cell: its line records (8 elements each, record n at base - 8 (n + 1)),
    // then its leaf block at base
    size_t total = 0;
    for (size_t k = 0; k < cells.size(); k++) total += lrec[k].size() * 8 + CCp;
    if (total >= ((size_t)1 << 30)) return false;  // element offsets share a word with the table's flags
    blocks.assign(total, kMixed);
    base.assign(cells.size(), 0);
    size_t at = 0;
    for (size_t k = 0; k < cells.size(); k++) {
        const size_t nl = lrec[k].size();
        for (size_t n = 0; n < nl; n++) memcpy(&blocks[at + 8 * (nl - 1 - n)], &lrec[k][n], sizeof(LineRec));
        at += 8 * nl;
        base[k] = (uint32_t)at;
        memcpy(&blocks[at], ent[k].data(), CCp * 2);
        at += CCp;
    }
    return true;
}

}  // namespace tiles
}  // namespace mosaic
