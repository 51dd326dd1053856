// Measurement tool (not product code): builds the H3 tile directory + point raster of
// mosaic_amd/csrc/tiles_build.cpp on the host for a chip set and reports, for uniform points over a
// box, which level of the raster decides them -- and what finer LDS quad levels would decide.
// Input: the chips.bin format of tests/native/tiles_selfcheck.cpp.
// Usage: raster_stats <chips.bin> <points> <x0> <y0> <x1> <y1> [S C threads]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <random>
#include <set>
#include <unordered_map>
#include <vector>

#include "../mosaic_amd/csrc/geom_build.h"
#include "../mosaic_amd/csrc/tiles_build.cpp"

using namespace mosaic;

int main(int argc, char** argv) {
    if (argc < 7) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    int32_t res = 0;
    uint32_t nchips = 0;
    if (fread(&res, 4, 1, f) != 1 || fread(&nchips, 4, 1, f) != 1) return 2;
    struct Row {
        int64_t cell;
        uint8_t core;
        int32_t key;
        std::vector<uint8_t> wkb;
    };
    std::vector<Row> rows(nchips);
    int32_t npoly = 0;
    for (auto& r : rows) {
        uint32_t len = 0;
        if (fread(&r.cell, 8, 1, f) != 1 || fread(&r.core, 1, 1, f) != 1 || fread(&r.key, 4, 1, f) != 1 ||
            fread(&len, 4, 1, f) != 1)
            return 2;
        r.wkb.resize(len);
        if (len && fread(r.wkb.data(), 1, len, f) != len) return 2;
        npoly = std::max(npoly, r.key + 1);
    }
    fclose(f);
    std::stable_sort(rows.begin(), rows.end(), [](const Row& a, const Row& b) { return a.cell < b.cell; });
    GeomBuilder gb;
    std::vector<uint32_t> meta(nchips);
    for (uint32_t k = 0; k < nchips; k++) {
        meta[k] = ((uint32_t)rows[k].key << 1) | (rows[k].core ? 1u : 0u);
        if (!gb.add(rows[k].core ? nullptr : rows[k].wkb.data(), rows[k].core ? 0 : rows[k].wkb.size())) return 3;
    }
    std::vector<int64_t> cells;
    std::vector<uint32_t> first, count;
    for (uint32_t k = 0; k < nchips; k++) {
        if (cells.empty() || cells.back() != rows[k].cell) {
            cells.push_back(rows[k].cell);
            first.push_back(k);
            count.push_back(0);
        }
        count.back()++;
    }
    const uint32_t n = (uint32_t)cells.size();
    std::unordered_map<int64_t, int64_t> slot;
    std::vector<uint32_t> slot_first(n), slot_count(n);
    for (uint32_t k = 0; k < n; k++) {
        slot.emplace(cells[k], (int64_t)k);
        slot_first[k] = first[k];
        slot_count[k] = count[k];
    }
    auto slot_of = [&](int64_t h) -> int64_t {
        auto it = slot.find(h);
        return it == slot.end() ? -1 : it->second;
    };
    const long npts = atol(argv[2]);
    const double bx0 = atof(argv[3]), by0 = atof(argv[4]), bx1 = atof(argv[5]), by1 = atof(argv[6]);
    const int S = argc > 8 ? atoi(argv[7]) : 64, C = argc > 8 ? atoi(argv[8]) : 16;
    const int threads = argc > 9 ? atoi(argv[9]) : 8;
    auto t0 = std::chrono::steady_clock::now();
    tiles::Builder tb;
    tb.leaf_lines = getenv("NO_LEAF_LINES") == nullptr;
    if (!tb.build(res, cells, slot_of)) {
        fprintf(stderr, "directory not built: %s\n", tb.why);
        return 1;
    }
    if (getenv("DEVICE_QUAD")) {
        // the quad-level budget of a chip table built for the stream kernels (mosaic_hip.hip): the
        // LDS of one 1024-thread workgroup beside its counts, stages and (when small) tile_base
        size_t avail = 160 * 1024 - 16 * 128 * 4 - 1024 - ((size_t)npoly + 64) * 4;
        const size_t tbytes = tb.tile_idx.size() * 4;
        if (tbytes <= avail / 3 && !getenv("NO_TB_LDS")) avail -= tbytes;
        tb.quad_max = (int)std::min<size_t>(tiles::kQuadLimit, avail / 4);
        tb.quad_lds_bytes = avail;
    }
    auto t1 = std::chrono::steady_clock::now();
    tiles::Builder::ChipSource src;
    src.slot_first = slot_first.data();
    src.slot_count = slot_count.data();
    src.meta = meta.data();
    src.store = pip::GeomStore{gb.verts.data(), gb.ring_start.data(), gb.ring_bbox.data(), gb.part_ring.data(),
                               gb.geom_part.data(), gb.geom_bbox.data()};
    src.n_polygons = npoly;
    if (!tb.build_raster(src, S, C, threads)) {
        fprintf(stderr, "raster not built\n");
        return 1;
    }
    auto t2 = std::chrono::steady_clock::now();
    printf("directory %.3f s, raster %.3f s (%d threads)\n", std::chrono::duration<double>(t1 - t0).count(),
           std::chrono::duration<double>(t2 - t1).count(), threads);
    {
        auto fnv = [](const void* p, size_t n) {
            uint64_t h = 1469598103934665603ull;
            for (size_t i = 0; i < n; i++) h = (h ^ ((const uint8_t*)p)[i]) * 1099511628211ull;
            return (unsigned long long)h;
        };
        printf("hash sub %016llx blocks %016llx tile_base %016llx quad %016llx\n", fnv(tb.sub.data(), tb.sub.size() * 2),
               fnv(tb.blocks.data(), tb.blocks.size() * 2), fnv(tb.tile_base.data(), tb.tile_base.size() * 4),
               fnv(tb.quad.data(), tb.quad.size() * 2));
    }
    const int64_t NX = (int64_t)tb.grid.nx * S, NY = (int64_t)tb.grid.ny * S;
    printf("grid %d x %d tiles, %lld x %lld sub-blocks, records %zu; sub pure %lld mixed %lld line %lld; "
           "blocks %zu elements; quad %d x %d shift %d\n",
           tb.grid.nx, tb.grid.ny, (long long)NX, (long long)NY, tb.recs.size(), (long long)tb.n_sub_pure,
           (long long)tb.n_sub_mixed, (long long)tb.n_sub_line, tb.blocks.size(), tb.qnx, tb.qny, tb.qshift);
    printf("leaf cells: mixed %lld, leaf lines %lld\n", (long long)tb.n_cell_mixed, (long long)tb.n_cell_line);
    const uint16_t* sub = tb.sub.data();
    auto sub_at = [&](int64_t i, int64_t j) { return sub[(size_t)(j * NX + i)]; };
    // per quad shift q: uniform quads (one pure code over all their sub-blocks)
    for (int q = 1; q <= 5; q++) {
        const int64_t qnx = (NX + (1 << q) - 1) >> q, qny = (NY + (1 << q) - 1) >> q;
        std::vector<uint16_t> qc((size_t)(qnx * qny), 0xfffe);
        for (int64_t j = 0; j < NY; j++)
            for (int64_t i = 0; i < NX; i++) {
                uint16_t e = sub_at(i, j);
                uint16_t c = (e & tiles::kSubBlock) ? tiles::kMixed : e;
                uint16_t& d = qc[(size_t)((j >> q) * qnx + (i >> q))];
                if (d == 0xfffe) d = c;
                else if (d != c) d = tiles::kMixed;
            }
        int64_t nonu = 0;
        for (uint16_t c : qc) nonu += c == tiles::kMixed;
        // super-tiles of 16 x 16 quads: distinct codes
        const int64_t snx = (qnx + 15) / 16, sny = (qny + 15) / 16;
        std::vector<std::set<uint16_t>> pal((size_t)(snx * sny));
        for (int64_t j = 0; j < NY; j++)
            for (int64_t i = 0; i < NX; i++) {
                uint16_t e = sub_at(i, j);
                if (e & tiles::kSubBlock) continue;
                pal[(size_t)(((j >> q) / 16) * snx + ((i >> q) / 16))].insert(e);
            }
        size_t pmax = 0, over14 = 0, over6 = 0;
        for (auto& s : pal) {
            pmax = std::max(pmax, s.size());
            over14 += s.size() > 14;
            over6 += s.size() > 6;
        }
        // uniform points
        std::mt19937_64 rng(7);
        std::uniform_real_distribution<double> u(0.0, 1.0);
        long in_uni = 0, in_grid = 0;
        for (long k = 0; k < npts / 4; k++) {
            double x = bx0 + (bx1 - bx0) * u(rng), y = by0 + (by1 - by0) * u(rng);
            double gx = (x - tb.grid.x0) * tb.grid.sx * S, gy = (y - tb.grid.y0) * tb.grid.sy * S;
            if (!(gx >= 0 && gx < NX && gy >= 0 && gy < NY)) {
                in_uni++;
                continue;
            }
            in_grid++;
            if (qc[(size_t)(((int64_t)gy >> q) * qnx + ((int64_t)gx >> q))] != tiles::kMixed) in_uni++;
        }
        printf("q %d: %lld x %lld quads (%lld), non-uniform %lld (%.1f%%); points decided by the quad level %.4f; "
               "super-tiles %lld, palette max %zu, >6 codes %zu, >14 codes %zu; LDS nibbles %.1f KB\n",
               q, (long long)qnx, (long long)qny, (long long)(qnx * qny), (long long)nonu,
               100.0 * nonu / (qnx * qny), (double)in_uni / (npts / 4), (long long)(snx * sny), pmax, over6, over14,
               qnx * qny / 2048.0);
    }
    // LDS records for the non-uniform quads of the q = 4 level: a 2^(4-L) x 2^(4-L) grid of
    // sub-quads (2^L x 2^L sub-blocks) each naming one of the quad's K most frequent uniform codes
    // (or "gather"): share of the uniform points such a record decides.
    for (int q = 3; q <= 6; q++) {
        const int64_t qnx = (NX + (1 << q) - 1) >> q, qny = (NY + (1 << q) - 1) >> q;
        auto code_at = [&](int64_t i, int64_t j) -> uint16_t {
            if (i >= NX || j >= NY) return 0;
            uint16_t e = sub_at(i, j);
            return (e & tiles::kSubBlock) ? tiles::kMixed : e;
        };
        for (int L = q - 4; L <= q - 2; L++)
            for (int K = 1; K <= 2; K++) {
                if (L < 0) continue;
                const int g = 1 << (q - L);  // sub-quads per quad side
                // per quad: its sub-quad codes (kMixed: not uniform) and its top-K codes
                std::vector<uint16_t> sq((size_t)(qnx * qny * g * g));
                std::vector<std::vector<uint16_t>> top((size_t)(qnx * qny));
                int64_t nonu = 0;
                for (int64_t qj = 0; qj < qny; qj++)
                    for (int64_t qi = 0; qi < qnx; qi++) {
                        std::unordered_map<uint16_t, int> cnt;
                        bool uni = true;
                        uint16_t first = code_at(qi << q, qj << q);
                        for (int b = 0; b < g; b++)
                            for (int a = 0; a < g; a++) {
                                uint16_t c = 0xfffe;
                                for (int dj = 0; dj < (1 << L); dj++)
                                    for (int di = 0; di < (1 << L); di++) {
                                        uint16_t e = code_at((qi << q) + (a << L) + di, (qj << q) + (b << L) + dj);
                                        if (c == 0xfffe) c = e;
                                        else if (c != e) c = tiles::kMixed;
                                        uni = uni && e == first && e != tiles::kMixed;
                                    }
                                sq[(size_t)((qj * qnx + qi) * g * g + b * g + a)] = c;
                                if (c != tiles::kMixed) cnt[c]++;
                            }
                        if (uni) continue;
                        nonu++;
                        std::vector<std::pair<int, uint16_t>> v;
                        for (auto& kv : cnt) v.push_back({-kv.second, kv.first});
                        std::sort(v.begin(), v.end());
                        for (int k = 0; k < K && k < (int)v.size(); k++) top[(size_t)(qj * qnx + qi)].push_back(v[k].second);
                    }
                std::mt19937_64 rng(7);
                std::uniform_real_distribution<double> u(0.0, 1.0);
                long dec = 0, tot = 0;
                for (long k = 0; k < npts / 4; k++) {
                    double x = bx0 + (bx1 - bx0) * u(rng), y = by0 + (by1 - by0) * u(rng);
                    double gx = (x - tb.grid.x0) * tb.grid.sx * S, gy = (y - tb.grid.y0) * tb.grid.sy * S;
                    tot++;
                    if (!(gx >= 0 && gx < NX && gy >= 0 && gy < NY)) { dec++; continue; }
                    const int64_t ix = (int64_t)gx, iy = (int64_t)gy, qq = (iy >> q) * qnx + (ix >> q);
                    const auto& t = top[(size_t)qq];
                    if (t.empty()) { dec++; continue; }
                    const uint16_t c = sq[(size_t)(qq * g * g + ((iy >> L) & (g - 1)) * g + ((ix >> L) & (g - 1)))];
                    if (c != tiles::kMixed && std::find(t.begin(), t.end(), c) != t.end()) dec++;
                }
                const int bits = K == 1 ? 1 : 2;
                const double kb = nonu * ((g * g * bits + 7) / 8 + 2 * K) / 1024.0;
                printf("q%d records: sub-quads %dx%d (L %d), top-%d codes: decided %.4f; %lld records x %d B = %.1f KB"
                       " + quad table %.1f KB = %.1f KB\n",
                       q, g, g, L, K, (double)dec / tot, (long long)nonu, (g * g * bits + 7) / 8 + 2 * K, kb,
                       qnx * qny * 2 / 1024.0, kb + qnx * qny * 2 / 1024.0);
            }
    }
    // point categories under the built raster (its own quad level)
    std::mt19937_64 rng(11);
    std::uniform_real_distribution<double> u(0.0, 1.0);
    long c_out = 0, c_quad = 0, c_sub = 0, c_line = 0, c_line_mixed = 0, c_leaf = 0, c_leaf_mixed = 0, c_submixed = 0;
    const int qs = tb.qshift;
    for (long k = 0; k < npts; k++) {
        double x = bx0 + (bx1 - bx0) * u(rng), y = by0 + (by1 - by0) * u(rng);
        double gx = (x - tb.grid.x0) * tb.grid.sx * S, gy = (y - tb.grid.y0) * tb.grid.sy * S;
        if (!(gx >= 0 && gx < NX && gy >= 0 && gy < NY)) {
            c_out++;
            continue;
        }
        int64_t ix = (int64_t)gx, iy = (int64_t)gy;
        uint16_t qe = tb.quad.empty() ? tiles::kMixed : tb.quad[(size_t)((iy >> qs) * tb.qnx + (ix >> qs))];
        if (!(qe & tiles::kSubBlock)) {
            c_quad++;
            continue;
        }
        uint16_t e = sub_at(ix, iy);
        if (!tiles::sub_is_block(e)) {
            if (e == tiles::kMixed) c_submixed++;
            else c_sub++;
            continue;
        }
        uint16_t code = tiles::raster_code(
            tiles::PointRaster{sub, tb.tile_base.data(), tb.blocks.data(), tb.grid.sx * S, tb.grid.sy * S, (int32_t)NX,
                               (int32_t)NY, C, tb.sshift, tb.grid.nx, tb.cshift, nullptr, 0, 0, 0, nullptr, nullptr, 0, 0,
                               tb.tile_lbase.data(), tb.llines.empty() ? nullptr : tb.llines.data()},
            tb.grid.x0, tb.grid.y0, x, y);
        if (e & tiles::kLineBit) {
            c_line++;
            c_line_mixed += code == tiles::kMixed;
        } else {
            c_leaf++;
            c_leaf_mixed += code == tiles::kMixed;
        }
    }
    printf("uniform points %ld: outside grid %.4f, quad level %.4f, sub-block pure %.4f, sub-block mixed %.4f, "
           "line %.4f (mixed band %.5f), leaf %.4f (mixed cell %.5f)\n",
           npts, (double)c_out / npts, (double)c_quad / npts, (double)c_sub / npts, (double)c_submixed / npts,
           (double)c_line / npts, (double)c_line_mixed / npts, (double)c_leaf / npts, (double)c_leaf_mixed / npts);
    // POINTS=file (float64 x[n] then y[n]): the stream kernel's groups of 256 consecutive rows --
    // rows whose quad entry (after the quad records) is not a code are "pending" (k_join_stream_cpt
    // compacts them into 64-row sets: P <= 64 one pipelined set, <= 128 two, more: unpipelined sets)
    if (const char* pf = getenv("POINTS")) {
        FILE* fp = fopen(pf, "rb");
        if (!fp) return 4;
        fseek(fp, 0, SEEK_END);
        const long nb = ftell(fp);
        fseek(fp, 0, SEEK_SET);
        const size_t np = (size_t)nb / 16;
        std::vector<double> px(np), py(np);
        if (fread(px.data(), 8, np, fp) != np || fread(py.data(), 8, np, fp) != np) return 4;
        fclose(fp);
        tiles::PointRaster pr{};
        pr.sub = tb.sub.data();
        pr.tile_base = tb.tile_base.data();
        pr.blocks = tb.blocks.data();
        pr.sx = tb.grid.sx * S;
        pr.sy = tb.grid.sy * S;
        pr.nx = (int32_t)NX;
        pr.ny = (int32_t)NY;
        pr.C = C;
        pr.sshift = tb.sshift;
        pr.tnx = tb.grid.nx;
        pr.cshift = tb.cshift;
        pr.quad = tb.quad.data();
        pr.qnx = tb.qnx;
        pr.qny = tb.qny;
        pr.qshift = tb.qshift;
        pr.qrec_mask = tb.qrec_mask.empty() ? nullptr : tb.qrec_mask.data();
        pr.qrec_code = tb.qrec_code.empty() ? nullptr : tb.qrec_code.data();
        pr.n_qrec = (int32_t)tb.qrec_code.size();
        pr.qrec_shift = tb.qrec_shift;
        const int F = tiles::kFixBits;
        const double ax = pr.sx * C * (double)(1 << F), ay = pr.sy * C * (double)(1 << F);
        const double bx = -tb.grid.x0 * ax, by = -tb.grid.y0 * ay;
        const uint32_t gxmax = (uint32_t)(((int64_t)NX * C - 1) << F), gymax = (uint32_t)(((int64_t)NY * C - 1) << F);
        long groups = 0, g64 = 0, g128 = 0, pend = 0, line = 0, leaf = 0, mixed = 0, extra_sets = 0;
        long hist[5] = {0, 0, 0, 0, 0};  // P: 0, 1-16, 17-64, 65-128, > 128
        for (size_t g0 = 0; g0 + 256 <= np; g0 += 256) {
            int P = 0;
            for (size_t r = g0; r < g0 + 256; r++) {
                uint32_t gix = tiles::fix_cvt(fma(px[r], ax, bx)), giy = tiles::fix_cvt(fma(py[r], ay, by));
                gix = gix > gxmax ? gxmax : gix;
                giy = giy > gymax ? gymax : giy;
                const int ixC = (int)(gix >> F), iyC = (int)(giy >> F), ix = ixC >> tb.cshift, iy = iyC >> tb.cshift;
                uint32_t q = pr.quad[(uint32_t)(iy >> pr.qshift) * (uint32_t)pr.qnx + (uint32_t)(ix >> pr.qshift)];
                if (q >= tiles::kSubBlock && (q & 0x7fffu) < (uint32_t)pr.n_qrec) {
                    const uint32_t rr = q & 0x7fffu;
                    const uint32_t b = (uint32_t)((((iy >> pr.qrec_shift) & 7) << 3) | ((ix >> pr.qrec_shift) & 7));
                    if ((pr.qrec_mask[2 * rr + (b >> 5)] >> (b & 31)) & 1u) q = pr.qrec_code[rr];
                }
                if (q < tiles::kSubBlock) continue;
                P++;
                const int qm = (1 << pr.qshift) - 1;
                const uint32_t e = pr.sub[(size_t)pr.nx * pr.ny + ((size_t)(q & 0x7fffu) << (2 * pr.qshift)) +
                                          (size_t)(((iy & qm) << pr.qshift) | (ix & qm))];
                if (tiles::sub_is_block(e)) (e & tiles::kLineBit) ? line++ : leaf++;
                const uint16_t code = tiles::raster_code_fixed(pr, ax, bx, ay, by, gxmax, gymax, px[r], py[r]);
                mixed += code == tiles::kMixed;
            }
            groups++;
            pend += P;
            g64 += P > 64;
            g128 += P > 128;
            if (P > 128) extra_sets += (P + 63) / 64 - 2;
            hist[P == 0 ? 0 : (P <= 16 ? 1 : (P <= 64 ? 2 : (P <= 128 ? 3 : 4)))]++;
        }
        printf("points %zu in %ld groups of 256: pending rows (sub-block gathers) %.4f per point; groups with "
               "P > 64 (second set) %.4f, P > 128 (unpipelined sets) %.4f, unpipelined sets per group %.4f; "
               "P histogram 0 / 1-16 / 17-64 / 65-128 / >128: %.4f %.4f %.4f %.4f %.4f; line gathers %.4f, leaf "
               "gathers %.4f, mixed rows %.5f per point\n",
               np, groups, (double)pend / (groups * 256.0), (double)g64 / groups, (double)g128 / groups,
               (double)extra_sets / groups, (double)hist[0] / groups, (double)hist[1] / groups, (double)hist[2] / groups,
               (double)hist[3] / groups, (double)hist[4] / groups, (double)line / (groups * 256.0),
               (double)leaf / (groups * 256.0), (double)mixed / (groups * 256.0));
    }
    return 0;
}
