// Test-only: builds the H3 tile directory of mosaic_amd/csrc/tiles.h on the host for a set of chip
// cells and checks the kernel's per-point decision (k_join_tiled / tiled_cell) against h3_exact
// (the H3 C restatement, glibc libm, as the oracle) on uniform points over and around the grid,
// points on and next to tile and grid boundaries, and points near the chip cells.
// With chip rows it also builds the point raster (tiles_build.cpp) and checks every pure raster
// code against the exact answer: the keys of the core chips of the point's exact cell plus the keys
// of its border chips whose JTS contains() (pip_device.h, itself pinned against the oracle) holds.
// Input file: int32 res, uint32 n_chips, then per chip: int64 cell, uint8 is_core, int32 key,
//             uint32 wkb length, wkb bytes.
// Usage: tiles_selfcheck <chips.bin> <points> <seed> [S C]
//   -> prints "built mismatches checked skipped_tiles full_tiles uncertified window_misses
//              raster_built raster_bad raster_pure raster_mixed"
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <unordered_map>
#include <vector>

#include <algorithm>

#include "../../mosaic_amd/csrc/geom_build.h"
#include "../../mosaic_amd/csrc/tiles_build.cpp"

using namespace mosaic;

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    int32_t res = 0;
    uint32_t nchips = 0;
    if (fread(&res, 4, 1, f) != 1 || fread(&nchips, 4, 1, f) != 1) return 2;
    // chips sorted by cell (as the chip table orders them)
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
    uint32_t n = (uint32_t)cells.size();
    long npts = atol(argv[2]);
    std::mt19937_64 rng(atoi(argv[3]));
    std::uniform_real_distribution<double> u(0.0, 1.0);
    std::unordered_map<int64_t, int64_t> slot;
    // slots: cell k -> slot 3k + 1 (arbitrary, sparse), with its chip range
    std::vector<uint32_t> slot_first((size_t)n * 3 + 2, 0), slot_count((size_t)n * 3 + 2, 0);
    for (uint32_t k = 0; k < n; k++) {
        slot.emplace(cells[k], (int64_t)k * 3 + 1);
        slot_first[(size_t)k * 3 + 1] = first[k];
        slot_count[(size_t)k * 3 + 1] = count[k];
    }
    auto slot_of = [&](int64_t h) -> int64_t {
        auto it = slot.find(h);
        return it == slot.end() ? -1 : it->second;
    };
    tiles::Builder tb;
    bool ok = tb.build(res, cells, slot_of);
    if (!ok) {
        printf("0 0 0 0 0 0 0 0 0 0 0\n");
        fprintf(stderr, "not built: %s\n", tb.why);
        return 0;
    }
    int S = argc > 5 ? atoi(argv[4]) : 16, Cc = argc > 5 ? atoi(argv[5]) : 8;
    tiles::Builder::ChipSource src;
    src.slot_first = slot_first.data();
    src.slot_count = slot_count.data();
    src.meta = meta.data();
    src.store = pip::GeomStore{gb.verts.data(), gb.ring_start.data(), gb.ring_bbox.data(), gb.part_ring.data(),
                               gb.geom_part.data(), gb.geom_bbox.data()};
    src.n_polygons = npoly;
    // the stream kernel's LDS shape: quad level in half of ~130 KB, quad records in the rest
    tb.quad_max = 16384;
    tb.leaf_lines = getenv("TILES_NO_LEAF_LINES") == nullptr;  // leaf lines certified too (every pure code is checked)
    tb.quad_lds_bytes = 130 * 1024;
    bool rok = tb.build_raster(src, S, Cc, 8);
    tiles::PointRaster pr{};
    if (rok) {
        pr.sub = tb.sub.data();
        pr.tile_base = tb.tile_base.data();
        pr.sshift = tb.sshift;
        pr.tnx = tb.grid.nx;
        pr.blocks = tb.blocks.data();
        pr.sx = tb.grid.sx * S;
        pr.sy = tb.grid.sy * S;
        pr.nx = tb.grid.nx * S;
        pr.ny = tb.grid.ny * S;
        pr.C = Cc;
        pr.cshift = tb.cshift;
        pr.quad = tb.quad.empty() ? nullptr : tb.quad.data();
        pr.qnx = tb.qnx;
        pr.qny = tb.qny;
        pr.qshift = tb.qshift;
        pr.qrec_mask = tb.qrec_mask.empty() ? nullptr : tb.qrec_mask.data();
        pr.qrec_code = tb.qrec_code.empty() ? nullptr : tb.qrec_code.data();
        pr.n_qrec = (int32_t)tb.qrec_code.size();
        pr.qrec_shift = tb.qrec_shift;
        pr.tile_lbase = tb.tile_lbase.data();
        pr.llines = tb.llines.empty() ? nullptr : tb.llines.data();
        fprintf(stderr, "quad level %d x %d shift %d, %d quad records\n", tb.qnx, tb.qny, tb.qshift, pr.n_qrec);
    }
    long rbad = 0, rpure = 0, rfpure = 0, rmixed = 0, uni = 0, uni_mixed = 0;
    double bx0 = argc > 9 ? atof(argv[6]) : 0, by0 = argc > 9 ? atof(argv[7]) : 0;
    double bx1 = argc > 9 ? atof(argv[8]) : 0, by1 = argc > 9 ? atof(argv[9]) : 0;
    long st_out = 0, st_skip = 0, st_sub = 0, st_quad = 0;
    int Q = argc > 10 ? atoi(argv[10]) : 4;
    // quad level: Q x Q sub-blocks with one shared pure code
    std::vector<uint8_t> quad_pure;
    if (rok) {
        int qx = (pr.nx + Q - 1) / Q, qy = (pr.ny + Q - 1) / Q;
        quad_pure.assign((size_t)qx * qy, 1);
        for (int j = 0; j < pr.ny; j++)
            for (int i = 0; i < pr.nx; i++) {
                uint16_t e = pr.sub[(size_t)j * pr.nx + i];
                uint16_t e0 = pr.sub[(size_t)(j / Q * Q) * pr.nx + (i / Q * Q)];
                if (tiles::sub_is_block(e) || e != e0) quad_pure[(size_t)(j / Q) * qx + i / Q] = 0;
            }
    }
    if (rok && argc > 9)  // raster hit statistics for uniform points over a bbox
        for (long k = 0; k < npts; k++) {
            double x = bx0 + (bx1 - bx0) * u(rng), y = by0 + (by1 - by0) * u(rng);
            uni++;
            if (tiles::raster_code(pr, tb.grid.x0, tb.grid.y0, x, y) == tiles::kMixed) uni_mixed++;
            double gx = (x - tb.grid.x0) * pr.sx, gy = (y - tb.grid.y0) * pr.sy;
            if (!(gx >= 0 && gx < pr.nx && gy >= 0 && gy < pr.ny)) {
                st_out++;
                continue;
            }
            int ix = (int)gx, iy = (int)gy;
            if (tb.tile_idx[(size_t)(iy / tb.S) * tb.grid.nx + ix / tb.S] == tiles::kSkip) st_skip++;
            if (!tiles::sub_is_block(pr.sub[(size_t)iy * pr.nx + ix])) st_sub++;
            if (quad_pure[(size_t)(iy / Q) * ((pr.nx + Q - 1) / Q) + ix / Q]) st_quad++;
        }
    if (uni)
        fprintf(stderr, "uniform: outside %.4f skip-tile %.4f pure-sub %.4f pure-quad(%d) %.4f\n", (double)st_out / uni,
                (double)st_skip / uni, (double)st_sub / uni, Q, (double)st_quad / uni);
    const tiles::Grid& g = tb.grid;
    double w = g.nx / g.sx, h = g.ny / g.sy;
    long bad = 0, checked = 0, skipped = 0, full = 0, unc = 0, miss = 0;
    auto check = [&](double x, double y) {
        uint32_t code = tiles::tile_of(g, tb.tile_idx.data(), x, y);
        double lat = h3::to_radians(y, 8), lon = h3::to_radians(x, 8);
        int64_t want = (int64_t)h3::h3_exact(lat, lon, res);
        int64_t want_slot = slot_of(want);
        if (rok) {
            uint16_t rc = tiles::raster_code(pr, g.x0, g.y0, x, y);
            // the kernel's path through the quad level and its compact copies agrees with it
            const uint16_t rq = tiles::raster_code(pr, g.x0, g.y0, x, y, true);
            if (rq != rc) {
                rbad++;
                if (rbad < 10) fprintf(stderr, "quad lookup: %u vs %u\n", rq, rc);
            }
            // k_join_stream_pipe's fixed-point form: every pure code it gives is the exact answer too
            const double fs = (double)(1 << tiles::kFixBits), sxC = pr.sx * pr.C, syC = pr.sy * pr.C;
            const uint16_t rf = !pr.quad ? (uint16_t)tiles::kMixed : tiles::raster_code_fixed(
                pr, sxC * fs, (-g.x0 * sxC) * fs, syC * fs, (-g.y0 * syC) * fs,
                (uint32_t)(((int64_t)pr.nx * pr.C - 1) << tiles::kFixBits), (uint32_t)(((int64_t)pr.ny * pr.C - 1) << tiles::kFixBits),
                x, y);
            if (rf != tiles::kMixed) rfpure++;
            if (rc == tiles::kMixed && rf == tiles::kMixed) {
                rmixed++;
            } else {
                if (rc != tiles::kMixed) rpure++;
                std::vector<int32_t> keys;
                if (want_slot >= 0)
                    for (uint32_t c = slot_first[want_slot]; c < slot_first[want_slot] + slot_count[want_slot]; c++)
                        if ((meta[c] & 1u) || pip::contains(src.store, c, x, y)) keys.push_back((int32_t)(meta[c] >> 1));
                uint16_t wc = keys.empty() ? 0 : (keys.size() == 1 ? (uint16_t)(keys[0] + 1) : tiles::kMixed);
                if (rc != tiles::kMixed && wc != rc) {
                    rbad++;
                    if (rbad < 10)
                        fprintf(stderr, "raster: %.17g %.17g code %u want %u (cell %llx)\n", x, y, rc, wc,
                                (unsigned long long)want);
                }
                if (rf != tiles::kMixed && wc != rf) {
                    rbad++;
                    if (rbad < 10)
                        fprintf(stderr, "raster (fixed point): %.17g %.17g code %u want %u (cell %llx)\n", x, y, rf,
                                wc, (unsigned long long)want);
                }
            }
        }
        if (code == tiles::kFull) {
            full++;
            return;
        }
        if (code == tiles::kSkip) {
            skipped++;
            checked++;
            if (want_slot >= 0) {
                bad++;
                if (bad < 10) fprintf(stderr, "skip but joins: %.17g %.17g cell %llx\n", x, y, (unsigned long long)want);
            }
            return;
        }
        const tiles::TileRec r = tb.recs[code - 2];
        int face = (int)(r.dims & 0xffu), wa = (int)((r.dims >> 8) & 0xfffu), wb = (int)(r.dims >> 20);
        double px, py, pz, vx, vy, best;
        h3::fast_unit(y, x, &px, &py, &pz);
        h3::fast_plane(px, py, pz, face, res, &vx, &vy, &best);
        int ba, bb;
        if (!h3::fast_hex(vx, vy, res, &ba, &bb)) {
            unc++;
            return;
        }
        checked++;
        int ra = ba - r.a0, rb = bb - r.b0;
        int64_t got_slot;
        if ((unsigned)ra < (unsigned)wa && (unsigned)rb < (unsigned)wb) {
            uint32_t e = tb.entries[r.off + (uint32_t)(ra * wb + rb)];
            got_slot = e ? (int64_t)e - 1 : -1;
        } else {
            miss++;
            got_slot = slot_of((int64_t)h3::face_axial_to_h3(face, ba, bb, res));
        }
        if (got_slot != want_slot) {
            bad++;
            if (bad < 10)
                fprintf(stderr, "window: %.17g %.17g got %lld want %lld (cell %llx)\n", x, y, (long long)got_slot,
                        (long long)want_slot, (unsigned long long)want);
        }
    };
    for (long k = 0; k < npts; k++) {
        int kind = (int)(k % 6);
        double x, y;
        if (kind == 0) {  // uniform over the grid widened by 10 %
            x = g.x0 - 0.1 * w + 1.2 * w * u(rng);
            y = g.y0 - 0.1 * h + 1.2 * h * u(rng);
        } else if (kind == 1) {  // on / next to a tile column boundary
            int i = (int)(u(rng) * (g.nx + 1));
            x = g.x0 + i / g.sx;
            int s = (int)(u(rng) * 5) - 2;
            for (int t = 0; t < abs(s); t++) x = nextafter(x, s > 0 ? INFINITY : -INFINITY);
            y = g.y0 + h * u(rng);
        } else if (kind == 2) {  // on / next to a tile row boundary
            int j = (int)(u(rng) * (g.ny + 1));
            y = g.y0 + j / g.sy;
            int s = (int)(u(rng) * 5) - 2;
            for (int t = 0; t < abs(s); t++) y = nextafter(y, s > 0 ? INFINITY : -INFINITY);
            x = g.x0 + w * u(rng);
        } else if (kind >= 4 && gb.verts.size() > 1) {  // on / next to border chip vertices and segments
            size_t v = (size_t)(u(rng) * (gb.verts.size() - 1));
            double t = kind == 4 ? 0.0 : u(rng);
            x = gb.verts[v].x + t * (gb.verts[v + 1].x - gb.verts[v].x);
            y = gb.verts[v].y + t * (gb.verts[v + 1].y - gb.verts[v].y);
            int sx = (int)(u(rng) * 5) - 2, sy = (int)(u(rng) * 5) - 2;
            for (int q = 0; q < abs(sx); q++) x = nextafter(x, sx > 0 ? INFINITY : -INFINITY);
            for (int q = 0; q < abs(sy); q++) y = nextafter(y, sy > 0 ? INFINITY : -INFINITY);
        } else {  // near a chip cell centre (within ~2 hex units)
            int64_t c = cells[(size_t)(u(rng) * n) % n];
            double cx, cy;
            tiles::cell_center((uint64_t)c, res, &cx, &cy);
            x = cx + (u(rng) - 0.5) * 4.0 / (g.sx * 4.0) * 2.0;
            y = cy + (u(rng) - 0.5) * 4.0 / (g.sy * 4.0) * 2.0;
        }
        check(x, y);
    }
    if (rok && !tb.edge_ok) {
        rbad++;
        fprintf(stderr, "an edge sub-block answers a pair\n");
    }
    // tile-frame line records: one copy per tile and edge -- the records a tile's line sub-blocks
    // name are pairwise distinct (the assembly's deduplication) and fewer than those sub-blocks
    if (rok && !tb.sub.empty()) {
        const int64_t NXs = (int64_t)g.nx << tb.sshift, NYs = (int64_t)g.ny << tb.sshift;
        long nrec = 0, dup = 0;
        for (int64_t tj = 0; tj < g.ny; tj++)
            for (int64_t ti = 0; ti < g.nx; ti++) {
                uint32_t nmax = 0;
                bool any = false;
                for (int64_t sj = tj << tb.sshift; sj < (tj + 1) << tb.sshift && sj < NYs; sj++)
                    for (int64_t si = ti << tb.sshift; si < (ti + 1) << tb.sshift && si < NXs; si++) {
                        const uint16_t e = tb.sub[(size_t)(sj * NXs + si)];
                        if (tiles::sub_is_block(e) && (e & tiles::kLineBit)) {
                            nmax = std::max<uint32_t>(nmax, (uint32_t)(e & 0x3fffu) + 1u);
                            any = true;
                        }
                    }
                if (!any) continue;
                nrec += nmax;
                const size_t base = tb.tile_base[(size_t)(tj * g.nx + ti)];
                for (uint32_t p = 0; p < nmax; p++)
                    for (uint32_t q = p + 1; q < nmax; q++)
                        dup += memcmp(tb.blocks.data() + base - 8 * (size_t)(p + 1), tb.blocks.data() + base - 8 * (size_t)(q + 1),
                                      sizeof(tiles::LineRec)) == 0;
            }
        fprintf(stderr, "line records %ld for %lld line sub-blocks, duplicates %ld\n", nrec, (long long)tb.n_sub_line, dup);
    }
    fprintf(stderr, "pure codes: float form %ld, fixed-point form %ld\n", rpure, rfpure);
    printf("1 %ld %ld %ld %ld %ld %ld %d %ld %ld %ld\n", bad, checked, skipped, full, unc, miss, rok ? 1 : 0, rbad, rpure,
           rmixed);
    if (uni) fprintf(stderr, "uniform over bbox: %ld points, %.4f mixed\n", uni, (double)uni_mixed / uni);
    fprintf(stderr, "raster S %d C %d: sub %zu block elements %zu, pure sub %lld mixed sub %lld (line %lld) mixed cells %lld\n",
            S, Cc, tb.sub.size(), tb.blocks.size(), (long long)tb.n_sub_pure, (long long)tb.n_sub_mixed,
            (long long)tb.n_sub_line, (long long)tb.n_cell_mixed);
    fprintf(stderr, "grid %d x %d, rings %d, records %zu, entries %zu, full tiles %lld\n", g.nx, g.ny, tb.rings,
            tb.recs.size(), tb.entries.size(), (long long)tb.n_full);
    return 0;
}
