// CPU check of the binned join's tile images (mosaic_amd/csrc/tile_images.h) on a chip set in the
// chips.bin format of tiles_selfcheck.cpp: every image's header (record, level, part) and chip
// records (meta, geometry reference, window slot, outward-rounded envelope, f32-frame vertices)
// against the chip table, and for random points of every tile -- computed into the envelope raster
// exactly as k_bin_cover / k_join_tiles do -- every window chip whose envelope holds the point is
// listed in the point's raster cell of its part's image, and the record's cover bit of that cell is
// set exactly when the cell's list is not empty.
// Prints: records, images, points checked, failures, records at levels 0, 1, 2.
#include <math.h>

#include <cmath>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <unordered_map>
#include <vector>

#include "../../mosaic_amd/csrc/geom_build.h"
#include "../../mosaic_amd/csrc/tile_images.h"
#include "../../mosaic_amd/csrc/tiles_build.cpp"

using namespace mosaic;

int main(int argc, char** argv) {
    if (argc < 3) return 2;
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
    for (auto& r : rows) {
        uint32_t len = 0;
        if (fread(&r.cell, 8, 1, f) != 1 || fread(&r.core, 1, 1, f) != 1 || fread(&r.key, 4, 1, f) != 1 ||
            fread(&len, 4, 1, f) != 1)
            return 2;
        r.wkb.resize(len);
        if (len && fread(r.wkb.data(), 1, len, f) != len) return 2;
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
    auto first_of = [&](uint32_t e) { return first[e - 1]; };
    std::unordered_map<int64_t, int64_t> slot;
    for (uint32_t k = 0; k < n; k++) slot.emplace(cells[k], (int64_t)k);
    auto slot_of = [&](int64_t h) -> int64_t {
        auto it = slot.find(h);
        return it == slot.end() ? -1 : it->second;
    };
    tiles::Builder tb;
    if (!tb.build(res, cells, slot_of)) {
        fprintf(stderr, "not built: %s\n", tb.why);
        printf("0 0 0 0\n");
        return 0;
    }
    binned::ImageSource is;
    is.recs = tb.recs.data();
    is.n_recs = tb.recs.size();
    is.grid = tb.grid;
    is.tile_idx = tb.tile_idx.data();
    is.entries = tb.entries.data();
    is.slot_first = first.data();
    is.slot_count = count.data();
    is.meta = meta.data();
    is.store = pip::GeomStore{gb.verts.data(), gb.ring_start.data(), gb.ring_bbox.data(), gb.part_ring.data(),
                              gb.geom_part.data(), gb.geom_bbox.data()};
    is.threads = 8;
    if (argc > 3) is.cap_words = (uint32_t)atol(argv[3]);
    binned::ImageSet set;
    if (!binned::build_tile_images(is, set)) return 4;
    const size_t nr = tb.recs.size();
    if (set.cover.size() != nr * binned::kImgCoverWords || set.rec_key.size() != nr || set.rec.size() != set.off.size())
        return 5;
    const int G = binned::kImgRaster;
    std::mt19937_64 rng(5);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    const long pts_per_tile = atol(argv[2]);
    long imaged = 0, checked = 0, bad = 0;
    const tiles::Grid& g = tb.grid;
    // every image: header, and chip records against the chip table
    for (size_t k = 0; k < set.off.size(); k++) {
        const uint32_t r = set.rec[k];
        const uint32_t level = set.rec_key[r] & 3u, first = set.rec_key[r] >> 2;
        bad += k < first || k - first >= (1u << (2 * level));
        if (set.off[k] == binned::kNoImage) continue;
        imaged++;
        const uint32_t* im = set.words.data() + set.off[k];
        bad += im[5] != r || im[6] != (level | (uint32_t)(k - first) << 8);
        const tiles::TileRec& tr = tb.recs[r];
        const uint32_t nc = im[0];
        const uint32_t* chips = im + im[2];
        const float* V = (const float*)(im + im[3]);
        for (uint32_t c = 0; c < nc; c++) {
            const uint32_t* cr = chips + binned::kImgChipWords * c;
            const uint32_t q = cr[2], e = tb.entries[tr.off + cr[3]];
            bool ok = e != 0 && q >= first_of(e) && q < first_of(e) + count[e - 1] && cr[0] == meta[q];
            if (!ok) {
                bad++;
                continue;
            }
            float fb[4];
            memcpy(fb, cr + 4, 16);
            const pip::Box& bx = gb.geom_bbox[q];
            if (!(meta[q] & 1u) && bx.minx <= bx.maxx)
                ok = ok && fb[0] <= bx.minx && fb[1] <= bx.miny && fb[2] >= bx.maxx && fb[3] >= bx.maxy;
            const uint32_t vc = cr[1] >> 16;
            if (!(meta[q] & 1u) && vc != binned::kImgGlobal) {
                const uint32_t v0 = gb.ring_start[gb.part_ring[gb.geom_part[q]]];
                ok = ok && vc == gb.ring_start[gb.part_ring[gb.geom_part[q]] + 1] - v0;
                for (uint32_t v = 0; ok && v < vc; v++)
                    ok = V[2 * ((cr[1] & 0xffffu) + v)] == (float)(gb.verts[v0 + v].x - (double)fb[0]) &&
                         V[2 * ((cr[1] & 0xffffu) + v) + 1] == (float)(gb.verts[v0 + v].y - (double)fb[1]);
            }
            bad += !ok;
        }
    }
    // points of every record's tile (random, on tile edges, and the window chips' envelope corners
    // and edge midpoints): every window chip whose envelope holds the point is listed in the point's
    // raster cell of its part's image, and the record's cover bit of the cell is set exactly when
    // that list is not empty
    for (int64_t t = 0; t < (int64_t)g.nx * g.ny; t++) {
        const uint32_t code = tb.tile_idx[(size_t)t];
        if (code < 2) continue;
        const uint32_t r = code - 2;
        const tiles::TileRec& tr = tb.recs[r];
        std::vector<uint32_t> wchips;
        const uint32_t ns = ((tr.dims >> 8) & 0xfffu) * (tr.dims >> 20);
        for (uint32_t k = 0; k < ns; k++) {
            const uint32_t e = tb.entries[tr.off + k];
            if (e)
                for (uint32_t q = first_of(e); q < first_of(e) + count[e - 1]; q++) wchips.push_back(q);
        }
        const int ti = (int)(t % g.nx), tj = (int)(t / g.nx);
        std::vector<std::pair<double, double>> pts;
        for (long k = 0; k < pts_per_tile; k++) {
            double ux = U(rng), uy = U(rng);
            if (k % 8 == 0) ux = 0.0;
            if (k % 8 == 1) uy = 0.0;
            pts.push_back({g.x0 + (ti + ux) / g.sx, g.y0 + (tj + uy) / g.sy});
        }
        if (pts_per_tile > 0)
            for (uint32_t q : wchips) {
                const pip::Box& bx = gb.geom_bbox[q];
                if (!(bx.minx <= bx.maxx)) continue;
                const double xs[3] = {bx.minx, 0.5 * (bx.minx + bx.maxx), bx.maxx};
                const double ys[3] = {bx.miny, 0.5 * (bx.miny + bx.maxy), bx.maxy};
                for (double px : xs)
                    for (double py : ys) pts.push_back({px, py});
            }
        const uint32_t level = set.rec_key[r] & 3u, first = set.rec_key[r] >> 2;
        for (const auto& pt : pts) {
            const double x = pt.first, y = pt.second;
            if (tiles::tile_of(g, tb.tile_idx.data(), x, y) != code) continue;  // (rounding off the tile)
            const double fx = (x - g.x0) * g.sx, fy = (y - g.y0) * g.sy;
            const int gx = std::min((int)((fx - (double)(int)fx) * (double)G), G - 1);
            const int gy = std::min((int)((fy - (double)(int)fy) * (double)G), G - 1);
            const int cell = gy * G + gx;
            const uint32_t k = first + binned::image_part(cell, (int)level);
            const bool covered = (set.cover[(size_t)r * binned::kImgCoverWords + (cell >> 5)] >> (cell & 31)) & 1u;
            checked++;
            if (set.off[k] == binned::kNoImage) {
                // (no image: the generic path; the cover bit must still keep every holding chip's points)
                for (uint32_t q : wchips) {
                    const pip::Box& bx = gb.geom_bbox[q];
                    const bool holds = (meta[q] & 1u) || (x >= bx.minx && x <= bx.maxx && y >= bx.miny && y <= bx.maxy);
                    bad += holds && !covered;
                }
                continue;
            }
            const uint32_t* im = set.words.data() + set.off[k];
            const uint32_t* chips = im + im[2];
            const uint16_t* rl = (const uint16_t*)(im + im[4]);
            std::vector<uint32_t> lst;
            for (uint32_t p = rl[cell]; p < rl[cell + 1]; p++) lst.push_back(chips[binned::kImgChipWords * rl[p] + 2]);
            bad += covered != !lst.empty();
            for (uint32_t q : wchips) {
                const pip::Box& bx = gb.geom_bbox[q];
                const bool holds = (meta[q] & 1u) || (x >= bx.minx && x <= bx.maxx && y >= bx.miny && y <= bx.maxy);
                if (holds && std::find(lst.begin(), lst.end(), q) == lst.end()) bad++;
            }
        }
    }
    // k_bin_cover's per-point arithmetic on adversarial coordinates (off the grid on every side,
    // fractions below zero, huge, NaN, infinities, tile corners): every gather in range, every key
    // within the image keys, an in-grid point's key an image of its own record, and the bin map's
    // key and keep equal to those of the record tables
    {
        std::vector<double> vx = {g.x0, g.x0 - 1e-9, g.x0 - 0.5 / g.sx, g.x0 - 5.5 / g.sx, g.x0 + (g.nx - 1e-9) / g.sx,
                                  g.x0 + (double)g.nx / g.sx, 1e300, -1e300, NAN, INFINITY, -INFINITY, 0.0};
        std::vector<double> vy = {g.y0, g.y0 - 1e-9, g.y0 - 0.5 / g.sy, g.y0 - 5.5 / g.sy, g.y0 + (g.ny - 1e-9) / g.sy,
                                  g.y0 + (double)g.ny / g.sy, 1e300, -1e300, NAN, INFINITY, -INFINITY, 0.0};
        for (int k = 0; k < 4000; k++) {
            vx.push_back(g.x0 + (U(rng) * 1.2 - 0.1) * g.nx / g.sx);
            vy.push_back(g.y0 + (U(rng) * 1.2 - 0.1) * g.ny / g.sy);
        }
        for (double x : vx)
            for (double y : vy) {
                const binned::BinCell bc = binned::bin_cell(g, x, y);
                checked++;
                if (bc.slot < 0 || bc.slot >= (int64_t)g.nx * g.ny || bc.q < 0 || bc.q >= G * G) {
                    bad++;
                    continue;
                }
                uint32_t code = tb.tile_idx[(size_t)bc.slot];
                if (!bc.in) code = (std::isfinite(x) && std::isfinite(y)) ? tiles::kSkip : tiles::kFull;
                bad += tiles::tile_of(g, tb.tile_idx.data(), x, y) != code;  // (the keygen's code is tile_of's)
                const uint32_t r = code >= 2 ? code - 2 : 0;
                if (r >= nr || (size_t)r * binned::kImgCoverWords + (uint32_t)(bc.q >> 5) >= set.cover.size()) {
                    bad++;
                    continue;
                }
                const uint32_t key = binned::bin_key(code, set.rec_key[r], bc.q);
                if (code >= 2) bad += key < 2 || key - 2 >= set.off.size() || set.rec[key - 2] != r;
                else bad += key != code;
                const bool keep = code != tiles::kSkip &&
                                  (code < 2 || ((set.cover[(size_t)r * binned::kImgCoverWords + (bc.q >> 5)] >> (bc.q & 31)) & 1u));
                // k_bin_cover's reads: the tile's bin map record (in range), then the same key and keep
                const size_t mi = (size_t)bc.slot * binned::kBinMapWords;
                if (mi + binned::kBinMapWords > set.bin_map.size()) {
                    bad++;
                    continue;
                }
                uint32_t kw = set.bin_map[mi], cw = set.bin_map[mi + 1 + (bc.q >> 5)];
                if (!bc.in) {
                    kw = (std::isfinite(x) && std::isfinite(y)) ? tiles::kSkip : tiles::kFull;
                    cw = ~0u;
                }
                bad += binned::bin_map_keep(kw, cw, bc.q) != keep;
                if (keep) bad += binned::bin_map_key(kw, bc.q) != key;
            }
    }
    printf("%zu %ld %ld %ld %u %u %u\n", nr, imaged, checked, bad, set.levels[0], set.levels[1], set.levels[2]);
    return 0;
}
