// CPU check of the binned join's tile images (mosaic_amd/csrc/tile_images.h) on a chip set in the
// chips.bin format of tiles_selfcheck.cpp: every image's chip records (meta, geometry reference,
// window slot, outward-rounded envelope, vertices) against the chip table, and for random points
// of every imaged tile -- computed into the envelope raster exactly as k_join_tiles does -- every
// chip of the tile whose envelope holds the point is listed in the point's raster cell.
// Prints: records, imaged records, points checked, failures.
#include <math.h>
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
    std::vector<uint32_t> words, off;
    uint32_t max_words = 0;
    if (!binned::build_tile_images(is, words, off, max_words)) return 4;
    const int G = binned::kImgRaster;
    std::mt19937_64 rng(5);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    const long pts_per_tile = atol(argv[2]);
    long imaged = 0, checked = 0, bad = 0;
    const tiles::Grid& g = tb.grid;
    for (int64_t t = 0; t < (int64_t)g.nx * g.ny; t++) {
        const uint32_t code = tb.tile_idx[(size_t)t];
        if (code < 2 || off[code - 2] == binned::kNoImage) continue;
        imaged++;
        const uint32_t* im = words.data() + off[code - 2];
        const tiles::TileRec& tr = tb.recs[code - 2];
        const uint32_t ns = im[0] & 0xffffu, nc = im[0] >> 16;
        const uint32_t* chips = im + im[2];
        const double* V = (const double*)(im + im[3]);
        const uint16_t* rl = (const uint16_t*)(im + im[4]);
        // chip records against the table, in window order
        uint32_t c = 0;
        for (uint32_t s = 0; s < ns; s++) {
            const uint32_t e = tb.entries[tr.off + s];
            if (!e) continue;
            for (uint32_t q = first[e - 1]; q < first[e - 1] + count[e - 1]; q++, c++) {
                const uint32_t* cr = chips + 8u * c;
                float fb[4];
                memcpy(fb, cr + 4, 16);
                const pip::Box& bx = gb.geom_bbox[q];
                bool ok = cr[0] == meta[q] && cr[2] == q && cr[3] == s;
                if (!(meta[q] & 1u) && bx.minx <= bx.maxx)
                    ok = ok && fb[0] <= bx.minx && fb[1] <= bx.miny && fb[2] >= bx.maxx && fb[3] >= bx.maxy;
                const uint32_t vc = cr[1] >> 16;
                if (!(meta[q] & 1u) && vc != binned::kImgGlobal) {
                    const uint32_t v0 = gb.ring_start[gb.part_ring[gb.geom_part[q]]];
                    ok = ok && vc == gb.ring_start[gb.part_ring[gb.geom_part[q]] + 1] - v0;
                    for (uint32_t v = 0; ok && v < vc; v++)
                        ok = V[2 * ((cr[1] & 0xffffu) + v)] == gb.verts[v0 + v].x &&
                             V[2 * ((cr[1] & 0xffffu) + v) + 1] == gb.verts[v0 + v].y;
                }
                bad += !ok;
            }
        }
        bad += c != nc;
        // random points of the tile (and on its edges): listed chips cover every envelope holding them
        const int ti = (int)(t % g.nx), tj = (int)(t / g.nx);
        std::vector<std::pair<double, double>> pts;
        for (long k = 0; k < pts_per_tile; k++) {
            double ux = U(rng), uy = U(rng);
            if (k % 8 == 0) ux = 0.0;
            if (k % 8 == 1) uy = 0.0;
            pts.push_back({g.x0 + (ti + ux) / g.sx, g.y0 + (tj + uy) / g.sy});
        }
        for (uint32_t cc = 0; cc < nc; cc++) {  // envelope corners and edge midpoints
            const pip::Box& bx = gb.geom_bbox[chips[8u * cc + 2]];
            if (!(bx.minx <= bx.maxx)) continue;
            const double xs[3] = {bx.minx, 0.5 * (bx.minx + bx.maxx), bx.maxx};
            const double ys[3] = {bx.miny, 0.5 * (bx.miny + bx.maxy), bx.maxy};
            for (double px : xs)
                for (double py : ys) pts.push_back({px, py});
        }
        for (const auto& pt : pts) {
            const double x = pt.first, y = pt.second;
            if (tiles::tile_of(g, tb.tile_idx.data(), x, y) != code) continue;  // (rounding off the tile)
            const double fx = (x - g.x0) * g.sx, fy = (y - g.y0) * g.sy;
            const int gx = std::min((int)((fx - (double)(int)fx) * (double)G), G - 1);
            const int gy = std::min((int)((fy - (double)(int)fy) * (double)G), G - 1);
            const int cell = gy * G + gx;
            std::vector<uint16_t> lst(rl + rl[cell], rl + rl[cell + 1]);
            for (uint32_t cc = 0; cc < nc; cc++) {
                const uint32_t q = chips[8u * cc + 2];
                const pip::Box& bx = gb.geom_bbox[q];
                const bool holds = (meta[q] & 1u) || (x >= bx.minx && x <= bx.maxx && y >= bx.miny && y <= bx.maxy);
                if (holds && std::find(lst.begin(), lst.end(), (uint16_t)cc) == lst.end()) bad++;
            }
            checked++;
        }
    }
    printf("%zu %ld %ld %ld\n", tb.recs.size(), imaged, checked, bad);
    return 0;
}
