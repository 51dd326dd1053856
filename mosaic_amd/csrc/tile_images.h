// Per-tile chip images of the binned join (join_binned.hip k_join_tiles): layout and the host
// builder.  Host-compilable (tests/native/tile_images_check.cpp builds and checks them on the CPU).
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "pip_device.h"
#include "tiles.h"

namespace binned {
using namespace mosaic;

// ---- per-tile chip images (the LDS tiles of k_join_tiles)
// One image per tile record, copied whole into a workgroup's LDS for the sorted points of that
// tile: its window's chip ranges, per chip (meta, geometry reference, hexagon, f32 envelope
// rounded outwards), an envelope raster, and the rings of its one-ring border chips.  Layout
// (32-bit words):
//   [0] n_slots | n_chips << 16   [1] n_verts   [2] chip word offset   [3] vertex word offset
//   [4] envelope-raster word offset   [5..7] 0
//   [8 ..] slot_first: n_slots + 1 uint16 (chip index range of window slot s: [first[s], first[s+1]))
//   envelope raster: kImgRaster^2 + 1 uint16 list offsets, then the lists (uint16 chip indices):
//     cell (gx, gy) of the tile's kImgRaster x kImgRaster split lists every chip whose f64 envelope
//     meets it (core chips: every cell), so a point tests only the chips listed for its cell
//   chips (at a multiple of 4 words): 8 words each -- meta (polygon_key << 1 | is_core), vinfo
//     (vertex offset | count << 16; count 0: no geometry (core chip), kImgGlobal: tested from the
//     global geometry store), global chip index, window slot of its hexagon, f32 minx, miny, maxx,
//     maxy (outward rounded)
//   vertices (at a multiple of 4 words): double2, ring after ring (closed)
// A point's raster cell is computed from its grid position exactly as its tile is
// (tiles::tile_of): f = (x - x0) sx, cell floor((f - floor(f)) kImgRaster); the builder maps
// envelope corners through the same arithmetic, which is monotone, so a point inside an envelope
// lands in a cell that lists the chip.
static const uint32_t kImgCapWords = 5120;     // 20 KB of LDS per workgroup: 4 workgroups per CU
static const uint32_t kImgHdrWords = 8;
static const int kImgRaster = 16;
static const uint32_t kNoImage = 0xFFFFFFFFu;  // the record's chip records do not fit: generic path
static const uint32_t kImgGlobal = 0xFFFFu;
struct ImageSource {
    const tiles::TileRec* recs;
    size_t n_recs;
    tiles::Grid grid;
    const uint32_t* tile_idx;    // per tile: kSkip, kFull or record + 2
    const uint32_t* entries;     // window entries: chip-table slot + 1 (0: no chips)
    const uint32_t* slot_first;  // per chip-table slot: first chip, chip count
    const uint32_t* slot_count;
    const uint32_t* meta;
    pip::GeomStore store;
    int threads;
};

// ---- building the images (host)
inline float f32_down(double v) {
    float f = (float)v;
    if ((double)f > v) f = nextafterf(f, -INFINITY);
    return f;
}
inline float f32_up(double v) {
    float f = (float)v;
    if ((double)f < v) f = nextafterf(f, INFINITY);
    return f;
}

// image of record r (tile (ti, tj) of the grid): its words (empty: kNoImage)
inline void tile_image(const ImageSource& s, size_t r, int ti, int tj, std::vector<uint32_t>& w) {
    w.clear();
    const tiles::TileRec& tr = s.recs[r];
    const uint32_t wa = (tr.dims >> 8) & 0xfffu, wb = tr.dims >> 20, ns = wa * wb;
    if (ns == 0 || ns >= 0xffffu || ti < 0) return;
    std::vector<uint32_t> first(ns + 1, 0);
    uint32_t nc = 0;
    for (uint32_t k = 0; k < ns; k++) {
        first[k] = nc;
        const uint32_t e = s.entries[tr.off + k];
        if (e) nc += s.slot_count[e - 1];
    }
    first[ns] = nc;
    if (nc >= 0xffffu) return;
    // the envelope raster: per cell the chips whose envelope meets it (cell range of an envelope
    // through tile_of's arithmetic; see join_binned.h)
    const int G = kImgRaster;
    auto cell_of = [&](double v, double v0, double sc, int t) {
        const double f = (v - v0) * sc - (double)t;
        const double c = floor(f * G);
        return (int)std::min<double>(G - 1, std::max<double>(0.0, c));
    };
    std::vector<std::vector<uint16_t>> lists((size_t)G * G);
    uint32_t c = 0;
    for (uint32_t k = 0; k < ns; k++) {
        const uint32_t e = s.entries[tr.off + k];
        if (!e) continue;
        const uint32_t f0 = s.slot_first[e - 1], f1 = f0 + s.slot_count[e - 1];
        for (uint32_t g = f0; g < f1; g++, c++) {
            int x0 = 0, x1 = G - 1, y0 = 0, y1 = G - 1;
            if (!(s.meta[g] & 1u)) {
                const pip::Box& bx = s.store.geom_bbox[g];
                if (!(bx.minx <= bx.maxx && bx.miny <= bx.maxy)) continue;  // empty: never contains
                x0 = cell_of(bx.minx, s.grid.x0, s.grid.sx, ti);
                x1 = cell_of(bx.maxx, s.grid.x0, s.grid.sx, ti);
                y0 = cell_of(bx.miny, s.grid.y0, s.grid.sy, tj);
                y1 = cell_of(bx.maxy, s.grid.y0, s.grid.sy, tj);
            }
            for (int gy = y0; gy <= y1; gy++)
                for (int gx = x0; gx <= x1; gx++) lists[(size_t)gy * G + gx].push_back((uint16_t)c);
        }
    }
    uint32_t n_ent = 0;
    for (auto& l : lists) n_ent += (uint32_t)l.size();
    const uint32_t slot_words = (ns + 2) / 2;
    const uint32_t rast_off = kImgHdrWords + slot_words;
    const uint32_t rast_words = ((uint32_t)(G * G + 1) + n_ent + 1) / 2;
    const uint32_t chip_off = (rast_off + rast_words + 3u) & ~3u;
    const uint32_t vert_off = chip_off + 8u * nc;
    if (vert_off > kImgCapWords || (uint32_t)(G * G + 1) + n_ent >= 0xffffu) return;
    w.assign(vert_off, 0u);
    w[0] = ns | nc << 16;
    w[2] = chip_off;
    w[3] = vert_off;
    w[4] = rast_off;
    uint16_t* sf = (uint16_t*)(w.data() + kImgHdrWords);
    for (uint32_t k = 0; k <= ns; k++) sf[k] = (uint16_t)first[k];
    uint16_t* rl = (uint16_t*)(w.data() + rast_off);
    uint32_t pos = (uint32_t)(G * G + 1);
    for (int q = 0; q < G * G; q++) {
        rl[q] = (uint16_t)pos;
        for (uint16_t v : lists[(size_t)q]) rl[pos++] = v;
    }
    rl[G * G] = (uint16_t)pos;
    uint32_t nv = 0;
    c = 0;
    for (uint32_t k = 0; k < ns; k++) {
        const uint32_t e = s.entries[tr.off + k];
        if (!e) continue;
        const uint32_t f0 = s.slot_first[e - 1], f1 = f0 + s.slot_count[e - 1];
        for (uint32_t g = f0; g < f1; g++, c++) {
            uint32_t* cr = &w[chip_off + 8u * c];
            cr[0] = s.meta[g];
            cr[2] = g;
            cr[3] = k;
            const pip::Box& bx = s.store.geom_bbox[g];
            const float fb[4] = {f32_down(bx.minx), f32_down(bx.miny), f32_up(bx.maxx), f32_up(bx.maxy)};
            memcpy(cr + 4, fb, 16);
            if (s.meta[g] & 1u) continue;  // core: no geometry read
            cr[1] = kImgGlobal << 16;
            const uint32_t p0 = s.store.geom_part[g], p1 = s.store.geom_part[g + 1];
            if (p1 - p0 != 1) continue;
            const uint32_t r0 = s.store.part_ring[p0], r1 = s.store.part_ring[p0 + 1];
            if (r1 - r0 != 1) continue;
            const uint32_t v0 = s.store.ring_start[r0], v1 = s.store.ring_start[r0 + 1], m = v1 - v0;
            // (a ring of < 4 vertices stays global: pip::contains' own handling of degenerate rings)
            if (m < 4 || m >= kImgGlobal || vert_off + 4u * (nv + m) > kImgCapWords) continue;
            cr[1] = nv | m << 16;
            for (uint32_t v = 0; v < m; v++) {
                const pip::Vec2 q = s.store.verts[v0 + v];
                uint32_t qw[4];
                memcpy(qw, &q, 16);
                w.insert(w.end(), qw, qw + 4);
            }
            nv += m;
        }
    }
    w[1] = nv;
}

// words: the images back to back; off[r]: word offset of record r's image or kNoImage; max_words:
// the largest image.  False when the images would pass 2^32 words.
inline bool build_tile_images(const ImageSource& s, std::vector<uint32_t>& words, std::vector<uint32_t>& off,
                       uint32_t& max_words) {
    const size_t nr = s.n_recs;
    const int nt = std::max(1, std::min<int>(s.threads, (int)(nr / 64) + 1));
    std::vector<int> tile_of_rec(nr, -1);  // record -> tile (ti + tj nx)
    for (int64_t t = 0; t < (int64_t)s.grid.nx * s.grid.ny; t++)
        if (s.tile_idx[t] >= 2 && s.tile_idx[t] - 2 < nr) tile_of_rec[s.tile_idx[t] - 2] = (int)t;
    std::vector<std::vector<uint32_t>> part((size_t)nt);
    std::vector<std::vector<uint32_t>> part_off((size_t)nt);
    std::vector<uint32_t> part_max((size_t)nt, 0);
    auto work = [&](int t) {
        std::vector<uint32_t> w;
        auto& pw = part[(size_t)t];
        auto& po = part_off[(size_t)t];
        for (size_t r = nr * t / nt; r < nr * (t + 1) / nt; r++) {
            const int tile = tile_of_rec[r];
            tile_image(s, r, tile < 0 ? -1 : tile % s.grid.nx, tile < 0 ? -1 : tile / s.grid.nx, w);
            if (w.empty()) {
                po.push_back(kNoImage);
                continue;
            }
            po.push_back((uint32_t)pw.size());
            pw.insert(pw.end(), w.begin(), w.end());
            part_max[(size_t)t] = std::max(part_max[(size_t)t], (uint32_t)w.size());
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; t++) pool.emplace_back(work, t);
    work(0);
    for (auto& th : pool) th.join();
    size_t total = 0;
    for (auto& p : part) total += p.size();
    if (total >= (size_t)kNoImage) return false;
    words.clear();
    words.reserve(total);
    off.clear();
    off.reserve(nr);
    max_words = 0;
    for (int t = 0; t < nt; t++) {
        const uint32_t base = (uint32_t)words.size();
        for (uint32_t o : part_off[(size_t)t]) off.push_back(o == kNoImage ? kNoImage : o + base);
        words.insert(words.end(), part[(size_t)t].begin(), part[(size_t)t].end());
        max_words = std::max(max_words, part_max[(size_t)t]);
    }
    return true;
}

}  // namespace binned
