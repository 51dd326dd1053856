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
// A tile record's chips -- those of its window whose envelope meets the tile -- go into images that
// a workgroup copies whole into LDS for the sorted points they serve.  A record is split into
// 4^level parts (level 0, 1 or 2: the whole tile, 2 x 2 or 4 x 4 blocks of its envelope raster)
// when its chips do not fit one image with their rings; a part holds the chips whose envelope
// meets its block.  The sort key of a point is its part's image key (2 + image index: k_bin_cover),
// so the points of one image are contiguous.  Image layout (32-bit words):
//   [0] n_chips   [1] n_verts   [2] chip word offset   [3] vertex word offset   [4] raster word
//   offset   [5] record   [6] level | part << 8   [7] 0
//   envelope raster (at word 8): kImgRaster^2 + 1 uint16 list offsets, then the lists (uint16 chip
//     indices): cell (gx, gy) of the tile's kImgRaster x kImgRaster split lists every chip of the
//     image whose f64 envelope meets it (core chips: every cell); cells outside the part: empty
//   chips (at a multiple of 4 words): kImgChipWords each -- meta (polygon_key << 1 | is_core), vinfo
//     (vertex offset | count << 16; count 0: no geometry (core chip), kImgGlobal: tested from the
//     global geometry store), global chip index, window slot of its hexagon, f32 minx, miny, maxx,
//     maxy (outward rounded), a pad word
//   vertices (at a multiple of 4 words): float2 in the chip's f32 frame (ring_walk.h f32_frame:
//     float(v - envelope minimum)), ring after ring (closed); the image is padded to 4 words
// A point's raster cell is computed from its grid position exactly as its tile is
// (tiles::tile_of): f = (x - x0) sx, cell floor((f - floor(f)) kImgRaster); the builder maps
// envelope corners through the same arithmetic, which is monotone, so a point inside an envelope
// lands in a cell that lists the chip, and a chip whose envelope maps wholly below 0 or from 1 up
// on either axis holds no point of the tile (it is left out).
static const uint32_t kImgCapWords = 6144;  // 24 KB of LDS per workgroup (4 workgroups per CU)
static const uint32_t kImgHdrWords = 8;
static const int kImgRaster = 16;
static const uint32_t kImgRasterWords = (kImgRaster * kImgRaster + 2) / 2;  // the list offsets
// chip records: 8 words and a pad word (a stride of 9 words spreads the records of random chips over
// the 64 LDS banks; at 8 words every record started in one of 8 banks)
static const uint32_t kImgChipWords = 9;
static const uint32_t kImgMaxChips = (kImgCapWords - kImgHdrWords - kImgRasterWords) / kImgChipWords;
static const int kImgMaxLevel = 2;
// per tile record: kImgRaster^2 bits, bit q set when some chip's envelope meets envelope-raster cell
// q (all set for a record without images); k_bin_cover drops the points of clear cells, which no
// chip can hold, before the sort
static const int kImgCoverWords = kImgRaster * kImgRaster / 32;
static const uint32_t kNoImage = 0xFFFFFFFFu;  // the part's chip records do not fit: generic path
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
    uint32_t cap_words = kImgCapWords;  // image size limit (tests: smaller, to exercise the levels)
};
// the built images
struct ImageSet {
    std::vector<uint32_t> words;    // the images back to back
    std::vector<uint32_t> off;      // per image: word offset, or kNoImage
    std::vector<uint32_t> rec;      // per image: its tile record
    std::vector<uint32_t> rec_key;  // per record: first image index << 2 | level
    std::vector<uint32_t> cover;    // per record: kImgCoverWords
    std::vector<uint32_t> bin_map;  // per tile: kBinMapWords (k_bin_cover's one table)
    uint32_t max_words = 0;
    uint32_t levels[kImgMaxLevel + 1] = {0, 0, 0};  // records per level
};

// part of envelope-raster cell q = gy kImgRaster + gx at a level (k_bin_cover's key arithmetic)
MOSAIC_HD uint32_t image_part(int q, int level) {
    const int sh = 4 - level;  // (kImgRaster = 16 = 2^4)
    return (uint32_t)((((q >> 4) >> sh) << level) | ((q & 15) >> sh));
}

// k_bin_cover's (and k_join_tiles') per-point arithmetic, host-checked with adversarial inputs in
// tests/native/tile_images_check.cpp: the tile-index slot to read (0 off the grid: its code is then
// kSkip or kFull), and the envelope-raster cell q in [0, kImgRaster^2) (0 off the grid)
struct BinCell {
    int64_t slot;
    int q;
    bool in;
};
MOSAIC_HD BinCell bin_cell(const tiles::Grid& g, double x, double y) {
    const double fx = (x - g.x0) * g.sx, fy = (y - g.y0) * g.sy;
    BinCell c;
    c.in = fx >= 0.0 && fx < (double)g.nx && fy >= 0.0 && fy < (double)g.ny;
    const double sx = c.in ? fx : 0.0, sy = c.in ? fy : 0.0;  // (no conversion of an off-grid value)
    const int ix = (int)sx, iy = (int)sy;
    c.slot = (int64_t)iy * g.nx + ix;
    const int gx = (int)((sx - (double)ix) * (double)kImgRaster), gy = (int)((sy - (double)iy) * (double)kImgRaster);
    c.q = (gy < kImgRaster - 1 ? gy : kImgRaster - 1) * kImgRaster + (gx < kImgRaster - 1 ? gx : kImgRaster - 1);
    return c;
}
// the sort key of a point of tile code `code` (tiles::tile_of) in raster cell q; rk: its record's
// rec_key (ignored for codes < 2)
MOSAIC_HD uint32_t bin_key(uint32_t code, uint32_t rk, int q) {
    return code < 2u ? code : 2u + (rk >> 2) + image_part(q, (int)(rk & 3u));
}
// k_bin_cover's table, per tile of the grid (one cache-line-sized record, so a point's two reads
// share a line): [0] key word -- tiles::kSkip, tiles::kFull, or (2 + first image of the tile's
// record) << 2 | level -- and [1 ..] the record's cover bits (kFull: all set)
static const int kBinMapWords = 1 + kImgCoverWords;
// a point's key and whether it is kept, from its tile's key word kw and cover word cw of cell q
MOSAIC_HD uint32_t bin_map_key(uint32_t kw, int q) {
    return kw < 2u ? kw : (kw >> 2) + image_part(q, (int)(kw & 3u));
}
MOSAIC_HD bool bin_map_keep(uint32_t kw, uint32_t cw, int q) {
    return kw != tiles::kSkip && ((cw >> (q & 31)) & 1u);
}

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

// a chip of a record's window that may hold points of the tile: its cell range (inclusive)
struct TileChip {
    uint32_t g, slot;
    int x0, x1, y0, y1;
};

// the chips of record r (tile (ti, tj)) that may hold a point of the tile, in window order
inline void tile_chips(const ImageSource& s, size_t r, int ti, int tj, std::vector<TileChip>& out) {
    out.clear();
    const tiles::TileRec& tr = s.recs[r];
    const uint32_t wa = (tr.dims >> 8) & 0xfffu, wb = tr.dims >> 20, ns = wa * wb;
    const int G = kImgRaster;
    // f = (v - v0) sc - t, the point's (f - floor(f)) arithmetic (monotone in v)
    auto fpos = [&](double v, double v0, double sc, int t) { return (v - v0) * sc - (double)t; };
    auto cell = [&](double f) { return (int)std::min<double>(G - 1, std::max<double>(0.0, floor(f * G))); };
    for (uint32_t k = 0; k < ns; k++) {
        const uint32_t e = s.entries[tr.off + k];
        if (!e) continue;
        const uint32_t f0 = s.slot_first[e - 1], f1 = f0 + s.slot_count[e - 1];
        for (uint32_t g = f0; g < f1; g++) {
            TileChip c{g, k, 0, G - 1, 0, G - 1};
            if (!(s.meta[g] & 1u)) {
                const pip::Box& bx = s.store.geom_bbox[g];
                if (!(bx.minx <= bx.maxx && bx.miny <= bx.maxy)) continue;  // empty: never contains
                const double ax = fpos(bx.minx, s.grid.x0, s.grid.sx, ti), bxx = fpos(bx.maxx, s.grid.x0, s.grid.sx, ti);
                const double ay = fpos(bx.miny, s.grid.y0, s.grid.sy, tj), by = fpos(bx.maxy, s.grid.y0, s.grid.sy, tj);
                if (bxx < 0.0 || by < 0.0 || ax >= 1.0 || ay >= 1.0) continue;  // off the tile
                c.x0 = cell(ax);
                c.x1 = cell(bxx);
                c.y0 = cell(ay);
                c.y1 = cell(by);
            }
            out.push_back(c);
        }
    }
}

// image of cell block [bx0, bx1] x [by0, by1] of record r from its tile chips; false when it does
// not fit (w then holds nothing useful); *n_global: one-ring chips whose ring did not fit (those stay
// in the global store, as do multi-ring and multi-part chips)
inline bool block_image(const ImageSource& s, uint32_t r, uint32_t level_part, const std::vector<TileChip>& tc,
                        int bx0, int bx1, int by0, int by1, std::vector<uint32_t>& w, uint32_t* n_global) {
    const int G = kImgRaster;
    std::vector<uint32_t> sel;
    for (uint32_t k = 0; k < (uint32_t)tc.size(); k++)
        if (tc[k].x1 >= bx0 && tc[k].x0 <= bx1 && tc[k].y1 >= by0 && tc[k].y0 <= by1) sel.push_back(k);
    const uint32_t nc = (uint32_t)sel.size();
    if (nc > kImgMaxChips || kImgChipWords * nc > s.cap_words) return false;
    std::vector<std::vector<uint16_t>> lists((size_t)G * G);
    uint32_t n_ent = 0;
    for (uint32_t c = 0; c < nc; c++) {
        const TileChip& t = tc[sel[c]];
        for (int gy = std::max(t.y0, by0); gy <= std::min(t.y1, by1); gy++)
            for (int gx = std::max(t.x0, bx0); gx <= std::min(t.x1, bx1); gx++) {
                lists[(size_t)gy * G + gx].push_back((uint16_t)c);
                n_ent++;
            }
    }
    const uint32_t rast_off = kImgHdrWords;
    const uint32_t rast_words = ((uint32_t)(G * G + 1) + n_ent + 1) / 2;
    const uint32_t chip_off = (rast_off + rast_words + 3u) & ~3u;
    const uint32_t vert_off = (chip_off + kImgChipWords * nc + 3u) & ~3u;
    if (vert_off > s.cap_words || (uint32_t)(G * G + 1) + n_ent >= 0xffffu) return false;
    w.assign(vert_off, 0u);
    w[0] = nc;
    w[2] = chip_off;
    w[3] = vert_off;
    w[4] = rast_off;
    w[5] = r;
    w[6] = level_part;
    uint16_t* rl = (uint16_t*)(w.data() + rast_off);
    uint32_t pos = (uint32_t)(G * G + 1);
    for (int q = 0; q < G * G; q++) {
        rl[q] = (uint16_t)pos;
        for (uint16_t v : lists[(size_t)q]) rl[pos++] = v;
    }
    rl[G * G] = (uint16_t)pos;
    uint32_t nv = 0, glob = 0;
    for (uint32_t c = 0; c < nc; c++) {
        const uint32_t g = tc[sel[c]].g;
        uint32_t* cr = &w[chip_off + kImgChipWords * c];
        cr[0] = s.meta[g];
        cr[2] = g;
        cr[3] = tc[sel[c]].slot;
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
        if (m < 4 || m >= kImgGlobal) continue;
        if (vert_off + 2u * (nv + m) > s.cap_words) {
            glob++;
            continue;
        }
        cr[1] = nv | m << 16;
        for (uint32_t v = 0; v < m; v++) {  // the f32 walk's frame (ring_walk.h f32_frame)
            const pip::Vec2 q = s.store.verts[v0 + v];
            const float rel[2] = {(float)(q.x - (double)fb[0]), (float)(q.y - (double)fb[1])};
            uint32_t qw[2];
            memcpy(qw, rel, 8);
            w.insert(w.end(), qw, qw + 2);
        }
        nv += m;
    }
    w[1] = nv;
    w.resize((w.size() + 3u) & ~(size_t)3u, 0u);  // (whole 16-byte words: k_join_tiles copies uint4s)
    *n_global = glob;
    return true;
}

// the images of record r: the lowest level whose parts all fit with every ring (else the deepest
// level, parts that do not fit without an image); appended to parts (kNoImage: empty vector)
inline void record_images(const ImageSource& s, uint32_t r, int tile, std::vector<std::vector<uint32_t>>& parts,
                          int& level, uint32_t* cover) {
    for (int q = 0; q < kImgCoverWords; q++) cover[q] = 0xffffffffu;  // (no chips known: every cell may join)
    parts.clear();
    level = 0;
    const tiles::TileRec& tr = s.recs[r];
    const uint32_t wa = (tr.dims >> 8) & 0xfffu, wb = tr.dims >> 20;
    if (tile < 0 || wa * wb == 0 || wa * wb >= 0xffffu) {
        parts.emplace_back();
        return;
    }
    std::vector<TileChip> tc;
    tile_chips(s, r, tile % s.grid.nx, tile / s.grid.nx, tc);
    const int G = kImgRaster;
    for (int q = 0; q < kImgCoverWords; q++) cover[q] = 0u;
    for (const TileChip& t : tc)
        for (int gy = t.y0; gy <= t.y1; gy++)
            for (int gx = t.x0; gx <= t.x1; gx++) cover[(gy * G + gx) >> 5] |= 1u << ((gy * G + gx) & 31);
    for (level = 0; level <= kImgMaxLevel; level++) {
        const int np = 1 << level, bw = G >> level;
        parts.assign((size_t)np * np, std::vector<uint32_t>());
        bool all = true;
        for (int py = 0; py < np; py++)
            for (int px = 0; px < np; px++) {
                uint32_t glob = 0;
                auto& w = parts[(size_t)py * np + px];
                const bool ok = block_image(s, r, (uint32_t)level | (uint32_t)(py * np + px) << 8, tc, px * bw,
                                            px * bw + bw - 1, py * bw, py * bw + bw - 1, w, &glob);
                if (!ok) w.clear();
                all = all && ok && glob == 0;
            }
        if (all || level == kImgMaxLevel) return;
    }
}

// all records' images (host threads); false when the images would pass 2^32 words
inline bool build_tile_images(const ImageSource& s, ImageSet& out) {
    const size_t nr = s.n_recs;
    const int nt = std::max(1, std::min<int>(s.threads, (int)(nr / 64) + 1));
    std::vector<int> tile_of_rec(nr, -1);  // record -> tile (ti + tj nx)
    for (int64_t t = 0; t < (int64_t)s.grid.nx * s.grid.ny; t++)
        if (s.tile_idx[t] >= 2 && s.tile_idx[t] - 2 < nr) tile_of_rec[s.tile_idx[t] - 2] = (int)t;
    out.cover.assign(nr * kImgCoverWords, 0xffffffffu);
    std::vector<int> level(nr, 0);
    struct Part {
        std::vector<uint32_t> words, off, rec;
        uint32_t max = 0;
    };
    std::vector<Part> part((size_t)nt);
    auto work = [&](int t) {
        std::vector<std::vector<uint32_t>> imgs;
        Part& pt = part[(size_t)t];
        for (size_t r = nr * t / nt; r < nr * (t + 1) / nt; r++) {
            record_images(s, (uint32_t)r, tile_of_rec[r], imgs, level[r], out.cover.data() + r * kImgCoverWords);
            for (const auto& w : imgs) {
                pt.rec.push_back((uint32_t)r);
                if (w.empty()) {
                    pt.off.push_back(kNoImage);
                    continue;
                }
                pt.off.push_back((uint32_t)pt.words.size());
                pt.words.insert(pt.words.end(), w.begin(), w.end());
                pt.max = std::max(pt.max, (uint32_t)w.size());
            }
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; t++) pool.emplace_back(work, t);
    work(0);
    for (auto& th : pool) th.join();
    size_t total = 0, n_img = 0;
    for (auto& p : part) {
        total += p.words.size();
        n_img += p.off.size();
    }
    if (total >= (size_t)kNoImage || n_img >= ((size_t)1 << 29)) return false;
    out.words.clear();
    out.words.reserve(total);
    out.off.clear();
    out.off.reserve(n_img);
    out.rec.clear();
    out.rec.reserve(n_img);
    out.max_words = 0;
    for (int t = 0; t < nt; t++) {
        const uint32_t base = (uint32_t)out.words.size();
        for (uint32_t o : part[(size_t)t].off) out.off.push_back(o == kNoImage ? kNoImage : o + base);
        out.rec.insert(out.rec.end(), part[(size_t)t].rec.begin(), part[(size_t)t].rec.end());
        out.words.insert(out.words.end(), part[(size_t)t].words.begin(), part[(size_t)t].words.end());
        out.max_words = std::max(out.max_words, part[(size_t)t].max);
    }
    // per record: first image index << 2 | level (images are in record order)
    out.rec_key.assign(nr, 0u);
    for (int l = 0; l <= kImgMaxLevel; l++) out.levels[l] = 0;
    for (size_t k = n_img; k-- > 0;) out.rec_key[out.rec[k]] = (uint32_t)k << 2;
    for (size_t r = 0; r < nr; r++) {
        out.rec_key[r] |= (uint32_t)level[r];
        out.levels[level[r]]++;
    }
    const int64_t ntiles = (int64_t)s.grid.nx * s.grid.ny;
    out.bin_map.assign((size_t)ntiles * kBinMapWords, 0u);
    for (int64_t t = 0; t < ntiles; t++) {
        uint32_t* m = &out.bin_map[(size_t)t * kBinMapWords];
        const uint32_t code = s.tile_idx[t];
        if (code >= 2 && code - 2 < nr) {
            const uint32_t r = code - 2;
            m[0] = (2u + (out.rec_key[r] >> 2)) << 2 | (out.rec_key[r] & 3u);
            for (int q = 0; q < kImgCoverWords; q++) m[1 + q] = out.cover[(size_t)r * kImgCoverWords + q];
        } else {
            m[0] = code == tiles::kFull ? tiles::kFull : tiles::kSkip;
            for (int q = 0; q < kImgCoverWords; q++) m[1 + q] = m[0] == tiles::kFull ? ~0u : 0u;
        }
    }
    return true;
}

}  // namespace binned
