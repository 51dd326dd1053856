// Host interface of the binned chip join (join_binned.hip): scratch owned by a thread state of
// mosaic_hip.hip and the one launcher run_join calls.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "join_common.h"

namespace binned {

// sorted point values: coordinates, plus the source row for the pairs output
struct Pt {
    double x, y;
};
struct PtRow {
    double x, y;
    long long row;
};
__host__ __device__ inline void set_row(Pt&, int64_t) {}
__host__ __device__ inline void set_row(PtRow& p, int64_t r) { p.row = (long long)r; }
__host__ __device__ inline int64_t row_of(const Pt&, int64_t i) { return i; }
__host__ __device__ inline int64_t row_of(const PtRow& p, int64_t) { return (int64_t)p.row; }
inline const long long* row_map(const Pt*) { return nullptr; }
inline const long long* row_map(const PtRow* p) { return &p->row; }

struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
    hipError_t reserve(size_t n) {
        if (n <= bytes) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        hipError_t e = hipMalloc(&p, n);
        if (e == hipSuccess) bytes = n;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

struct Scratch {
    Buf keys[2], vals[2], temp, n_skip;
    JoinArgs exact_args;  // the join's arguments as the exact-H3 pass must read them (sorted points)
    size_t held() const {
        return keys[0].bytes + keys[1].bytes + vals[0].bytes + vals[1].bytes + temp.bytes + n_skip.bytes;
    }
    void release() {
        for (Buf* b : {&keys[0], &keys[1], &vals[0], &vals[1], &temp, &n_skip}) b->release();
    }
};

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
    const uint32_t* tile_idx;  // per tile: kSkip, kFull or record + 2
    const uint32_t* entries;
    const HashEntry* table;
    const uint32_t* meta;
    pip::GeomStore store;
    int threads;
};
// words: the images back to back; off[r]: word offset of record r's image or kNoImage; max_words:
// the largest image.  False when the images would pass 2^32 words.
bool build_tile_images(const ImageSource& s, std::vector<uint32_t>& words, std::vector<uint32_t>& off,
                       uint32_t& max_words);

struct Images {
    const uint32_t* words = nullptr;  // nullptr: no images (k_join_binned runs)
    const uint32_t* off = nullptr;
    uint32_t max_words = 0;
};

// Rows [lo, n) of a.x / a.y: key, sort, join (enqueued on stream).  max_code: the largest tile code
// (tile records + 1).  s.exact_args receives the JoinArgs the exact-H3 pass runs with.
hipError_t join(const JoinArgs& a, int64_t lo, int64_t n, uint32_t max_code, bool lds_counts, int n_cu,
                const Images& img, Scratch& s, hipStream_t stream);

}  // namespace binned
