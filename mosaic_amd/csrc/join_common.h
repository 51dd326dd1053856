// Shared by the join kernels of mosaic_hip.hip and the stream kernels of join_stream.hip: the
// chip-hash entry, the join arguments, the per-wave mixed-row stage and the stream kernels' argument
// blocks and LDS helpers.  Device code and plain structs only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bng_device.h"
#include "pip_device.h"
#include "raster.h"
#include "tiles.h"

using namespace mosaic;

// ------------------------------------------------------------------------------------------------
// device-side data structures
static const int64_t kEmptyKey = INT64_MIN;

struct HashEntry {  // 16 bytes: one dwordx4 load per probe
    int64_t key;
    uint32_t first;
    uint32_t count;
};

__host__ __device__ inline uint64_t mix64(uint64_t h) {
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdULL;
    h ^= h >> 33;
    h *= 0xc4ceb9fe1a85ec53ULL;
    h ^= h >> 33;
    return h;
}

struct JoinArgs {
    const double* x;
    const double* y;
    const uint8_t* valid;
    int64_t n;
    int res, jdk;
    const HashEntry* table;
    uint64_t mask;
    const uint32_t* chip_meta;  // (polygon_key << 1) | is_core, in table order
    const raster::ChipHdr* hdr;     // per chip: envelope + ray-parity raster (raster.h)
    const raster::CellRec* cells;   // raster cells
    const pip::Edge* rast_edges;    // raster cell segment lists
    uint32_t lane_edges;            // cell lists up to this long are evaluated by the owning lane
    pip::GeomStore store;       // geometry g == chip g (table order)
    tiles::Grid tgrid;                // tile directory (tiles.h); tile_idx == nullptr: none
    const uint32_t* tile_idx;
    const tiles::TileRec* tile_rec;
    const uint32_t* tile_ent;
    tiles::PointRaster praster;       // point raster (tiles.h); praster.sub == nullptr: none
    const uint32_t* bng_cells;        // BNG dense cell table (k_join_stream_bng); nullptr: none
    const uint16_t* bng_leaf;         // its leaf blocks (C x C codes per border cell)
    int32_t bng_e0, bng_n0, bng_ne, bng_nn, bng_div, bng_C;
    int32_t bng_wedge;                // k_join_mixed_bng answers wedge sub-cells first (tiles.h)
    int64_t row_lo;                   // k_join_stream / k_join_mixed: rows [row_lo, n)
    uint32_t* mixq;                   // rows (- row_lo) in mixed raster cells, dense, in
    unsigned long long* mixq_count;   //   mixq[0 .. *mixq_count)
    unsigned long long* counts;  // [n_polygons]
    int n_polygons;
    unsigned long long* amb_queue;  // rows for the exact H3 pass
    unsigned long long* amb_count;
    unsigned long long amb_cap;
    // tiled_cell: rows the fast path cannot certify are answered in place with h3_exact (counted
    // in amb_count, not queued) -- k_join_mixed behind a stream kernel, so no exact pass follows
    int exact_inline = 0;
    long long* pair_row;
    int* pair_key;
    unsigned long long* pair_count;
    long long pair_cap;
    unsigned long long* tests;  // (point, border chip) contains evaluations
    unsigned int* flags;        // bit 0: NaN seen (BNG)
    // k_join_h3_exact's view of the points: queued row q's coordinates are x[q * cstride],
    // y[q * cstride] and its source row rowmap[q * cstride] (rowmap == nullptr: q itself) -- the
    // binned join (join_binned.hip) queues positions in its sorted (x, y[, row]) records
    int32_t cstride;
    const long long* rowmap;
};

// Count modes of the join kernels' hits (template argument CM; a bool true / false reads as 1 / 0):
// global atomics, the workgroup's LDS count array (n_polygons <= kLdsCountsMax), or a per-wave LDS
// hash of (key, count) flushed with one global atomic per distinct key (k_join_binned: many
// polygons, but the few keys of a tile's points).
static const int kCountGlobal = 0, kCountLds = 1, kCountWaveHash = 2;
// k_join_tiles only: per image chip LDS counters, added to the chip's polygon count when the run
// ends (hits on chips of the table: global atomics)
static const int kCountChips = 3;
static const int kWaveHashSlots = 256;  // per wave: keys[256] (key + 1, 0 = empty), counts[256], fill
static const int kWaveHashWords = 2 * kWaveHashSlots + 1;

__device__ inline void wave_hash_add(const JoinArgs& a, uint32_t* t, uint32_t key) {
    uint32_t h = (key * 0x9E3779B1u) >> 24;
    for (int p = 0; p < 16; p++) {
        const uint32_t s = (h + (uint32_t)p) & (kWaveHashSlots - 1);
        uint32_t k = t[s];
        if (k == 0) {
            k = atomicCAS(&t[s], 0u, key + 1u);
            if (k == 0) {
                atomicAdd(&t[2 * kWaveHashSlots], 1u);
                k = key + 1u;
            }
        }
        if (k == key + 1u) {
            atomicAdd(&t[kWaveHashSlots + s], 1u);
            return;
        }
    }
    atomicAdd(&a.counts[key], 1ULL);  // probe limit: straight to the global count
}

// Wave-uniform: adds the wave's hash to the global counts and empties it (always, or only when
// it is over half full).
__device__ inline void wave_hash_flush(const JoinArgs& a, uint32_t* t, bool always) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (!always && t[2 * kWaveHashSlots] < (uint32_t)(kWaveHashSlots / 2)) return;
    const int lane = (int)(threadIdx.x & 63);
    for (int s = lane; s < kWaveHashSlots; s += 64) {
        const uint32_t k = t[s];
        if (k) {
            atomicAdd(&a.counts[k - 1u], (unsigned long long)t[kWaveHashSlots + s]);
            t[s] = 0;
            t[kWaveHashSlots + s] = 0;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) t[2 * kWaveHashSlots] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One (row, key) pair: the count, and the pair itself for the pairs output.
template <int CM, bool PAIRS>
__device__ inline void emit_hit(const JoinArgs& a, int64_t row, uint32_t key, unsigned int* lds) {
    if (CM == kCountLds)
        atomicAdd(&lds[key], 1u);
    else if (CM == kCountWaveHash)
        wave_hash_add(a, lds, key);
    else
        atomicAdd(&a.counts[key], 1ULL);
    if (PAIRS) {
        unsigned long long idx = atomicAdd(a.pair_count, 1ULL);
        if ((long long)idx < a.pair_cap) {
            a.pair_row[idx] = row;
            a.pair_key[idx] = (int)key;
        }
    }
}

// Per-wave LDS stage of rows for the mixed-cell queue: rows are appended with a ballot, and the
// stage goes to the global queue in one atomic once >= 64 rows wait (a per-iteration atomic on one
// counter serialises the grid).  Wave-uniform calls.
__device__ inline void stage_push(uint32_t* wq, uint32_t& wn, bool mixed, uint32_t rowoff, unsigned long long lt_mask) {
    const unsigned long long mm = __ballot(mixed);
    if (mixed) wq[wn + __popcll(mm & lt_mask)] = rowoff;
    wn += (uint32_t)__popcll(mm);
}
__device__ inline void stage_flush(const JoinArgs& a, uint32_t* wq, uint32_t& wn, int lane, uint32_t min_rows) {
    if (wn < min_rows || wn == 0) return;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(a.mixq_count, (unsigned long long)wn);
    base = __shfl(base, 0, 64);
    for (uint32_t k = (uint32_t)lane; k < wn; k += 64) a.mixq[base + k] = wq[k];
    __builtin_amdgcn_wave_barrier();
    wn = 0;
}

struct StreamArgs {
    double x0, y0, sxC, syC;  // fine-cell coordinates g = (x - x0) sxC, (y - y0) syC (C per sub-block)
    double gxmax, gymax;      // clamp: NX C - 1, NY C - 1
    int32_t cs, qsh, tsh, qs;  // log2 C; cs + quad shift; cs + tile shift (sub-blocks per tile); quad shift
    int32_t qnx, tnx;         // quad-level entries per row, tiles per row
    int32_t n_quad_words, n_tiles;  // LDS copies: quad level (uint32 words), tile_base (if tb_lds)
    int32_t tb_lds;           // 1: tile_base in LDS; 0: gathered through its descriptor
    int32_t stage_words;      // per-wave mixed-row stage
    const uint32_t* quad;     // quad level, uint16 entries packed in uint32 words
    const uint32_t* tile_base;
    const uint16_t* csub;     // compact sub-block copies (PointRaster::sub + nx * ny)
    const uint16_t* blocks;   // line records and leaf blocks
    uint32_t csub_bytes, blocks_bytes, tile_base_bytes;
    // quad records (tiles::PointRaster::qrec_*), copied to LDS behind the quad level: 2 n_qrec mask
    // words, then the n_qrec uint16 codes; n_qrec_words >= 2 (index 0 is always readable)
    const uint32_t* qrec;
    int32_t n_qrec, n_qrec_words, qrl;
    // fixed-point fine-cell coordinates of k_join_stream_pipe (tiles::raster_code_fixed): g =
    // clamp(cvt_i32(fma(x, sxF, gx0F)), 0, gxmaxF) with F = tiles::kFixBits fraction bits
    double sxF, syF, gx0F, gy0F;
    int32_t gxmaxF, gymaxF, fix_ok;  // fix_ok: (NX C) 2^F and (NY C) 2^F fit an int32
    // leaf lines (tiles::PointRaster::tile_lbase / llines; nullptr: none): k_join_leaf only
    const uint32_t* tile_lbase;
    const tiles::LineRec* llines;
};
// per-wave mixed-row stage of the stream kernels (words): rows are appended one slot (<= 64 rows)
// at a time and flushed at >= 64
static const int kStageWords = 128;
// k_join_stream_cpt's per-wave compaction buffer (words): 64 slots x 3 words
static const int kCptBufWords = 192;
static const uint32_t kNoLoad = 0x7ffffff0u;  // out-of-range buffer offset (every table is < 2 GiB)
// cache-policy bits (aux) of the stream kernels' gathers: sub-block entries, line records, leaf
// codes, BNG sub-cell entries (build-time A/B knobs; 2 = nt)
// k_join_stream_pipe: groups of coordinates in flight ahead of the one being looked up (1 or 2)

typedef double v2d __attribute__((ext_vector_type(2)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

// A stream kernel's LDS fill: n words from global memory, 8 coalesced loads per thread in flight
// before the stores (a plain strided loop waits for each load in turn: ~40 serial round trips for
// a full quad level)
__device__ inline void lds_fill(uint32_t* dst, const uint32_t* __restrict__ src, int n) {
    const int nt = (int)blockDim.x;
    int k = (int)threadIdx.x;
    for (; k + 7 * nt < n; k += 8 * nt) {
        uint32_t v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = src[k + j * nt];
#pragma unroll
        for (int j = 0; j < 8; j++) dst[k + j * nt] = v[j];
    }
    for (; k < n; k += nt) dst[k] = src[k];
}

__device__ inline __amdgpu_buffer_rsrc_t stream_rsrc(const void* p, uint32_t bytes) {
    // wave-uniform inputs made provably uniform (no waterfall loops around the loads)
    const uint64_t u = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u), hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                             (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// a * b + c for a, b < 2^24 as one v_mad_u32_u24 (b wave-uniform).  Written out because the compiler
// turns __umul24(a, b) + c into v_mad_u64_u32 (a quarter-rate instruction) or a multiply, two
// shifts and an add when the sum is an address
__device__ inline uint32_t mad_u24(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    __asm__("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(c));
    return r;
}

// The LDS quad level's entry for fine cell (ixC, iyC), resolved through the quad's record when the
// point's sub-quad is uniform with the record's code (tiles::raster_code with use_quad, branch-free)
// (SH0: fraction bits below the fine-cell coordinates ixC, iyC -- 0, or kFixBits for the
// fixed-point coordinates of k_join_stream_pipe)
template <int SH0 = 0>
__device__ inline uint32_t quad_lookup(const StreamArgs& s, const uint16_t* quad, const uint32_t* qmask,
                                       const uint16_t* qcode, uint32_t ixC, uint32_t iyC) {
    const uint32_t q = quad[mad_u24(iyC >> (s.qsh + SH0), (uint32_t)s.qnx, ixC >> (s.qsh + SH0))];
    // q >= 0x8000 with record index q & 0x7fff < n_qrec, as one unsigned compare (q < 0x8000 wraps)
    const uint32_t r = q - 0x8000u;
    const bool rec = r < (uint32_t)s.n_qrec;
    const uint32_t sh = (uint32_t)(s.cs + s.qrl + SH0);
    const uint32_t b = (__builtin_amdgcn_ubfe(iyC, sh, 3u) << 3) | __builtin_amdgcn_ubfe(ixC, sh, 3u);
    const uint32_t rr = rec ? r : 0u;  // record 0 (mask words 0 and 1) is always readable
    const uint32_t w = qmask[2u * rr + (b >> 5)];
    const uint32_t c = qcode[rr];
    return (rec && __builtin_amdgcn_ubfe(w, b & 31u, 1u)) ? c : q;
}

// ---- BNG dense cell table (positive resolutions): BNGIndexSystem.pointToIndex
// (BNGIndexSystem.scala:277-291, 528-541) maps a point with 0 <= toInt(e), toInt(n) < 1e7 to the id
// of cell (toInt(e) / divisor, toInt(n) / divisor) -- one-to-one there, the two letters being the
// leading digits of those quotients (100000 is a multiple of every positive-resolution divisor).
// The host builds a dense table over the chip cells' cell range: 0 = no chip, kBngPure | (k + 1) =
// exactly one chip, a core chip of polygon k, kBngLeaf | block for other cells (below).  One
// L2-resident gather per point (two in border cells) decides all but the rows in mixed sub-cells
// (and rows outside that integer range), which go to the mixed queue and k_join_mixed_bng (the
// generic point_to_index + probe + chip loop).
// Border cells carry kBngLeaf | base: C x C sub-cell entries at leaf[base] (the H3 point raster's
// codes, tiles_build.cpp bng_leaf_blocks) -- a code, kMixed (the row goes to the mixed queue) or
// kSubBlock | kLineBit | n: the sub-cell is split by one straight chip edge, LineRec n of the cell at
// leaf[base - 8 (n + 1)] decides the point from its offset in the sub-cell.  A dense sub-block level
// (per cell one code per 4 x 4 group of sub-cells, or kSubBlock: read the leaf code) sits beside.
static const uint32_t kBngPure = 0x80000000u, kBngLeaf = 0x40000000u;
static const uint32_t kBngLdsGather = 0xFFu;
struct BngStreamArgs {
    int32_t e0, n0, ne, nn, C;
    double inv_div, div, f;  // 1 / divisor (rounded), divisor, C / divisor
    int32_t idiv;            // divisor
    float ff;                // C / divisor (f32)
    const uint32_t* cells;
    const uint16_t* leaf;
    uint32_t cells_bytes, leaf_bytes;
    const uint32_t* lcell;   // LDS cell level (bytes packed in words); nullptr / lcell_words == 0: none
    int32_t lcell_words, lsh, lnx;
    const uint16_t* lvl;     // sub-block levels: cell index i's at lvl[i lvl_stride] (tiles.h
    uint32_t lvl_bytes;      // bng_level_code), lvl_cb groups of 4 x 4 sub-cells per row; only
    int32_t lvl_stride, lvl_cb;  // k_join_stream_bng_cpt reads them
};

// The stream kernels (join_stream.hip), by template arguments: the host picks one and launches it
// with hipLaunchKernel.  pipe: k_join_stream_pipe (needs vec); else k_join_stream<lds, pairs, vec>.
const void* stream_kernel_h3(int pipe, bool lds, bool pairs, bool vec);
// k_join_leaf<lds, pairs> (join_stream.hip): the mixed queue's leaf-line rows, before k_join_mixed
const void* leaf_kernel(bool lds, bool pairs);
const void* stream_kernel_bng(bool lds, bool pairs, bool vec, bool cpt);  // cpt: k_join_stream_bng_cpt (needs vec)
