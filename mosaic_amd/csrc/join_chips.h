// The chip loop shared by the join kernels of mosaic_hip.hip and join_binned.hip: the hash probe,
// the per-chip ray-parity raster walk with its wave-cooperative segment evaluation (raster_chips),
// and the tile path from a point's tile record to its chips (tiled_cell).  Device code only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "h3_device.h"
#include "join_common.h"
#include "pip_coop.h"
#include "pip_device.h"
#include "raster.h"
#include "tiles.h"

using namespace mosaic;

template <bool LDS_COUNTS, bool PAIRS>
__device__ inline void join_point(const JoinArgs& a, int64_t row, double x, double y, int64_t cell, unsigned int* lds,
                                  unsigned int& tests) {
    if (cell == kEmptyKey) return;
    uint64_t slot = mix64((uint64_t)cell) & a.mask;
    HashEntry e;
    while (true) {
        e = a.table[slot];
        if (e.key == cell) break;
        if (e.key == kEmptyKey) return;
        slot = (slot + 1) & a.mask;
    }
    for (uint32_t c = e.first; c < e.first + e.count; c++) {
        uint32_t meta = a.chip_meta[c];
        bool hit = meta & 1u;
        if (!hit) {
            tests++;
            hit = pip::contains(a.store, c, x, y);
        }
        if (hit) {
            uint32_t key = meta >> 1;
            if (LDS_COUNTS)
                atomicAdd(&lds[key], 1u);
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
    }
}

template <bool LDS_COUNTS>
__device__ inline void counts_init(const JoinArgs& a, unsigned int* lds) {
    if (LDS_COUNTS) {
        for (int k = threadIdx.x; k < a.n_polygons; k += blockDim.x) lds[k] = 0;
        __syncthreads();
    }
}

template <bool LDS_COUNTS>
__device__ inline void counts_flush(const JoinArgs& a, unsigned int* lds, unsigned int tests) {
    // one wave-level add for the test counter
    for (int off = 32; off > 0; off >>= 1) tests += __shfl_down(tests, off, 64);
    if ((threadIdx.x & 63) == 0 && tests) atomicAdd(a.tests, (unsigned long long)tests);
    if (LDS_COUNTS) {
        __syncthreads();
        for (int k = threadIdx.x; k < a.n_polygons; k += blockDim.x)
            if (lds[k]) atomicAdd(&a.counts[k], (unsigned long long)lds[k]);
    }
}

__device__ inline void probe(const JoinArgs& a, int64_t cell, uint32_t& first, uint32_t& end) {
    first = end = 0;
    if (cell == kEmptyKey) return;
    uint64_t slot = mix64((uint64_t)cell) & a.mask;
    while (true) {
        HashEntry e = a.table[slot];
        if (e.key == cell) {
            first = e.first;
            end = e.first + e.count;
            return;
        }
        if (e.key == kEmptyKey) return;
        slot = (slot + 1) & a.mask;
    }
}

// Work items of the wave-cooperative chip evaluation (raster_chips): a general chip (multi-ring /
// multi-part) or a raster cell's segment list.
static const uint32_t kGeneralItem = 0xffffffffu;

struct SlabItem {
    double x, y;
    uint32_t e0, m;
};

// ---- raster chip loop: per border chip one ray-parity raster lookup
// (raster.h); pure cells are decided by the lookup, short cell lists by the owning lane, and only
// long lists and general (multi-ring / multi-part) chips go to the wave-cooperative evaluation.

// Walks this lane's chips from `cur`: core chips are accepted, border chips decided by the raster
// where the lane can; stops at the first chip that needs the wave (cur < end on return, with its
// item (e0, m, par); m == kGeneralItem for general chips).
template <int CM, bool PAIRS>
__device__ inline void advance_raster(const JoinArgs& a, int64_t row, uint32_t& cur, uint32_t end, double x, double y,
                                      unsigned int& tests, uint32_t& e0, uint32_t& m, uint32_t& par,
                                      unsigned int* lds) {
    for (; cur < end; cur++) {
        const uint32_t meta = a.chip_meta[cur];
        if (meta & 1u) {
            emit_hit<CM, PAIRS>(a, row, meta >> 1, lds);
            continue;
        }
        tests++;
        const raster::ChipHdr h = a.hdr[cur];
        if (pip::box_excludes(h.box, x, y)) continue;
        if (h.cell_base == raster::kNoRaster) {
            e0 = 0;
            m = kGeneralItem;
            par = 0;
            return;
        }
        const raster::CellRec rec = a.cells[raster::cell_index(h, x, y)];
        if (rec.m > a.lane_edges) {
            e0 = rec.word >> 1;
            m = rec.m;
            par = rec.word & 1u;
            return;
        }
        if (raster::cell_contains(rec, a.rast_edges, x, y)) emit_hit<CM, PAIRS>(a, row, meta >> 1, lds);
    }
}

// The chips [cur, end) of every lane's point, raster strategy: lane-local where the raster decides,
// wave-cooperative for long segment lists and general chips.  Wave-uniform call.
template <int CM, bool PAIRS>
__device__ inline void raster_chips(const JoinArgs& a, int64_t i, uint32_t cur, uint32_t end, double x, double y,
                                    unsigned int& tests, unsigned int* lds, SlabItem* items) {
    const int lane = (int)(threadIdx.x & 63);
    const unsigned long long lt_mask = (1ULL << lane) - 1ULL;
    uint32_t e0 = 0, m = 0, par = 0;
    advance_raster<CM, PAIRS>(a, i, cur, end, x, y, tests, e0, m, par, lds);
    unsigned long long pending = __ballot(cur < end);
    while (pending) {
        int s0 = __ffsll(pending) - 1;
        uint32_t m0 = pip::readlane_u32(m, s0);
        if (m0 > 32) {
            // one item for the whole wave: general chips, or cell lists over 32 records
            double qx = pip::readlane_f64(x, s0), qy = pip::readlane_f64(y, s0);
            bool hit;
            if (m0 == kGeneralItem) {
                hit = pip::coop_contains(a.store, pip::readlane_u32(cur, s0), qx, qy);
            } else {
                uint32_t q0 = pip::readlane_u32(e0, s0);
                unsigned long long onm = 0;
                int cross = (int)pip::readlane_u32(par, s0);
                for (uint32_t b = 0; b < m0; b += 64) {
                    bool on = false, cr = false;
                    if (b + lane < m0) pip::edge_rec_flags(a.rast_edges[q0 + b + lane], qx, qy, on, cr);
                    onm |= __ballot(on);
                    cross += __popcll(__ballot(cr));
                }
                hit = onm == 0 && (cross & 1);
            }
            if (lane == s0) {
                if (hit) emit_hit<CM, PAIRS>(a, i, a.chip_meta[cur] >> 1, lds);
                cur++;
                advance_raster<CM, PAIRS>(a, i, cur, end, x, y, tests, e0, m, par, lds);
            }
        } else {
            const int G = m0 <= 4 ? 4 : (m0 <= 8 ? 8 : (m0 <= 16 ? 16 : 32));
            const int cap = 64 / G;
            bool cand = cur < end && m <= (uint32_t)G;
            unsigned long long cmask = __ballot(cand);
            int rank = __popcll(cmask & lt_mask);
            bool chosen = cand && rank < cap;
            if (chosen) {
                SlabItem it;
                it.x = x;
                it.y = y;
                it.e0 = e0;
                it.m = m;
                items[rank] = it;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            int ng = __popcll(cmask);
            ng = ng < cap ? ng : cap;
            int k = lane / G, j = lane - k * G;
            bool on = false, cr = false;
            if (k < ng) {
                SlabItem it = items[k];
                if ((uint32_t)j < it.m) pip::edge_rec_flags(a.rast_edges[it.e0 + j], it.x, it.y, on, cr);
            }
            unsigned long long onm = __ballot(on), crm = __ballot(cr);
            if (chosen) {
                const unsigned long long gm = (G == 32) ? 0xffffffffULL : ((1ULL << G) - 1ULL);
                unsigned long long om = (onm >> (rank * G)) & gm, xm = (crm >> (rank * G)) & gm;
                if (om == 0 && ((__popcll(xm) + par) & 1)) emit_hit<CM, PAIRS>(a, i, a.chip_meta[cur] >> 1, lds);
                cur++;
                advance_raster<CM, PAIRS>(a, i, cur, end, x, y, tests, e0, m, par, lds);
            }
            __builtin_amdgcn_wave_barrier();
        }
        pending = __ballot(cur < end);
    }
}

// ---- tiled variant (default for H3 chip tables with a tile directory, tiles.h).  With the point
// raster (RASTER), one or two L2-resident lookups give the whole answer of most points (no pair, or
// one pair with a known polygon key).  Otherwise, or for raster cells marked mixed, the point's
// tile decides whether it can join at all; points that can are compacted per wave in LDS (so the
// lanes of a wave all carry work), then get their hexagon from the tile's face and window (no
// index arithmetic, no hash probe) and go through the raster chip loop.
static const int kQueue = 128;  // per-wave LDS queue (entries)

struct TileQueue {
    double x[kQueue], y[kQueue];
    long long row[kQueue];
    uint32_t code[kQueue];
};

// H3's own cell of a point the fast path cannot certify (a call, so the exact path's registers do
// not count against the kernels that rarely take it)
__device__ __noinline__ int64_t exact_cell(double x, double y, int res, int jdk) {
    return (int64_t)h3::h3_exact(h3::to_radians(y, jdk), h3::to_radians(x, jdk), res);
}

// Chips of one queued point: tile path (certified hexagon -> window slot) or the generic
// fast path + probe (kFull tiles, window misses).  Uncertified points go to the exact queue, or
// (exact_inline) get h3_exact's cell here.
__device__ inline void tiled_cell(const JoinArgs& a, int64_t i, double x, double y, uint32_t code, uint32_t& cur,
                                  uint32_t& end) {
    cur = end = 0;
    int64_t cell;
    if (code >= 2) {
        const tiles::TileRec r = a.tile_rec[code - 2];
        const int face = (int)(r.dims & 0xffu);
        const int wa = (int)((r.dims >> 8) & 0xfffu), wb = (int)(r.dims >> 20);
        double px, py, pz, vx, vy, best;
        h3::fast_unit(y, x, &px, &py, &pz);
        h3::fast_plane(px, py, pz, face, a.res, &vx, &vy, &best);
        int ba, bb;
        if (!h3::fast_hex(vx, vy, a.res, &ba, &bb)) {
            unsigned long long q = atomicAdd(a.amb_count, 1ULL);
            if (a.exact_inline) {
                probe(a, exact_cell(x, y, a.res, a.jdk), cur, end);
            } else if (q < a.amb_cap) {
                a.amb_queue[q] = (unsigned long long)i;
            }
            return;
        }
        const int ra = ba - r.a0, rb = bb - r.b0;
        if ((unsigned)ra < (unsigned)wa && (unsigned)rb < (unsigned)wb) {
            const uint32_t e = a.tile_ent[r.off + (uint32_t)(ra * wb + rb)];
            if (e) {
                const HashEntry he = a.table[e - 1];
                cur = he.first;
                end = he.first + he.count;
            }
            return;
        }
        cell = (int64_t)h3::face_axial_to_h3(face, ba, bb, a.res);
    } else {
        bool amb;
        cell = (int64_t)h3::h3_fast(y, x, a.res, &amb);
        if (amb) {
            unsigned long long q = atomicAdd(a.amb_count, 1ULL);
            if (!a.exact_inline) {
                if (q < a.amb_cap) a.amb_queue[q] = (unsigned long long)i;
                return;
            }
            cell = exact_cell(x, y, a.res, a.jdk);
        }
    }
    probe(a, cell, cur, end);
}

