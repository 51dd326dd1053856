// The binned chip join (north_star kernel (c) for border-chip-heavy chip tables: SURVEY.md §7.3-4,
// C4 = building footprints chipped at H3 res 11, ~2.4 chips per cell, every chip a border chip).
//
// The unbinned tiled join (k_join_tiled) walks, per point in input order, a chain of dependent
// gathers into a multi-GB table (tile record -> window entry -> hash entry -> per chip: meta, header,
// raster cell, segments); uniform input order makes every link an HBM miss.  Here the points are
// first sorted by their tile code (tiles::tile_of: kSkip, kFull or tile record + 2) so that the
// 64 points of a wave and the waves of a workgroup share a tile: its window, hash entries, chip
// headers, rasters and rings are read once from HBM and then hit the CU's L1 / the XCD's L2.
//   k_bin_keys     one lane per point: tile code -> key, (x, y[, row]) -> value; counts kSkip rows
//   (hipcub radix sort of (key, value) over the key's significant bits)
//   k_join_binned  contiguous chunks of the sorted points per wave; kSkip rows (sorted first) are
//                  not visited; tile path + chip loop of join_chips.h; counts through a per-wave
//                  LDS hash of (key, count) when there are too many polygons for an LDS array
// The exact-H3 queue carries sorted positions; k_join_h3_exact reads their coordinates (and, for
// pairs, their source rows) through JoinArgs::cstride / rowmap.
#include <hip/hip_runtime.h>
#include <string.h>

#include <hipcub/hipcub.hpp>
#include <rocprim/rocprim.hpp>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "join_binned.h"
#include "join_chips.h"
#include "ring_walk.h"

using namespace mosaic;

template <class P>
__device__ __forceinline__ void bin_one(const JoinArgs& a, int64_t i, int64_t lo, double x, double y, uint32_t* keys, P* pts,
                                        unsigned int& skipped) {
    const uint32_t code = tiles::tile_of(a.tgrid, a.tile_idx, x, y);
    keys[i - lo] = code;
    P p;
    p.x = x;
    p.y = y;
    binned::set_row(p, i);
    pts[i - lo] = p;
    skipped += code == tiles::kSkip;
}

// VEC: two consecutive points per lane and step (16-byte loads of x and y; lo even and the columns
// 16-byte aligned)
template <class P, bool VEC>
__global__ void __launch_bounds__(256) k_bin_keys(JoinArgs a, int64_t lo, int64_t n, uint32_t* keys, P* pts,
                                                  unsigned long long* n_skip) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    unsigned int skipped = 0;
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (VEC) {
        const int64_t np = (n - lo) / 2;
        const v2d* X = (const v2d*)(a.x + lo);
        const v2d* Y = (const v2d*)(a.y + lo);
        for (int64_t k = t0; k < np; k += stride) {
            const v2d x = __builtin_nontemporal_load(&X[k]), y = __builtin_nontemporal_load(&Y[k]);
            bin_one(a, lo + 2 * k, lo, x.x, y.x, keys, pts, skipped);
            bin_one(a, lo + 2 * k + 1, lo, x.y, y.y, keys, pts, skipped);
        }
        if (t0 == 0 && ((n - lo) & 1)) bin_one(a, n - 1, lo, a.x[n - 1], a.y[n - 1], keys, pts, skipped);
    } else {
        for (int64_t i = lo + t0; i < n; i += stride) bin_one(a, i, lo, a.x[i], a.y[i], keys, pts, skipped);
    }
    for (int off = 32; off > 0; off >>= 1) skipped += __shfl_down(skipped, off, 64);
    if ((threadIdx.x & 63) == 0 && skipped) atomicAdd(n_skip, (unsigned long long)skipped);
}

// ---- k_bin_cover: k_bin_keys for tile-image tables, keeping only the points some chip may hold
// (tile code not kSkip, and for an imaged record a set cover bit of the point's envelope-raster cell,
// tile_images.h), compacted in one pass: workgroup b takes kBinChunk consecutive points, counts the
// kept ones and finds its output offset by decoupled look-back over the earlier workgroups' status
// words (flag | count: an aggregate published at once, then the inclusive prefix), so the sort and
// the join see only the kept points.  A workgroup's chunk is its ordered ticket (an atomic counter
// taken at start, status[gridDim.x]), not its blockIdx: every status it waits on belongs to a
// workgroup that took an earlier ticket, so is already running and publishes its aggregate without
// waiting on anything -- whatever order the hardware dispatches workgroups in.  The wait is still
// bounded (spin_cap polls; then *err is set and the caller reruns the pass uncompacted; spin_cap < 0
// forces that fallback, for its test).
#if defined(MOSAIC_BIN_PPT)
static const int kBinPPT = MOSAIC_BIN_PPT;  // (measurement builds: 2 .. 16)
#else
// points per thread (4: the pass 20 % slower than 8; 16, the most the per-(item, wave) scan of one wave
// holds: C4 at 1e6 buildings 15.12 -> 14.18 ms, gpurun_out/r06p)
static const int kBinPPT = 16;
#endif
static_assert(kBinPPT % 2 == 0 && kBinPPT * 4 <= 64, "k_bin_cover's offsets scan is one wave");
static const int kBinChunk = 256 * kBinPPT;
static const unsigned long long kStAgg = 1ULL << 62, kStPre = 2ULL << 62, kStVal = (1ULL << 62) - 1;

// status words: one 8-byte word carries flag and count, so there is no payload to order; stores and
// polls go to memory (system scope: sc0 sc1), never to a stale L2 line of another XCD
__device__ __forceinline__ void st_publish(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned long long st_poll(unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// (explicit pointers and grid, not JoinArgs: they stay in scalar registers; every load is issued
// before the first use, with clamped indices instead of branches)
// Keys: kSkip (dropped), kFull, or the image key of the point's record part (tile_images.h
// bin_map_key); one table read per point and kept word (the tile's bin map record: key word and
// the cover word of the point's cell, one cache line).  COMPACT false (the fallback after a
// look-back failure): every point at its own position, dropped ones keyed kSkip (sorted first;
// *total counts them).
template <class P, bool VEC, bool COMPACT>
__global__ void __launch_bounds__(256) k_bin_cover(const double* __restrict__ X, const double* __restrict__ Y,
                                                   tiles::Grid g, const uint32_t* __restrict__ bin_map, int64_t lo,
                                                   int64_t n, uint32_t* keys, P* pts, unsigned long long* status,
                                                   unsigned long long* total, unsigned int* err, int spin_cap) {
    __shared__ uint32_t woff[kBinPPT * 4];  // per (item, wave): kept count, then output offset in the workgroup
    __shared__ unsigned long long base_s, ticket_s;
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    const unsigned long long lt_mask = (1ULL << lane) - 1ULL;
    if (COMPACT) {
        if (threadIdx.x == 0) ticket_s = atomicAdd(&status[gridDim.x], 1ULL);
        __syncthreads();
    }
    const int64_t b = COMPACT ? (int64_t)ticket_s : (int64_t)blockIdx.x;
    const int64_t cs = lo + b * kBinChunk;
    // item k of this thread: point cs + 2 (k/2 256 + t) + k%2 (VEC: 16-byte loads of both columns)
    // or cs + k 256 + t
    auto item = [&](int k) -> int64_t {
        return VEC ? cs + 2 * ((int64_t)(k >> 1) * 256 + threadIdx.x) + (k & 1) : cs + (int64_t)k * 256 + threadIdx.x;
    };
    double xs[kBinPPT], ys[kBinPPT];
    if (VEC) {
        // (n - lo >= 2: the caller's condition) the last pair start with both points in range
        const int64_t vlast = lo + (((n - lo) >> 1) - 1) * 2;
#pragma unroll
        for (int k = 0; k < kBinPPT; k += 2) {
            const int64_t i0 = item(k), li = i0 < vlast ? i0 : vlast;
            const v2d x = __builtin_nontemporal_load((const v2d*)(X + li)), y = __builtin_nontemporal_load((const v2d*)(Y + li));
            xs[k] = x.x;
            xs[k + 1] = x.y;
            ys[k] = y.x;
            ys[k + 1] = y.y;
        }
        if ((n - lo) & 1) {  // an odd last point: its own loads (last workgroup only)
#pragma unroll
            for (int k = 0; k < kBinPPT; k += 2)
                if (item(k) == n - 1) {
                    xs[k] = X[n - 1];
                    ys[k] = Y[n - 1];
                }
        }
    } else {
#pragma unroll
        for (int k = 0; k < kBinPPT; k++) {
            const int64_t i = item(k) < n ? item(k) : n - 1;
            xs[k] = X[i];
            ys[k] = Y[i];
        }
    }
    // the tile's bin map record: key word and the cover word of the point's envelope-raster cell
    // (binned::bin_cell: the cell as k_join_tiles computes it; both reads issued for every item
    // before any is used)
    uint32_t kw[kBinPPT], cw[kBinPPT];
    int q[kBinPPT];
#pragma unroll
    for (int k = 0; k < kBinPPT; k++) {
        const binned::BinCell bc = binned::bin_cell(g, xs[k], ys[k]);
        const uint32_t* m = bin_map + (size_t)bc.slot * binned::kBinMapWords;
        kw[k] = m[0];
        cw[k] = m[1 + (bc.q >> 5)];
        q[k] = bc.q;
        if (!bc.in) {  // off the grid: never kept, unless not finite (kFull: the generic path)
            kw[k] = (isfinite(xs[k]) && isfinite(ys[k])) ? tiles::kSkip : tiles::kFull;
            cw[k] = ~0u;
        }
        if (item(k) >= n) kw[k] = tiles::kSkip;
    }
    uint32_t code[kBinPPT];
    unsigned long long mk[kBinPPT];
#pragma unroll
    for (int k = 0; k < kBinPPT; k++) {
        const bool keep = binned::bin_map_keep(kw[k], cw[k], q[k]);
        code[k] = binned::bin_map_key(kw[k], q[k]);
        if (!COMPACT) {
            if (!keep) code[k] = tiles::kSkip;
            mk[k] = __ballot(item(k) < n && !keep);  // (dropped, counted)
            continue;
        }
        mk[k] = __ballot(keep);
        if (lane == 0) woff[k * 4 + wv] = (uint32_t)__popcll(mk[k]);
    }
    if (!COMPACT) {
        unsigned int dropped = 0;
#pragma unroll
        for (int k = 0; k < kBinPPT; k++) {
            dropped += (uint32_t)__popcll(mk[k]);
            const int64_t i = item(k);
            if (i < n) {
                keys[i - lo] = code[k];
                P p;
                p.x = xs[k];
                p.y = ys[k];
                binned::set_row(p, i);
                pts[i - lo] = p;
            }
        }
        if (lane == 0 && dropped) atomicAdd(total, (unsigned long long)dropped);
        return;
    }
    __syncthreads();
    if (wv == 0) {
        // offsets in (item, wave) order, the workgroup's count T
        const uint32_t c = lane < kBinPPT * 4 ? woff[lane] : 0u;
        uint32_t incl = c;
#pragma unroll
        for (int d = 1; d < kBinPPT * 4; d <<= 1) {
            const uint32_t t = __shfl_up(incl, d, 64);
            if (lane >= d) incl += t;
        }
        if (lane < kBinPPT * 4) woff[lane] = incl - c;
        const unsigned long long T = (unsigned long long)__shfl(incl, kBinPPT * 4 - 1, 64);
        // decoupled look-back: lane l reads workgroup j - l's status
        unsigned long long excl = 0;
        if (spin_cap < 0 && lane == 0) atomicOr(err, 1u);
        if (b > 0) {
            if (lane == 0) st_publish(&status[b], kStAgg | T);
            int64_t j = b - 1;
            int spins = 0;
            for (;;) {  // wave-uniform
                const int64_t k = j - lane;
                unsigned long long st = k >= 0 ? st_poll(&status[k]) : kStPre;
                while (__ballot((st >> 62) == 0)) {
                    if (++spins > spin_cap) {  // (never expected: see above)
                        if (lane == 0) atomicOr(err, 1u);
                        if ((st >> 62) == 0) st = kStPre;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                    if ((st >> 62) == 0) st = st_poll(&status[k]);
                }
                const unsigned long long pm = __ballot((st >> 62) == 2);
                const int stop = pm ? __ffsll((long long)pm) - 1 : 63;
                unsigned long long v = lane <= stop ? (st & kStVal) : 0ULL;
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
                excl += v;
                if (pm) break;
                j -= 64;
            }
        }
        if (lane == 0) {
            st_publish(&status[b], kStPre | (excl + T));
            base_s = excl;
            if (b == (int64_t)gridDim.x - 1) *total = excl + T;
        }
    }
    __syncthreads();
    const unsigned long long base = base_s;
#pragma unroll
    for (int k = 0; k < kBinPPT; k++) {
        if ((mk[k] >> lane) & 1ULL) {
            const int64_t i = item(k);
            const unsigned long long o = base + woff[k * 4 + wv] + (unsigned long long)__popcll(mk[k] & lt_mask);
            keys[o] = code[k];
            P p;
            p.x = xs[k];
            p.y = ys[k];
            binned::set_row(p, i);
            pts[o] = p;
        }
    }
}

// Waves take chunks of kChunkIters x 64 consecutive sorted points (chunk c by wave c mod W), so a
// wave stays inside one tile for many groups and its per-wave count hash sees few keys.
static const int kChunkIters = 16;

template <int CM, bool PAIRS, class P>
__global__ void __launch_bounds__(256) k_join_binned(JoinArgs a, const uint32_t* __restrict__ keys,
                                                     const P* __restrict__ pts, int64_t n, const unsigned long long* n_skip) {
    extern __shared__ unsigned int lds[];
    __shared__ SlabItem items[4][16];
    const int lane = (int)(threadIdx.x & 63);
    const int wv = (int)(threadIdx.x >> 6) & 3;
    unsigned int* cnt = lds;
    if (CM == kCountLds) {
        for (int k = threadIdx.x; k < a.n_polygons; k += blockDim.x) lds[k] = 0;
    } else if (CM == kCountWaveHash) {
        cnt = lds + wv * kWaveHashWords;
        for (int k = lane; k < kWaveHashWords; k += 64) cnt[k] = 0;
    }
    __syncthreads();
    unsigned int tests = 0;
    const int64_t lo = (int64_t)*n_skip;  // kSkip rows sort first: none of them can join
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t wid = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t chunk = 64 * kChunkIters;
    for (int64_t c0 = lo + wid * chunk; c0 < n; c0 += waves * chunk) {
        const int64_t c1 = c0 + chunk < n ? c0 + chunk : n;
        for (int64_t base = c0; base < c1; base += 64) {
            const int64_t i = base + lane;
            const bool live = i < c1;
            double x = 0.0, y = 0.0;
            int64_t row = -1;
            uint32_t cur = 0, end = 0;
            if (live) {
                const P p = pts[i];
                x = p.x;
                y = p.y;
                row = binned::row_of(p, i);
                tiled_cell(a, i, x, y, keys[i], cur, end);
            }
            raster_chips<CM, PAIRS>(a, row, cur, end, x, y, tests, cnt, items[wv]);
            if (CM == kCountWaveHash) wave_hash_flush(a, cnt, false);
        }
    }
    if (CM == kCountWaveHash) wave_hash_flush(a, cnt, true);
    for (int off = 32; off > 0; off >>= 1) tests += __shfl_down(tests, off, 64);
    if (lane == 0 && tests) atomicAdd(a.tests, (unsigned long long)tests);
    if (CM == kCountLds) {
        __syncthreads();
        for (int k = threadIdx.x; k < a.n_polygons; k += blockDim.x)
            if (lds[k]) atomicAdd(&a.counts[k], (unsigned long long)lds[k]);
    }
}

// ---- k_join_tiles: the binned join over per-tile chip images in LDS (north_star kernel (c): chip
// rings tiled into LDS).  A workgroup takes kSegPoints consecutive sorted points and walks their
// runs of equal tile code; per run it copies the tile's image (join_binned.h) into LDS once, then
// each lane finds its point's hexagon from the tile record (tiled_cell's face-plane rounding: the
// same certified hexagon) and tests the hexagon's chips from LDS: core chips count, border chips
// get the f32 envelope pre-test and JTS's ray-crossing ring walk (pip::locate_in_ring's
// arithmetic) on LDS vertices.  Chips kept in the global store (multi-ring / multi-part, or past
// the image's vertex budget) take pip::contains; runs without an image (kFull tiles, records over
// the image cap) and hexagons outside the window take the same pair path over the chip table
// (envelope from geom_bbox, then pip::contains; the sorted order keeps those reads in L1 / L2).
// Chip indices fit 26 bits (the caller's condition).
// The (point, chip) pairs of 64 points are taken 64 at a time, one per lane; core chips count at
// once, border chips get the f32 envelope test, and the pairs that pass it (a fraction: a point
// near a building lies in few of its cell's chip envelopes) are compacted into a per-wave LDS
// buffer whose full sets of 64 run the ring walk -- no lane of a ring-walking wave idles on a pair
// the envelope already rejected.
#if defined(MOSAIC_TJ_SEG)
static const int kSegPoints = MOSAIC_TJ_SEG;  // (measurement builds)
#else
static const int kSegPoints = 2048;
#endif

static const int kSurv = 128;  // per wave: surviving pairs (64 appended at most before a flush)
static const uint32_t kSurvGlobal = 0x80000000u;  // a buffered pair's chip is in the chip table
// a hit of the tile join's count mode kCountChips: image chip sc (kSurvGlobal: chip of the table)
__device__ __forceinline__ void tile_hit(const JoinArgs& a, unsigned int* ccnt, uint32_t sc, uint32_t key) {
    if (sc & 0x80000000u)
        atomicAdd(&a.counts[key], 1ULL);
    else
        atomicAdd(&ccnt[sc], 1u);
}

// false only when (x, y) lies outside the chip's f64 envelope (the f32 box is rounded outwards and
// rounding is monotone, so fx, fy of a point inside the f64 box are inside the f32 box)
__device__ __forceinline__ bool fbox_in(const uint32_t* cr, float fx, float fy) {
    return fx >= __uint_as_float(cr[4]) && fy >= __uint_as_float(cr[5]) && fx <= __uint_as_float(cr[6]) &&
           fy <= __uint_as_float(cr[7]);
}

// the tile join's f32 ring walk: rolled (no scratch; 152 bytes per lane with the unrolled form);
// a measurement build may set MOSAIC_TJ_UNROLLED_WALK
#if defined(MOSAIC_TJ_UNROLLED_WALK)
#define MOSAIC_TJ_WALK ringwalk::ring_interior_f32
#else
#define MOSAIC_TJ_WALK ringwalk::ring_interior_f32_rolled
#endif

// the tile join's rare paths, inlined (as calls, the C4 1e6 kernel went 8.87 -> 10.88 ms: call-site
// register saves and spills)
#define MOSAIC_TJ_NOINLINE __device__ __forceinline__
#if defined(MOSAIC_TJ_CONTAINS_CALL)  // measurement build: only the f64 walk (undecided pairs) as a call
__device__ __attribute__((noinline)) bool contains_call(const pip::GeomStore& s, uint32_t c, double x, double y) {
#else
MOSAIC_TJ_NOINLINE bool contains_call(const pip::GeomStore& s, uint32_t c, double x, double y) {
#endif
    return pip::contains(s, c, x, y);
}
MOSAIC_TJ_NOINLINE uint2 tiled_cell_call(const JoinArgs& a, int64_t i, double x, double y, uint32_t code) {
    uint32_t c0, c1;
    tiled_cell(a, i, x, y, code, c0, c1);
    return make_uint2(c0, c1);
}
MOSAIC_TJ_NOINLINE uint2 probe_call(const JoinArgs& a, int64_t cell) {
    uint32_t c0, c1;
    probe(a, cell, c0, c1);
    return make_uint2(c0, c1);
}

// (occupancy 4: 128 VGPRs; C4 1e6 measured 23.4 ms against 28.7 unconstrained and 27.1 at 5)
template <int CM, bool PAIRS, class P>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
k_join_tiles(JoinArgs a, const uint32_t* __restrict__ keys, const P* __restrict__ pts, int64_t n,
             const unsigned long long* n_skip, binned::Images img, uint32_t img_words) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_t[];
    __shared__ uint32_t pairs_all[4 * 64];  // per wave: a window of (point lane, chip) pairs
    __shared__ double surv_x[4][kSurv], surv_y[4][kSurv];
    __shared__ uint32_t surv_c[4][kSurv];
    __shared__ long long surv_r[PAIRS ? 4 : 1][PAIRS ? kSurv : 1];
    __shared__ unsigned long long run_end_s;
    const int lane = (int)(threadIdx.x & 63);
    const int wv = (int)(threadIdx.x >> 6) & 3;
    const unsigned long long lt_mask = (1ULL << lane) - 1ULL;
    uint32_t* im = lds_t;
    unsigned int* cnt = lds_t + img_words;  // kCountLds: per polygon; kCountChips: per image chip
    if (CM == kCountLds) {
        for (int k = threadIdx.x; k < a.n_polygons; k += blockDim.x) cnt[k] = 0;
    } else if (CM == kCountChips) {
        for (int k = threadIdx.x; k < (int)binned::kImgMaxChips; k += blockDim.x) cnt[k] = 0;
    }
    __syncthreads();
    unsigned int tests = 0;
    const int64_t s0 = (int64_t)*n_skip + (int64_t)blockIdx.x * kSegPoints;
    const int64_t s1 = s0 + kSegPoints < n ? s0 + kSegPoints : n;
    for (int64_t pos = s0; pos < s1;) {  // block-uniform: one run of equal tile code per iteration
        const uint32_t code = keys[pos];
        if (threadIdx.x == 0) run_end_s = (unsigned long long)s1;
        __syncthreads();
        for (int64_t b = pos + 1; b < s1; b += 256) {
            const int64_t i = b + threadIdx.x;
            if (i < s1 && keys[i] != code) atomicMin(&run_end_s, (unsigned long long)i);
            __syncthreads();
            const bool found = run_end_s < (unsigned long long)s1;
            __syncthreads();
            if (found) break;
        }
        const int64_t r1 = (int64_t)run_end_s;
        // the run's image key -> image, tile record (tcode: its tile code, for the generic path)
        const uint32_t ioff = code >= 2 ? img.off[code - 2] : binned::kNoImage;
        const uint32_t tcode = code >= 2 ? img.rec[code - 2] + 2u : code;
        tiles::TileRec tr{0, 0, 0, 0};
        if (ioff != binned::kNoImage) {
            tr = a.tile_rec[tcode - 2];
            const uint32_t* src = img.words + ioff;
            const uint32_t nw = (src[3] + 2u * src[1] + 3u) & ~3u;  // vertex offset + vertex words (padded)
            for (uint32_t k = 4u * threadIdx.x; k < nw; k += 4u * blockDim.x)
                *(uint4*)(im + k) = *(const uint4*)(src + k);
            __syncthreads();
        }
        const int face = (int)(tr.dims & 0xffu);
        const int wa = (int)((tr.dims >> 8) & 0xfffu), wb = (int)(tr.dims >> 20);
        const uint32_t* chips = im + im[2];
        const float* V = (const float*)(im + im[3]);
        const uint16_t* rl = (const uint16_t*)(im + im[4]);  // envelope raster: list offsets, lists
        // the ring walk over the wave's buffered pairs, 64 at a time from the top of the buffer
        // (all of them when `all`); wave-uniform
        uint32_t sn = 0;
        auto ring_tests = [&](bool all) {
            while (sn >= 64 || (all && sn > 0)) {
                const uint32_t m = sn < 64u ? sn : 64u;
                if ((uint32_t)lane < m) {
                    const uint32_t e = sn - m + (uint32_t)lane;
                    const double qx = surv_x[wv][e], qy = surv_y[wv][e];
                    const uint32_t sc = surv_c[wv][e];
                    bool hit;
                    uint32_t key;
                    if (sc & kSurvGlobal) {  // a chip of the table (a run without an image, a hexagon off the window)
                        const uint32_t c = sc & ~kSurvGlobal;
                        hit = contains_call(a.store, c, qx, qy);
                        key = a.chip_meta[c] >> 1;
                    } else {
                        const uint32_t* cr = chips + binned::kImgChipWords * sc;
                        const uint32_t vi = cr[1], vc = vi >> 16;
                        int r = 2;
                        if (vc != binned::kImgGlobal)
                            r = MOSAIC_TJ_WALK(V + 2u * (vi & 0xffffu), vc,
                                                            ringwalk::f32_frame(__uint_as_float(cr[4]), __uint_as_float(cr[5]),
                                                                                __uint_as_float(cr[6]), __uint_as_float(cr[7]), qx, qy));
                        // (global geometry, or a point the f32 walk leaves undecided: the f64 test)
                        hit = r == 2 ? contains_call(a.store, cr[2], qx, qy) : r == 1;
                        key = cr[0] >> 1;
                    }
                    if (hit) {
                        if (CM == kCountChips)
                            tile_hit(a, cnt, sc, key);
                        else
                            emit_hit<CM, PAIRS>(a, PAIRS ? (int64_t)surv_r[wv][e] : -1, key, cnt);
                    }
                }
                sn -= m;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        };
        for (int64_t g = pos + wv * 64; g < r1; g += 256) {  // wave-uniform
            const int64_t i = g + lane;
            double x = 0.0, y = 0.0;
            int64_t row = -1;
            uint32_t c0 = 0, c1 = 0;  // the point's candidates: envelope-raster list positions, or (glob) chips of the table
            uint32_t slot = 0;        // its hexagon's window slot (image runs)
            bool glob = false;
            if (i < r1) {
                const P p = pts[i];
                x = p.x;
                y = p.y;
                row = binned::row_of(p, i);
                if (ioff == binned::kNoImage) {
                    const uint2 r = tiled_cell_call(a, i, x, y, tcode);
                    c0 = r.x;
                    c1 = r.y;
                    glob = true;
                } else {
                    // the raster cell (k_bin_cover's arithmetic): chips whose envelope may hold the point
                    const int q = binned::bin_cell(a.tgrid, x, y).q;
                    c0 = rl[q];
                    c1 = rl[q + 1];
                    if (c1 > c0) {  // (a point no envelope holds joins nothing: its hexagon is not needed)
                        double px, py, pz, vx, vy, best;
                        h3::fast_unit(y, x, &px, &py, &pz);
                        h3::fast_plane(px, py, pz, face, a.res, &vx, &vy, &best);
                        int ba, bb;
                        if (!h3::fast_hex(vx, vy, a.res, &ba, &bb)) {
                            const unsigned long long qe = atomicAdd(a.amb_count, 1ULL);
                            if (qe < a.amb_cap) a.amb_queue[qe] = (unsigned long long)i;
                            c0 = c1 = 0;
                        } else {
                            const int ra = ba - tr.a0, rb = bb - tr.b0;
                            if ((unsigned)ra < (unsigned)wa && (unsigned)rb < (unsigned)wb) {
                                slot = (uint32_t)(ra * wb + rb);
#if !defined(MOSAIC_TJ_NO_SLOT_NARROW)
                                // a list holds its chips in ascending image order, which is ascending
                                // window slot (tile_images.h block_image): the point's own slot's chips
                                // are one run of it, found by two binary searches (without them 35 % of
                                // the pair windows held chips of other hexagons; C4 at 5e6 buildings
                                // 30.1 -> 27.6 ms, gpurun_out/r06nw)
                                uint32_t lo = c0, hi = c1;
                                while (lo < hi) {
                                    const uint32_t m = (lo + hi) >> 1;
                                    if (chips[binned::kImgChipWords * rl[m] + 3] < slot) lo = m + 1;
                                    else hi = m;
                                }
                                c0 = lo;
                                hi = c1;
                                while (lo < hi) {
                                    const uint32_t m = (lo + hi) >> 1;
                                    if (chips[binned::kImgChipWords * rl[m] + 3] <= slot) lo = m + 1;
                                    else hi = m;
                                }
                                c1 = lo;
#endif
                            } else {
                                const uint2 r = probe_call(a, (int64_t)h3::face_axial_to_h3(face, ba, bb, a.res));
                                c0 = r.x;
                                c1 = r.y;
                                glob = true;
                            }
                        }
                    }
                }
            }
            // the group's (point, chip) pairs, 64 at a time, one per lane: the work is spread over
            // the wave whatever the points' chip counts (a lane per point would run the wave for
            // its most crowded cell)
            const uint32_t n = c1 - c0;
            uint32_t incl = n;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t t = __shfl_up(incl, d, 64);
                if (lane >= d) incl += t;
            }
            const uint32_t off = incl - n, T = __shfl(incl, 63, 64);
            uint32_t* pb = pairs_all + wv * 64;
            for (uint32_t w0 = 0; w0 < T; w0 += 64) {  // wave-uniform
                const uint32_t e0 = off > w0 ? off : w0, e1 = off + n < w0 + 64 ? off + n : w0 + 64;
                for (uint32_t e = e0; e < e1; e++) pb[e - w0] = (uint32_t)lane | (c0 + (e - off)) << 6;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const bool live = w0 + (uint32_t)lane < T;
#if defined(MOSAIC_TJ_COUNT_FORMED)  // measurement build: the stat counts every pair formed instead
                tests += live ? 1u : 0u;
#endif
                const uint32_t ent = live ? pb[lane] : 0u;
                const int owner = (int)(ent & 63u);
                const double qx = __shfl(x, owner, 64), qy = __shfl(y, owner, 64);
                const int64_t qrow = PAIRS ? (int64_t)__shfl((long long)row, owner, 64) : -1;
                const bool qg = __shfl((int)glob, owner, 64) != 0;
                const uint32_t qslot = (uint32_t)__shfl((int)slot, owner, 64);
                bool surv = false;
                uint32_t c = ent >> 6;  // glob: a chip of the table; else a list position
                if (live && !qg) c = rl[c];
                const uint32_t* cr = chips + binned::kImgChipWords * c;
                if (live && (qg || cr[3] == qslot)) {  // (image chips of another hexagon: no pair)
                    const uint32_t meta = qg ? a.chip_meta[c] : cr[0];
                    if (meta & 1u) {
                        if (CM == kCountChips)
                            tile_hit(a, cnt, c | (qg ? kSurvGlobal : 0u), meta >> 1);
                        else
                            emit_hit<CM, PAIRS>(a, qrow, meta >> 1, cnt);
                    } else {
#if !defined(MOSAIC_TJ_COUNT_FORMED)
                        tests++;
#endif
                        surv = qg ? !pip::box_excludes(a.store.geom_bbox[c], qx, qy) : fbox_in(cr, (float)qx, (float)qy);
                    }
                }
                const unsigned long long sm = __ballot(surv);
                if (surv) {
                    const uint32_t e = sn + (uint32_t)__popcll(sm & lt_mask);
                    surv_x[wv][e] = qx;
                    surv_y[wv][e] = qy;
                    surv_c[wv][e] = c | (qg ? kSurvGlobal : 0u);
                    if (PAIRS) surv_r[wv][e] = (long long)qrow;
                }
                sn += (uint32_t)__popcll(sm);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (sn >= 64) ring_tests(false);
            }
        }
        ring_tests(true);  // the run's last buffered pairs, while its image is in LDS
        __syncthreads();  // every wave is done with this run's image
        if (CM == kCountChips && ioff != binned::kNoImage) {
            // the run's chip counts to their polygons (before the next run's image replaces the chips)
            const uint32_t nc = im[0];
            for (uint32_t k = threadIdx.x; k < nc; k += blockDim.x) {
                const uint32_t v = cnt[k];
                if (v) {
                    atomicAdd(&a.counts[chips[binned::kImgChipWords * k] >> 1], (unsigned long long)v);
                    cnt[k] = 0;
                }
            }
        }
        pos = r1;
    }
    for (int off = 32; off > 0; off >>= 1) tests += __shfl_down(tests, off, 64);
    if (lane == 0 && tests) atomicAdd(a.tests, (unsigned long long)tests);
    if (CM == kCountLds) {
        __syncthreads();
        for (int k = threadIdx.x; k < a.n_polygons; k += blockDim.x)
            if (cnt[k]) atomicAdd(&a.counts[k], (unsigned long long)cnt[k]);
    }
}

namespace binned {

// Onesweep radix sort of (key, point) over bits [0, end_bit) with R bits per pass: keys of 17-22
// bits (image keys of large tables) sort in two passes instead of hipcub's three 8-bit ones.
#if !defined(MOSAIC_SORT_BLOCK)  // (measurement builds may set the onesweep block and items per thread)
#define MOSAIC_SORT_BLOCK 1024
#define MOSAIC_SORT_ITEMS 12
#endif
template <unsigned R>
using OnesweepR = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<MOSAIC_SORT_BLOCK, MOSAIC_SORT_ITEMS>,
                                        rocprim::kernel_config<MOSAIC_SORT_BLOCK, MOSAIC_SORT_ITEMS>, R,
                                        rocprim::block_radix_rank_algorithm::match>>;
template <unsigned R, class P>
static hipError_t sort_r(void* tmp, size_t& tb, uint32_t* const k[2], P* const v[2], int64_t m, int end_bit,
                         hipStream_t stream, int& cur) {
    rocprim::double_buffer<uint32_t> kb(k[0], k[1]);
    rocprim::double_buffer<P> vb(v[0], v[1]);
    const hipError_t e = rocprim::radix_sort_pairs<OnesweepR<R>>(tmp, tb, kb, vb, (size_t)m, 0u, (unsigned)end_bit, stream);
    cur = kb.current() == k[0] ? 0 : 1;
    return e;
}
template <class P>
static hipError_t sort_wide(void* tmp, size_t& tb, uint32_t* const k[2], P* const v[2], int64_t m, int end_bit,
                            hipStream_t stream, int& cur) {
    if (end_bit <= 18) return sort_r<9, P>(tmp, tb, k, v, m, end_bit, stream, cur);
    if (end_bit <= 20) return sort_r<10, P>(tmp, tb, k, v, m, end_bit, stream, cur);
    return sort_r<11, P>(tmp, tb, k, v, m, end_bit, stream, cur);
}

template <class P>
static hipError_t sort_and_join(const JoinArgs& a0, int64_t lo, int64_t n, uint32_t max_code, int cm, int n_cu,
                                const Images& img, Scratch& s, hipStream_t stream) {
    int64_t m = n - lo;
    const size_t vb = sizeof(P);
    hipError_t e;
    const int64_t nb = (m + kBinChunk - 1) / kBinChunk;
    if ((e = s.keys[0].reserve((size_t)m * 4)) || (e = s.keys[1].reserve((size_t)m * 4)) ||
        (e = s.vals[0].reserve((size_t)m * vb)) || (e = s.vals[1].reserve((size_t)m * vb)) || (e = s.n_skip.reserve(32)) ||
        (img.words && (e = s.status.reserve((size_t)std::max<int64_t>(nb + 1, 1) * 8))))
        return e;
    // n_skip words: [0] kSkip rows (k_bin_keys) or kept rows (k_bin_cover), [1] 0, [2] look-back failure
    if ((e = hipMemsetAsync(s.n_skip.p, 0, 32, stream))) return e;
    unsigned long long* nsk = (unsigned long long*)s.n_skip.p;
    s.lookback_failed = 0;
    const bool vec = (((uintptr_t)(a0.x + lo) | (uintptr_t)(a0.y + lo)) & 15) == 0;
    bool keyed = false;  // keys from k_bin_cover (image keys)
    if (img.words && m > 0) {
        if ((e = hipMemsetAsync(s.status.p, 0, (size_t)(nb + 1) * 8, stream))) return e;  // (+ the ticket)
        unsigned int* err = (unsigned int*)(nsk + 2);
        unsigned long long* st = (unsigned long long*)s.status.p;
#define MOSAIC_BIN_COVER(VEC, COMPACT)                                                                                \
    hipLaunchKernelGGL((k_bin_cover<P, VEC, COMPACT>), dim3(nb), dim3(256), 0, stream, a0.x, a0.y, a0.tgrid,              \
                       img.bin_map, lo, n, (uint32_t*)s.keys[0].p, (P*)s.vals[0].p, st, nsk, err, s.spin_cap)
        if (vec && m >= 2)
            MOSAIC_BIN_COVER(true, true);
        else
            MOSAIC_BIN_COVER(false, true);
        if ((e = hipGetLastError())) return e;
        unsigned long long hw[3];
        if ((e = hipMemcpyAsync(hw, nsk, sizeof hw, hipMemcpyDeviceToHost, stream)) || (e = hipStreamSynchronize(stream)))
            return e;
        const bool ok = hw[2] == 0 && hw[0] <= (unsigned long long)m;
        s.lookback_failed = !ok;
        if (ok) {
            m = (int64_t)hw[0];
            nsk += 1;  // the join starts at sorted row 0
        }
        if (!ok) {
            // the look-back gave up: every row in place, dropped rows keyed kSkip (counted in word 0)
            if ((e = hipMemsetAsync(s.n_skip.p, 0, 32, stream))) return e;
            if (vec && m >= 2)
                MOSAIC_BIN_COVER(true, false);
            else
                MOSAIC_BIN_COVER(false, false);
            if ((e = hipGetLastError())) return e;
        }
#undef MOSAIC_BIN_COVER
        keyed = true;
        max_code = img.n_images + 1u;
    }
    if (!keyed) {
        const int gk = (int)std::max<int64_t>(1, std::min<int64_t>((m + 511) / 512, (int64_t)n_cu * 16));
        if (vec)
            hipLaunchKernelGGL((k_bin_keys<P, true>), dim3(gk), dim3(256), 0, stream, a0, lo, n, (uint32_t*)s.keys[0].p,
                               (P*)s.vals[0].p, nsk);
        else
            hipLaunchKernelGGL((k_bin_keys<P, false>), dim3(gk), dim3(256), 0, stream, a0, lo, n, (uint32_t*)s.keys[0].p,
                               (P*)s.vals[0].p, nsk);
        if ((e = hipGetLastError())) return e;
    }
    s.sorted_rows = m;
    // the key's significant bits (codes <= max_code)
    int end_bit = 1;
    while (end_bit < 32 && (max_code >> end_bit)) end_bit++;
    hipcub::DoubleBuffer<uint32_t> kb((uint32_t*)s.keys[0].p, (uint32_t*)s.keys[1].p);
    hipcub::DoubleBuffer<P> pb((P*)s.vals[0].p, (P*)s.vals[1].p);
    size_t tb = 0;
    if (end_bit > 16 && end_bit <= 22) {
        uint32_t* const k2[2] = {(uint32_t*)s.keys[0].p, (uint32_t*)s.keys[1].p};
        P* const v2[2] = {(P*)s.vals[0].p, (P*)s.vals[1].p};
        int cur = 0;
        if ((e = sort_wide<P>(nullptr, tb, k2, v2, m, end_bit, stream, cur))) return e;
        if ((e = s.temp.reserve(tb))) return e;
        if ((e = sort_wide<P>(s.temp.p, tb, k2, v2, m, end_bit, stream, cur))) return e;
        kb = hipcub::DoubleBuffer<uint32_t>(k2[cur], k2[1 - cur]);
        pb = hipcub::DoubleBuffer<P>(v2[cur], v2[1 - cur]);
    } else {
        if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kb, pb, (int)m, 0, end_bit, stream))) return e;
        if ((e = s.temp.reserve(tb))) return e;
        if ((e = hipcub::DeviceRadixSort::SortPairs(s.temp.p, tb, kb, pb, (int)m, 0, end_bit, stream))) return e;
    }
    JoinArgs a = a0;
    a.x = &pb.Current()->x;
    a.y = &pb.Current()->y;
    a.cstride = (int32_t)(sizeof(P) / 8);
    a.rowmap = row_map(pb.Current());
    a.row_lo = 0;
    const int blk = 256;
    const int gj = (int)std::max<int64_t>(1, std::min<int64_t>((m + 64 * kChunkIters * 4 - 1) / (64 * kChunkIters * 4),
                                                               (int64_t)n_cu * 8));
    const uint32_t* keys = kb.Current();
    const P* pts = pb.Current();
    const bool pairs = a.pair_row != nullptr;
    if (img.words) {
        // one workgroup per kSegPoints sorted points (those past the kSkip prefix exit at once)
        const uint32_t iw = (img.max_words + 3u) & ~3u;
        const int gt = (int)std::max<int64_t>(1, (m + kSegPoints - 1) / kSegPoints);
        const size_t cw = pairs ? 0 : (cm == kCountLds ? (size_t)a.n_polygons : (size_t)binned::kImgMaxChips);
        const size_t shm = ((size_t)iw + cw) * 4;
        if (pairs)
            hipLaunchKernelGGL((k_join_tiles<kCountGlobal, true, P>), dim3(gt), dim3(blk), shm, stream, a, keys, pts, m, nsk, img, iw);
        else if (cm == kCountLds)
            hipLaunchKernelGGL((k_join_tiles<kCountLds, false, P>), dim3(gt), dim3(blk), shm, stream, a, keys, pts, m, nsk, img, iw);
        else
            hipLaunchKernelGGL((k_join_tiles<kCountChips, false, P>), dim3(gt), dim3(blk), shm, stream, a, keys, pts, m, nsk,
                               img, iw);
    } else if (pairs) {
        hipLaunchKernelGGL((k_join_binned<kCountGlobal, true, P>), dim3(gj), dim3(blk), 0, stream, a, keys, pts, m, nsk);
    } else if (cm == kCountLds) {
        hipLaunchKernelGGL((k_join_binned<kCountLds, false, P>), dim3(gj), dim3(blk), (size_t)a.n_polygons * 4, stream, a,
                           keys, pts, m, nsk);
    } else {
        hipLaunchKernelGGL((k_join_binned<kCountWaveHash, false, P>), dim3(gj), dim3(blk),
                           (size_t)(blk / 64) * kWaveHashWords * 4, stream, a, keys, pts, m, nsk);
    }
    if ((e = hipGetLastError())) return e;
    s.exact_args = a;
    return hipSuccess;
}

hipError_t join(const JoinArgs& a, int64_t lo, int64_t n, uint32_t max_code, bool lds_counts, int n_cu,
                const Images& img, Scratch& s, hipStream_t stream) {
    const int cm = lds_counts ? kCountLds : kCountWaveHash;
    if (a.pair_row) return sort_and_join<PtRow>(a, lo, n, max_code, cm, n_cu, img, s, stream);
    return sort_and_join<Pt>(a, lo, n, max_code, cm, n_cu, img, s, stream);
}

}  // namespace binned

extern "C" uint64_t mosaic_layout_join_binned(void) { return mosaic_layout_fingerprint(); }
