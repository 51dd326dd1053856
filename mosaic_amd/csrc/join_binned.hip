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
#include <hipcub/hipcub.hpp>
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
static const int kSegPoints = 2048;
static const int kSurv = 128;  // per wave: surviving pairs (64 appended at most before a flush)
static const uint32_t kSurvGlobal = 0x80000000u;  // a buffered pair's chip is in the chip table

// false only when (x, y) lies outside the chip's f64 envelope (the f32 box is rounded outwards and
// rounding is monotone, so fx, fy of a point inside the f64 box are inside the f32 box)
__device__ __forceinline__ bool fbox_in(const uint32_t* cr, float fx, float fy) {
    return fx >= __uint_as_float(cr[4]) && fy >= __uint_as_float(cr[5]) && fx <= __uint_as_float(cr[6]) &&
           fy <= __uint_as_float(cr[7]);
}

// the tile join's rare paths, as calls: their registers (the general JTS walk over the chip table,
// the generic point -> chips path) do not count against the kernel's occupancy
__device__ __noinline__ bool contains_call(const pip::GeomStore& s, uint32_t c, double x, double y) {
    return pip::contains(s, c, x, y);
}
__device__ __noinline__ uint2 tiled_cell_call(const JoinArgs& a, int64_t i, double x, double y, uint32_t code) {
    uint32_t c0, c1;
    tiled_cell(a, i, x, y, code, c0, c1);
    return make_uint2(c0, c1);
}
__device__ __noinline__ uint2 probe_call(const JoinArgs& a, int64_t cell) {
    uint32_t c0, c1;
    probe(a, cell, c0, c1);
    return make_uint2(c0, c1);
}

template <int CM, bool PAIRS, class P>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) k_join_tiles(JoinArgs a, const uint32_t* __restrict__ keys,
                                                    const P* __restrict__ pts, int64_t n, const unsigned long long* n_skip,
                                                    binned::Images img, uint32_t img_words) {
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
    unsigned int* cnt = lds_t + img_words;
    if (CM == kCountLds) {
        for (int k = threadIdx.x; k < a.n_polygons; k += blockDim.x) cnt[k] = 0;
    } else if (CM == kCountWaveHash) {
        cnt += wv * kWaveHashWords;
        for (int k = lane; k < kWaveHashWords; k += 64) cnt[k] = 0;
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
        const uint32_t ioff = (code >= 2 && img.off) ? img.off[code - 2] : binned::kNoImage;
        tiles::TileRec tr{0, 0, 0, 0};
        if (ioff != binned::kNoImage) {
            tr = a.tile_rec[code - 2];
            const uint32_t* src = img.words + ioff;
            const uint32_t nw = src[3] + 4u * src[1];  // vertex offset + vertex words
            for (uint32_t k = 4u * threadIdx.x; k < nw; k += 4u * blockDim.x)
                *(uint4*)(im + k) = *(const uint4*)(src + k);
            __syncthreads();
        }
        const int face = (int)(tr.dims & 0xffu);
        const int wa = (int)((tr.dims >> 8) & 0xfffu), wb = (int)(tr.dims >> 20);
        const uint32_t* chips = im + im[2];
        const double* V = (const double*)(im + im[3]);
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
                        const uint32_t* cr = chips + 8u * sc;
                        const uint32_t vi = cr[1], vc = vi >> 16;
                        hit = vc == binned::kImgGlobal ? contains_call(a.store, cr[2], qx, qy)
                                                       : ringwalk::ring_interior(V + 2u * (vi & 0xffffu), vc, qx, qy);
                        key = cr[0] >> 1;
                    }
                    if (hit) emit_hit<CM, PAIRS>(a, PAIRS ? (int64_t)surv_r[wv][e] : -1, key, cnt);
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
                    const uint2 r = tiled_cell_call(a, i, x, y, code);
                    c0 = r.x;
                    c1 = r.y;
                    glob = true;
                } else {
                    // the raster cell (tile_of's arithmetic): chips whose envelope may hold the point
                    const double fx = (x - a.tgrid.x0) * a.tgrid.sx, fy = (y - a.tgrid.y0) * a.tgrid.sy;
                    const int gx = (int)((fx - (double)(int)fx) * (double)binned::kImgRaster);
                    const int gy = (int)((fy - (double)(int)fy) * (double)binned::kImgRaster);
                    const int q = min(gy, binned::kImgRaster - 1) * binned::kImgRaster + min(gx, binned::kImgRaster - 1);
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
                const uint32_t ent = live ? pb[lane] : 0u;
                const int owner = (int)(ent & 63u);
                const double qx = __shfl(x, owner, 64), qy = __shfl(y, owner, 64);
                const int64_t qrow = PAIRS ? (int64_t)__shfl((long long)row, owner, 64) : -1;
                const bool qg = __shfl((int)glob, owner, 64) != 0;
                const uint32_t qslot = (uint32_t)__shfl((int)slot, owner, 64);
                bool surv = false;
                uint32_t c = ent >> 6;  // glob: a chip of the table; else a list position
                if (live && !qg) c = rl[c];
                const uint32_t* cr = chips + 8u * c;
                if (live && (qg || cr[3] == qslot)) {  // (image chips of another hexagon: no pair)
                    const uint32_t meta = qg ? a.chip_meta[c] : cr[0];
                    if (meta & 1u) {
                        emit_hit<CM, PAIRS>(a, qrow, meta >> 1, cnt);
                    } else {
                        tests++;
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
            if (CM == kCountWaveHash) wave_hash_flush(a, cnt, false);
        }
        ring_tests(true);  // the run's last buffered pairs, while its image is in LDS
        if (CM == kCountWaveHash) wave_hash_flush(a, cnt, false);
        __syncthreads();  // every wave is done with this run's image
        pos = r1;
    }
    if (CM == kCountWaveHash) wave_hash_flush(a, cnt, true);
    for (int off = 32; off > 0; off >>= 1) tests += __shfl_down(tests, off, 64);
    if (lane == 0 && tests) atomicAdd(a.tests, (unsigned long long)tests);
    if (CM == kCountLds) {
        __syncthreads();
        for (int k = threadIdx.x; k < a.n_polygons; k += blockDim.x)
            if (cnt[k]) atomicAdd(&a.counts[k], (unsigned long long)cnt[k]);
    }
}

namespace binned {

template <class P>
static hipError_t sort_and_join(const JoinArgs& a0, int64_t lo, int64_t n, uint32_t max_code, int cm, int n_cu,
                                const Images& img, Scratch& s, hipStream_t stream) {
    const int64_t m = n - lo;
    const size_t vb = sizeof(P);
    hipError_t e;
    if ((e = s.keys[0].reserve((size_t)m * 4)) || (e = s.keys[1].reserve((size_t)m * 4)) ||
        (e = s.vals[0].reserve((size_t)m * vb)) || (e = s.vals[1].reserve((size_t)m * vb)) || (e = s.n_skip.reserve(8)))
        return e;
    if ((e = hipMemsetAsync(s.n_skip.p, 0, 8, stream))) return e;
    unsigned long long* nsk = (unsigned long long*)s.n_skip.p;
    const int gk = (int)std::max<int64_t>(1, std::min<int64_t>((m + 511) / 512, (int64_t)n_cu * 16));
    if ((((uintptr_t)(a0.x + lo) | (uintptr_t)(a0.y + lo)) & 15) == 0)
        hipLaunchKernelGGL((k_bin_keys<P, true>), dim3(gk), dim3(256), 0, stream, a0, lo, n, (uint32_t*)s.keys[0].p,
                           (P*)s.vals[0].p, nsk);
    else
        hipLaunchKernelGGL((k_bin_keys<P, false>), dim3(gk), dim3(256), 0, stream, a0, lo, n, (uint32_t*)s.keys[0].p,
                           (P*)s.vals[0].p, nsk);
    if ((e = hipGetLastError())) return e;
    // the key's significant bits (codes <= max_code)
    int end_bit = 1;
    while (end_bit < 32 && (max_code >> end_bit)) end_bit++;
    hipcub::DoubleBuffer<uint32_t> kb((uint32_t*)s.keys[0].p, (uint32_t*)s.keys[1].p);
    hipcub::DoubleBuffer<P> pb((P*)s.vals[0].p, (P*)s.vals[1].p);
    size_t tb = 0;
    if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kb, pb, (int)m, 0, end_bit, stream))) return e;
    if ((e = s.temp.reserve(tb))) return e;
    if ((e = hipcub::DeviceRadixSort::SortPairs(s.temp.p, tb, kb, pb, (int)m, 0, end_bit, stream))) return e;
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
        const size_t cw = pairs ? 0 : (cm == kCountLds ? (size_t)a.n_polygons : (size_t)(blk / 64) * kWaveHashWords);
        const size_t shm = ((size_t)iw + cw) * 4;
        if (pairs)
            hipLaunchKernelGGL((k_join_tiles<kCountGlobal, true, P>), dim3(gt), dim3(blk), shm, stream, a, keys, pts, m, nsk, img, iw);
        else if (cm == kCountLds)
            hipLaunchKernelGGL((k_join_tiles<kCountLds, false, P>), dim3(gt), dim3(blk), shm, stream, a, keys, pts, m, nsk, img, iw);
        else
            hipLaunchKernelGGL((k_join_tiles<kCountWaveHash, false, P>), dim3(gt), dim3(blk), shm, stream, a, keys, pts, m, nsk,
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
