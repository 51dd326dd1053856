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
#include <stdint.h>

#include "join_binned.h"
#include "join_chips.h"

using namespace mosaic;

template <class P>
__global__ void __launch_bounds__(256) k_bin_keys(JoinArgs a, int64_t lo, int64_t n, uint32_t* keys, P* pts,
                                                  unsigned long long* n_skip) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    unsigned int skipped = 0;
    for (int64_t i = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const double x = a.x[i], y = a.y[i];
        const uint32_t code = tiles::tile_of(a.tgrid, a.tile_idx, x, y);
        keys[i - lo] = code;
        P p;
        p.x = x;
        p.y = y;
        binned::set_row(p, i);
        pts[i - lo] = p;
        skipped += code == tiles::kSkip;
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

namespace binned {

template <class P>
static hipError_t sort_and_join(const JoinArgs& a0, int64_t lo, int64_t n, uint32_t max_code, int cm, int n_cu,
                                Scratch& s, hipStream_t stream) {
    const int64_t m = n - lo;
    const size_t vb = sizeof(P);
    hipError_t e;
    if ((e = s.keys[0].reserve((size_t)m * 4)) || (e = s.keys[1].reserve((size_t)m * 4)) ||
        (e = s.vals[0].reserve((size_t)m * vb)) || (e = s.vals[1].reserve((size_t)m * vb)) || (e = s.n_skip.reserve(8)))
        return e;
    if ((e = hipMemsetAsync(s.n_skip.p, 0, 8, stream))) return e;
    unsigned long long* nsk = (unsigned long long*)s.n_skip.p;
    const int gk = (int)std::max<int64_t>(1, std::min<int64_t>((m + 255) / 256, (int64_t)n_cu * 8));
    hipLaunchKernelGGL((k_bin_keys<P>), dim3(gk), dim3(256), 0, stream, a0, lo, n, (uint32_t*)s.keys[0].p,
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
    if (pairs) {
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

hipError_t join(const JoinArgs& a, int64_t lo, int64_t n, uint32_t max_code, bool lds_counts, int n_cu, Scratch& s,
                hipStream_t stream) {
    const int cm = lds_counts ? kCountLds : kCountWaveHash;
    if (a.pair_row) return sort_and_join<PtRow>(a, lo, n, max_code, cm, n_cu, s, stream);
    return sort_and_join<Pt>(a, lo, n, max_code, cm, n_cu, s, stream);
}

}  // namespace binned
