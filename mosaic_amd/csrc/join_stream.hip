// The stream kernels of the point-raster join: k_join_stream / k_join_stream_pipe (H3 tile
// directory + point raster, tiles.h) and k_join_stream_bng (BNG dense cell table).  A translation
// unit of their own (the host side that builds their arguments and launches them is mosaic_hip.hip).
#include "join_binned.h"
#include "join_common.h"

// ---- k_join_stream (default with a point raster, tiles.h): the point raster's answer for every
// point of the batch, branch-free.  Per point: fine-cell coordinates (two f64 ops per axis, clamped
// to the grid), the LDS quad level, and -- only for points whose quad is not uniform -- one 2-byte
// gather of the sub-block entry from the compact copies; points whose sub-block is a leaf block or
// a line record gather that (2 or 16 bytes).  Gathers go through buffer descriptors: a lane that
// needs no gather passes an out-of-range offset, which the hardware drops without a memory access,
// so no lane branches.  Answers: 0 (no pair), k + 1 (one pair with key k: an LDS atomic), kMixed
// (the row goes to the mixed queue for k_join_mixed).  tiles::raster_code is the same computation
// for one point on the host.
//
// Rows: each wave handles 256 consecutive rows per iteration; lane l holds rows 2l, 2l + 1,
// 128 + 2l, 129 + 2l, so each 16-byte coordinate load instruction reads 1 KiB contiguous.  The
// next iteration's coordinates are loaded after this iteration's gathers are issued (vector-memory
// returns retire in order: waiting for the gathers does not wait for them).
template <bool LDS_COUNTS, bool PAIRS, bool VEC>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4))) k_join_stream(JoinArgs a, StreamArgs s) {
    extern __shared__ unsigned int lds[];
    const int nwaves = (int)(blockDim.x >> 6);
    const int ncw = LDS_COUNTS ? a.n_polygons + 64 : 0;  // counts + one spill word per lane
    uint32_t* stage = lds + ncw;
    uint32_t* tb = stage + nwaves * s.stage_words;
    uint32_t* quadw = tb + (s.tb_lds ? s.n_tiles : 0);
    const uint16_t* quad = (const uint16_t*)quadw;
    uint32_t* qmask = quadw + s.n_quad_words;
    const uint16_t* qcode = (const uint16_t*)(qmask + 2 * s.n_qrec);
    lds_fill(quadw, s.quad, s.n_quad_words);
    lds_fill(qmask, s.qrec, s.n_qrec_words);
    if (s.tb_lds)
        lds_fill(tb, s.tile_base, s.n_tiles);
    for (int k = threadIdx.x; k < ncw; k += blockDim.x) lds[k] = 0;
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rsub = stream_rsrc(s.csub, s.csub_bytes);
    const __amdgpu_buffer_rsrc_t rblk = stream_rsrc(s.blocks, s.blocks_bytes);
    const __amdgpu_buffer_rsrc_t rtb = stream_rsrc(s.tile_base, s.tile_base_bytes);
    const int lane = (int)(threadIdx.x & 63);
    const unsigned long long lt_mask = (1ULL << lane) - 1ULL;
    // the wave index through readfirstlane: w0 and every branch on it are provably wave-uniform
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    uint32_t* wq = stage + wave * s.stage_words;
    uint32_t wn = 0;  // wave-uniform fill level of the stage
    const uint32_t cm = (1u << s.cs) - 1u, qm = (1u << s.qs) - 1u, tm = (1u << s.tsh) - 1u;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
    int64_t w0 = a.row_lo + ((int64_t)blockIdx.x * blockDim.x + (int64_t)wave * 64) * 4;
    // rows of slot k: w0 + (k >> 1) 128 + 2 lane + (k & 1)
    auto row_of = [&](int64_t wb, int k) -> int64_t { return wb + (k >> 1) * 128 + 2 * lane + (k & 1); };
    v2d px[2], py[2];
    auto load4 = [&](int64_t wb) {  // unconditional: past the end, the chunk's first rows (VEC: >= 256 of them)
        const int64_t r = (wb + 256 <= a.n) ? wb + 2 * lane : a.row_lo;
        px[0] = __builtin_nontemporal_load((const v2d*)(a.x + r));
        px[1] = __builtin_nontemporal_load((const v2d*)(a.x + r + 128));
        py[0] = __builtin_nontemporal_load((const v2d*)(a.y + r));
        py[1] = __builtin_nontemporal_load((const v2d*)(a.y + r + 128));
    };
    if (VEC) load4(w0);
    for (; w0 < a.n; w0 += stride) {
        const bool full = VEC && w0 + 256 <= a.n;  // wave-uniform
        double x[4], y[4];
        bool live[4];
        if (full) {
            x[0] = px[0].x, x[1] = px[0].y, x[2] = px[1].x, x[3] = px[1].y;
            y[0] = py[0].x, y[1] = py[0].y, y[2] = py[1].x, y[3] = py[1].y;
#pragma unroll
            for (int k = 0; k < 4; k++) live[k] = true;
        } else {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int64_t r = row_of(w0, k);
                live[k] = r < a.n;
                x[k] = live[k] ? a.x[r] : 0.0;
                y[k] = live[k] ? a.y[r] : 0.0;
            }
        }
        // stage A: fine-cell coordinates, quad level (LDS), tile base (LDS)
        double gx[4], gy[4];
        uint32_t ixC[4], iyC[4], qv[4], tbv[4], ta[4];
        bool fin[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            fin[k] = __builtin_isfinite(x[k] + y[k]);
            gx[k] = fmin(fmax((x[k] - s.x0) * s.sxC, 0.0), s.gxmax);  // NaN -> 0
            gy[k] = fmin(fmax((y[k] - s.y0) * s.syC, 0.0), s.gymax);
            ixC[k] = (uint32_t)(int)gx[k];
            iyC[k] = (uint32_t)(int)gy[k];
            // (indices < 2^24: 24-bit multiplies)
            qv[k] = quad_lookup(s, quad, qmask, qcode, ixC[k], iyC[k]);
            ta[k] = __umul24(iyC[k] >> s.tsh, (uint32_t)s.tnx) + (ixC[k] >> s.tsh);
            tbv[k] = s.tb_lds ? tb[ta[k]] : 0u;
        }
        // stage B: sub-block entries of the points in non-uniform quads
        uint32_t code[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t local = (((iyC[k] >> s.cs) & qm) << s.qs) | ((ixC[k] >> s.cs) & qm);
            const uint32_t off = ((((qv[k] & 0x7fffu) << (2 * s.qs)) + local) << 1);
            code[k] = __builtin_amdgcn_raw_buffer_load_b16(rsub, qv[k] >= 0x8000u ? off : kNoLoad, 0, 0);
        }
        // stage C: leaf codes and line records of the points in mixed sub-blocks
        uint32_t leaf[4];
        v4u lrec[4];
        bool blk[4], line[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            code[k] = qv[k] >= 0x8000u ? code[k] : qv[k];
            blk[k] = code[k] - 0x8000u < 0x7fffu;  // kSubBlock | n, not kMixed
            line[k] = blk[k] && (code[k] & 0x4000u);
            if (!s.tb_lds) tbv[k] = __builtin_amdgcn_raw_buffer_load_b32(rtb, blk[k] ? ta[k] << 2 : kNoLoad, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t n = code[k] & 0x3fffu;
            const uint32_t lf = ((iyC[k] & cm) << s.cs) | (ixC[k] & cm);
            const uint32_t loff = (tbv[k] + (n << (2 * s.cs)) + lf) << 1;
            const uint32_t roff = (tbv[k] - 8u * (n + 1u)) << 1;
            leaf[k] = __builtin_amdgcn_raw_buffer_load_b16(rblk, (blk[k] && !line[k]) ? loff : kNoLoad, 0, 0);
            lrec[k] = __builtin_amdgcn_raw_buffer_load_b128(rblk, line[k] ? roff : kNoLoad, 0, 0);
        }
        if (VEC) load4(w0 + stride);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            // tiles::line_code, as selects
            // (offsets from the tile's corner: line records are in the tile frame)
            const float u = (float)(gx[k] - (double)(ixC[k] & ~tm)), v = (float)(gy[k] - (double)(iyC[k] & ~tm));
            const float sv = fmaf(__uint_as_float(lrec[k].x), u, fmaf(__uint_as_float(lrec[k].y), v, __uint_as_float(lrec[k].z)));
            const uint32_t pos = lrec[k].w & 0xffffu, neg = lrec[k].w >> 16;
            uint32_t lc = sv >= 1.0f ? pos : (uint32_t)tiles::kMixed;
            lc = sv <= -1.0f ? neg : lc;
            uint32_t c = line[k] ? lc : (blk[k] ? leaf[k] : code[k]);
            c = fin[k] && c < 0x8000u ? c : (uint32_t)tiles::kMixed;  // (leaf lines: the mixed kernel)
            code[k] = live[k] ? c : 0u;
        }
        // counts: one LDS add per point (points without a pair add to the lane's spill word)
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (LDS_COUNTS && !PAIRS) {
                const uint32_t slot = code[k] - 1u < 0xfffeu ? code[k] - 1u : (uint32_t)(a.n_polygons + lane);
                atomicAdd(&lds[slot], 1u);
            } else if (code[k] - 1u < 0xfffeu) {
                emit_hit<LDS_COUNTS, PAIRS>(a, row_of(w0, k), code[k] - 1u, lds);
            }
        }
        // mixed rows to the per-wave stage (rare: one wave-uniform test per iteration)
        const bool anym = code[0] == tiles::kMixed || code[1] == tiles::kMixed || code[2] == tiles::kMixed ||
                          code[3] == tiles::kMixed;
        if (__ballot(anym)) {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const bool m = code[k] == tiles::kMixed;
                const unsigned long long mm = __ballot(m);
                if (m) wq[wn + __popcll(mm & lt_mask)] = (uint32_t)(row_of(w0, k) - a.row_lo);
                wn += (uint32_t)__popcll(mm);
                stage_flush(a, wq, wn, lane, 64);  // one atomic per >= 64 rows; the stage holds < 128
            }
        }
    }
    stage_flush(a, wq, wn, lane, 1);
    if (LDS_COUNTS) {
        __syncthreads();
        for (int k = threadIdx.x; k < a.n_polygons; k += blockDim.x)
            if (lds[k]) atomicAdd(&a.counts[k], (unsigned long long)lds[k]);
    }
}


// Gathers of the pipelined stream kernels, only by the lanes that need one (exec-masked; a wave with
// no such lane skips the instruction).  Measured against passing an out-of-range offset from the
// other lanes (branch-free) and against that plus a wave-uniform skip: C2 stream 3.47 / 3.52 ->
// 3.40 ms (profiles/r03_kbench_gather_modes.txt) -- the texture units and the data return path do
// no work for inactive lanes.
template <int aux>
__device__ inline uint32_t gather_b16(__amdgpu_buffer_rsrc_t r, bool need, uint32_t off) {
    uint32_t v = 0u;
    if (need) v = __builtin_amdgcn_raw_buffer_load_b16(r, off, 0, aux);
    return v;
}
__device__ inline uint32_t gather_b32(__amdgpu_buffer_rsrc_t r, bool need, uint32_t off) {
    uint32_t v = 0u;
    if (need) v = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
    return v;
}
template <int aux>
__device__ inline v4u gather_b128(__amdgpu_buffer_rsrc_t r, bool need, uint32_t off) {
    v4u v = {0u, 0u, 0u, 0u};
    if (need) v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, aux);
    return v;
}

// ---- k_join_stream_pipe: k_join_stream's per-point computation as a three-stage software
// pipeline over the wave's groups of 256 rows, so that the gathers of one group overlap the
// coordinate loads of the next instead of adding to them.  Iteration t: finish group t - 2 (its leaf
// codes / line records arrived), turn group t - 1's sub-block entries into leaf and line gathers,
// run group t's coordinates through the quad level and issue its sub-block gathers, and load group
// t + 1's coordinates -- issued in that order, so every wait is on the oldest loads in flight
// (vector-memory returns retire in order per wave).  Needs 16-byte aligned columns, tile_base in
// LDS and at least one full group; the wave's last partial group runs unpipelined.  Same answers
// as k_join_stream, point for point.  Fine-cell coordinates in fixed point
// (tiles::raster_code_fixed): one f64 fma, one saturating conversion and an integer clamp per axis,
// every index a bit-field of the result.  The pipe kernel serves the rasters k_join_stream_cpt
// cannot take (cs + qs > 8, more than 65,536 tiles, no LDS room for the compaction buffers).
struct PipeGroup {
    uint32_t gx[4], gy[4];  // fixed-point fine-cell coordinates (kFixBits fraction bits)
    uint32_t tbv[4];      // tile base
    uint32_t qv[4];       // quad-level entry
    uint32_t code[4];     // sub-block entry (gathered), then the answer
    uint32_t leaf[4];     // gathered leaf code
    v4u lrec[4];          // gathered line record
};
// quad-level value standing for "non-finite coordinates" in a group (never a code: codes are
// <= kMaxRasterKeys + 1 or >= kSubBlock): the row takes the tile path
static const uint32_t kPipeNonFinite = 0x7fffu;
static_assert(tiles::kMaxRasterKeys + 1 < 0x7fff, "key codes stay below kPipeNonFinite");
// stage B -> D marker of a row in a line sub-block (above every code)
static const uint32_t kPipeLine = 0x10000u;

template <bool LDS_COUNTS, bool PAIRS>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4))) k_join_stream_pipe(JoinArgs a, StreamArgs s) {
    extern __shared__ unsigned int lds[];
    const int nwaves = (int)(blockDim.x >> 6);
    const int ncw = LDS_COUNTS ? a.n_polygons + 64 : 0;
    uint32_t* stage = lds + ncw;
    uint32_t* tb = stage + nwaves * s.stage_words;
    uint32_t* quadw = tb + s.n_tiles;
    const uint16_t* quad = (const uint16_t*)quadw;
    uint32_t* qmask = quadw + s.n_quad_words;
    const uint16_t* qcode = (const uint16_t*)(qmask + 2 * s.n_qrec);
    lds_fill(quadw, s.quad, s.n_quad_words);
    lds_fill(qmask, s.qrec, s.n_qrec_words);
    lds_fill(tb, s.tile_base, s.n_tiles);
    for (int k = threadIdx.x; k < ncw; k += blockDim.x) lds[k] = 0;
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rsub = stream_rsrc(s.csub, s.csub_bytes);
    const __amdgpu_buffer_rsrc_t rblk = stream_rsrc(s.blocks, s.blocks_bytes);
    const int lane = (int)(threadIdx.x & 63);
    const unsigned long long lt_mask = (1ULL << lane) - 1ULL;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    uint32_t* wq = stage + wave * s.stage_words;
    uint32_t wn = 0;
    const uint32_t cm = (1u << s.cs) - 1u, qm = (1u << s.qs) - 1u;
    const double gx0 = -s.x0 * s.sxC, gy0 = -s.y0 * s.syC;
    const uint32_t spill = (uint32_t)(a.n_polygons + lane);  // the lane's spill word (LDS counts)
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
    const int64_t wbase = a.row_lo + ((int64_t)blockIdx.x * blockDim.x + (int64_t)wave * 64) * 4;
    // full groups of this wave: wbase + t stride, t < T
    const int64_t T = wbase + 256 <= a.n ? (a.n - 256 - wbase) / stride + 1 : 0;
    auto row_of = [&](int64_t wb, int k) -> int64_t { return wb + (k >> 1) * 128 + 2 * lane + (k & 1); };
    // stage A: coordinates -> fine cell, quad level and tile base (LDS) -> sub-block gathers
    auto stage_a = [&](const double* x, const double* y, const bool* live, bool valid, PipeGroup& g) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const bool lv = valid && live[k];
            // fixed point (tiles::raster_code_fixed): saturating conversion (negative, NaN -> 0), clamp
            const uint32_t ixC = min(tiles::fix_cvt(fma(x[k], s.sxF, s.gx0F)), (uint32_t)s.gxmaxF);
            const uint32_t iyC = min(tiles::fix_cvt(fma(y[k], s.syF, s.gy0F)), (uint32_t)s.gymaxF);
            g.gx[k] = ixC;
            g.gy[k] = iyC;
            constexpr int SH0 = tiles::kFixBits;
            const uint32_t q = quad_lookup<SH0>(s, quad, qmask, qcode, ixC, iyC);
            // dead rows answer 0.  Non-finite coordinates need no test: fmax / fmin clamp them onto
            // the grid's edge ring, whose sub-blocks are all 0 or kMixed (PointRaster edge_ok, a
            // precondition of this kernel), and a non-finite point joins nothing in the reference
            // (geoToH3 gives H3_NULL) -- 0 is its answer, kMixed sends it to the exact path.
            g.qv[k] = lv ? q : 0u;
            g.tbv[k] = tb[__umul24(iyC >> (s.tsh + SH0), (uint32_t)s.tnx) + (ixC >> (s.tsh + SH0))];
            const uint32_t local = (__builtin_amdgcn_ubfe(iyC, (uint32_t)(s.cs + SH0), (uint32_t)s.qs) << s.qs) |
                                   __builtin_amdgcn_ubfe(ixC, (uint32_t)(s.cs + SH0), (uint32_t)s.qs);
            const uint32_t off = ((((g.qv[k] & 0x7fffu) << (2 * s.qs)) + local) << 1);
            g.code[k] = gather_b16<0>(rsub, g.qv[k] >= 0x8000u, off);
        }
    };
    // stage B: sub-block entries -> leaf and line gathers
    auto stage_b = [&](PipeGroup& g) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t c = g.qv[k] >= 0x8000u ? g.code[k] : g.qv[k];
            const bool blk = c - 0x8000u < 0x7fffu;  // kSubBlock | n, not kMixed
            const bool line = blk && (c & 0x4000u);
            const uint32_t n = c & 0x3fffu;
            const uint32_t lf = (__builtin_amdgcn_ubfe(g.gy[k], (uint32_t)tiles::kFixBits, (uint32_t)s.cs) << s.cs) |
                                __builtin_amdgcn_ubfe(g.gx[k], (uint32_t)tiles::kFixBits, (uint32_t)s.cs);
            const uint32_t loff = (g.tbv[k] + (n << (2 * s.cs)) + lf) << 1;
            const uint32_t roff = (g.tbv[k] - 8u * (n + 1u)) << 1;
            g.leaf[k] = gather_b16<0>(rblk, blk && !line, loff);
            g.lrec[k] = gather_b128<0>(rblk, line, roff);
            // for stage D: kPipeLine for a line row, else the code to OR with the gathered leaf code
            // (0 for leaf rows; out-of-range gathers return 0)
            g.code[k] = line ? kPipeLine : (blk ? 0u : c);
        }
    };
    // stage D: the answers -> counts and the mixed-row stage
    auto stage_d = [&](PipeGroup& g, int64_t wb) {
        uint32_t code[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            // the offset in the tile (line records are in the tile frame), leaf cells, truncated to
            // 2^-kFixBits (exact in f32)
            const uint32_t fb = (uint32_t)(s.tsh + tiles::kFixBits);
            const float u = (float)__builtin_amdgcn_ubfe(g.gx[k], 0u, fb) * (1.0f / (float)(1 << tiles::kFixBits));
            const float v = (float)__builtin_amdgcn_ubfe(g.gy[k], 0u, fb) * (1.0f / (float)(1 << tiles::kFixBits));
            const float sv = fmaf(__uint_as_float(g.lrec[k].x), u,
                                  fmaf(__uint_as_float(g.lrec[k].y), v, __uint_as_float(g.lrec[k].z)));
            const uint32_t pos = g.lrec[k].w & 0xffffu, neg = g.lrec[k].w >> 16;
            uint32_t lc = sv >= 1.0f ? pos : (uint32_t)tiles::kMixed;
            lc = sv <= -1.0f ? neg : lc;
            // answers: 0, key + 1 (<= kMaxRasterKeys), or >= kPipeNonFinite (kMixed, non-finite):
            // the tile path
            code[k] = g.code[k] == kPipeLine ? lc : (g.code[k] | g.leaf[k]);
        }
        // counts: one LDS add per point (points without a pair add to the lane's spill word: a
        // masked add measured slower on clustered input)
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (LDS_COUNTS && !PAIRS) {
                // keys are < n_polygons <= 8192; 0 (no pair) wraps to 0xffffffff and kMixed / non-finite
                // codes are >= kPipeNonFinite: both land on the lane's spill word
                const uint32_t slot = min(code[k] - 1u, spill);
                atomicAdd(&lds[slot], 1u);
            } else if (code[k] - 1u < kPipeNonFinite - 1u) {
                emit_hit<LDS_COUNTS, PAIRS>(a, row_of(wb, k), code[k] - 1u, lds);
            }
        }
        const uint32_t cmax = max(max(code[0], code[1]), max(code[2], code[3]));
        if (__ballot(cmax >= kPipeNonFinite)) {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const bool m = code[k] >= kPipeNonFinite;
                const unsigned long long mm = __ballot(m);
                if (m) wq[wn + __popcll(mm & lt_mask)] = (uint32_t)(row_of(wb, k) - a.row_lo);
                wn += (uint32_t)__popcll(mm);
                stage_flush(a, wq, wn, lane, 64);  // the stage holds < 128
            }
        }
    };
    // coordinates of the next group (loaded one iteration ahead; two ahead measured slower:
    // registers, profiles/r03_kbench_pipe_depth.txt)
    struct Coords {
        v2d px[2], py[2];
    };
    auto load4 = [&](Coords& cb, int64_t wb, bool valid) {  // unconditional: invalid groups re-read the wave's first rows
        const int64_t r = valid ? wb + 2 * lane : wbase + 2 * lane;
        cb.px[0] = __builtin_nontemporal_load((const v2d*)(a.x + r));
        cb.px[1] = __builtin_nontemporal_load((const v2d*)(a.x + r + 128));
        cb.py[0] = __builtin_nontemporal_load((const v2d*)(a.y + r));
        cb.py[1] = __builtin_nontemporal_load((const v2d*)(a.y + r + 128));
    };
    Coords cb0, cb1;
    // two group slots used in turn (no copies of registers that loads are still landing in):
    // iteration t finishes the slot holding t - 2, advances the one holding t - 1, refills the first
    PipeGroup g0, g1;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        g0.qv[k] = g1.qv[k] = 0u;
        g0.code[k] = g1.code[k] = 0u;
        g0.tbv[k] = g1.tbv[k] = 0u;
        g0.gx[k] = g1.gx[k] = g0.gy[k] = g1.gy[k] = 0u;
    }
    // VALID: group t is a full group of this wave (t < T) -- a compile-time constant, so the main loop
    // carries no per-point validity test (only the two drain steps run with VALID false)
    auto step = [&](auto VALID, int64_t t, PipeGroup& gfin, PipeGroup& gadv, Coords& cb, Coords& cn) {
        const bool all[4] = {true, true, true, true};
        if (t >= 2) stage_d(gfin, wbase + (t - 2) * stride);
        stage_b(gadv);  // (invalid groups gather nothing)
        const double x[4] = {cb.px[0].x, cb.px[0].y, cb.px[1].x, cb.px[1].y};
        const double y[4] = {cb.py[0].x, cb.py[0].y, cb.py[1].x, cb.py[1].y};
        stage_a(x, y, all, decltype(VALID)::value, gfin);
        load4(cn, wbase + (t + 1) * stride, t + 1 < T);
    };
    if (T > 0) {
        load4(cb0, wbase, true);
        const std::true_type full;
        const std::false_type drain;
        int64_t t = 0;
        for (; t + 2 <= T; t += 2) {
            step(full, t, g0, g1, cb0, cb1);
            step(full, t + 1, g1, g0, cb1, cb0);
        }
        // groups t .. T - 1 (none or one) and the two drain steps (t = T, T + 1)
        if (t < T) {
            step(full, t, g0, g1, cb0, cb1);
            step(drain, t + 1, g1, g0, cb1, cb0);
            step(drain, t + 2, g0, g1, cb0, cb1);
        } else {
            step(drain, t, g0, g1, cb0, cb1);
            step(drain, t + 1, g1, g0, cb1, cb0);
        }
    }
    // the wave's partial group (rows past its last full group), unpipelined
    const int64_t wt = wbase + T * stride;
    if (wt < a.n) {
        double x[4], y[4];
        bool live[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int64_t r = row_of(wt, k);
            live[k] = r < a.n;
            x[k] = live[k] ? a.x[r] : 0.0;
            y[k] = live[k] ? a.y[r] : 0.0;
        }
        PipeGroup g;
        stage_a(x, y, live, true, g);
        stage_b(g);
        stage_d(g, wt);
    }
    stage_flush(a, wq, wn, lane, 1);
    if (LDS_COUNTS) {
        __syncthreads();
        for (int k = threadIdx.x; k < a.n_polygons; k += blockDim.x)
            if (lds[k]) atomicAdd(&a.counts[k], (unsigned long long)lds[k]);
    }
}


// ---- k_join_stream_cpt: k_join_stream_pipe with the rows that need gathers compacted.  87.6 % of
// uniform NYC points are decided by the LDS levels alone (the quad level and its records), yet the
// pipe kernel runs the sub-block / leaf / line stages -- about half of its VALU instructions -- on all
// 256 rows of every group, since a wave instruction costs the same however few lanes need it.  Here
// stage A decides and counts the LDS-resolved rows at once and moves the others ("pending": quad entry
// >= 0x8000) into one 64-lane set with ds_permute (no LDS memory: per row slot k, a rotation of the
// stable partition pending / not pending, so every lane sends and receives exactly one value); the
// set's sub-block gather, leaf / line gathers and answers then take one lane per pending row.  The
// set is software-pipelined like the pipe kernel's groups (iteration t: finish the set of t - 2, turn
// the set of t - 1's sub-block entries into leaf / line gathers, run group t through the LDS levels,
// compact it and gather its sub-block entries, load group t + 1).  Pending rows beyond 64 in a group
// (clustered input) are finished at once, unpipelined.  Per pending row the set carries: the low L =
// cs + kFixBits + qs bits of both fixed-point fine-cell coordinates (leaf cell, line offsets and the
// sub-block within the quad; L <= 24), the source lane and row slot, the quad entry and the tile.
// Same answers as k_join_stream_pipe, point for point.
// 1: a group's second set of pending rows (65 - 128) is pipelined like the first
// 1: compaction through a per-wave LDS buffer; 0: ds_permute (no LDS memory)
struct CptSet {
    uint32_t a;     // ix low bits | source lane << 24 | row slot k << 30
    uint32_t b;     // iy low bits
    uint32_t c;     // quad entry | tile index << 16
    uint32_t code;  // A -> B: gathered sub-block entry; B -> D: the answer, 0 for leaf rows, or kPipeLine
    uint32_t leaf;  // gathered leaf code
    v4u lrec;       // gathered line record
};

template <bool LDS_COUNTS, bool PAIRS>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4))) k_join_stream_cpt(JoinArgs a, StreamArgs s) {
    extern __shared__ unsigned int lds[];
    const int nwaves = (int)(blockDim.x >> 6);
    const int ncw = LDS_COUNTS ? a.n_polygons + 64 : 0;
    uint32_t* stage = lds + ncw;
    // per-wave compaction buffers: 64 slots x 3 words, structure of arrays
    uint32_t* cbuf_all = stage + nwaves * s.stage_words;
    // tile bases in LDS (s.tb_lds), or gathered beside the sub-block entry (large tile grids: their
    // LDS goes to a finer quad level instead)
    uint32_t* tb = cbuf_all + nwaves * kCptBufWords;
    uint32_t* quadw = tb + (s.tb_lds ? s.n_tiles : 0);
    const uint16_t* quad = (const uint16_t*)quadw;
    uint32_t* qmask = quadw + s.n_quad_words;
    const uint16_t* qcode = (const uint16_t*)(qmask + 2 * s.n_qrec);
    lds_fill(quadw, s.quad, s.n_quad_words);
    lds_fill(qmask, s.qrec, s.n_qrec_words);
    if (s.tb_lds) lds_fill(tb, s.tile_base, s.n_tiles);
    for (int k = threadIdx.x; k < ncw; k += blockDim.x) lds[k] = 0;
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rsub = stream_rsrc(s.csub, s.csub_bytes);
    const __amdgpu_buffer_rsrc_t rblk = stream_rsrc(s.blocks, s.blocks_bytes);
    const __amdgpu_buffer_rsrc_t rtb = stream_rsrc(s.tile_base, s.tile_base_bytes);
    const bool tb_lds = s.tb_lds != 0;
    const int lane = (int)(threadIdx.x & 63);
    const unsigned long long lt_mask = (1ULL << lane) - 1ULL;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    uint32_t* wq = stage + wave * s.stage_words;
    uint32_t* cbuf = cbuf_all + wave * kCptBufWords;
    uint32_t wn = 0;
    constexpr int F = tiles::kFixBits;
    const uint32_t cs = (uint32_t)s.cs, qs = (uint32_t)s.qs;
    // low bits carried per pending row: the sub-block within the quad and, for the line test, the
    // offset in the tile (line records are in the tile frame)
    const uint32_t lowm = (1u << max(cs + F + qs, (uint32_t)s.tsh + F)) - 1u;
    const uint32_t spill = (uint32_t)(a.n_polygons + lane);
    // the fixed-point offsets in VGPRs for the whole kernel (an fma reads one scalar operand; as
    // scalars they would be copied into VGPRs at every point)
    double gx0v, gy0v;
    __asm__("v_mov_b64 %0, %1" : "=v"(gx0v) : "s"(s.gx0F));
    __asm__("v_mov_b64 %0, %1" : "=v"(gy0v) : "s"(s.gy0F));
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
    const int64_t wbase = a.row_lo + ((int64_t)blockIdx.x * blockDim.x + (int64_t)wave * 64) * 4;
    const int64_t T = wbase + 256 <= a.n ? (a.n - 256 - wbase) / stride + 1 : 0;
    // a row's answer: count it (LDS) or emit the pair; kMixed / non-finite rows (>= kPipeNonFinite)
    // are returned to the caller's mixed-row stage
    auto answer = [&](uint32_t code, int64_t row) {
        if (LDS_COUNTS && !PAIRS) {
            atomicAdd(&lds[min(code - 1u, spill)], 1u);  // 0 wraps, mixed codes >= kPipeNonFinite: spill
        } else if (code - 1u < kPipeNonFinite - 1u) {
            emit_hit<LDS_COUNTS, PAIRS>(a, row, code - 1u, lds);
        }
    };
    // --- set stages
    // A: the sub-block gather (pending rows: quad entry >= 0x8000), and without tile bases in LDS
    // the tile base beside it (carried to B in z.leaf)
    auto set_a = [&](CptSet& z) {
        const uint32_t q = z.c & 0xffffu;
        const uint32_t local = (__builtin_amdgcn_ubfe(z.b, cs + F, qs) << qs) | __builtin_amdgcn_ubfe(z.a, cs + F, qs);
        uint32_t off = (((q & 0x7fffu) << (2 * qs)) + local) << 1;
#ifdef MOSAIC_ABL_GATHER_HIT
        if (MOSAIC_ABL_GATHER_HIT & 4) off &= 0xffeu;
#endif
        z.code = gather_b16<0>(rsub, q >= 0x8000u, off);
        if (!tb_lds) z.leaf = gather_b32(rtb, q >= 0x8000u, (z.c >> 16) << 2);
    };
    // B: sub-block entry -> leaf / line gather
    auto set_b = [&](CptSet& z) {
        const uint32_t q = z.c & 0xffffu;
        const uint32_t c = q >= 0x8000u ? z.code : q;
        const bool blk = c - 0x8000u < 0x7fffu;
        const bool line = blk && (c & 0x4000u);
        const uint32_t n = c & 0x3fffu;
        const uint32_t lf = (__builtin_amdgcn_ubfe(z.b, (uint32_t)F, cs) << cs) | __builtin_amdgcn_ubfe(z.a, (uint32_t)F, cs);
        const uint32_t tbv = tb_lds ? tb[z.c >> 16] : z.leaf;
        uint32_t loff = (tbv + (n << (2 * cs)) + lf) << 1;
        uint32_t roff = (tbv - 8u * (n + 1u)) << 1;
#ifdef MOSAIC_ABL_GATHER_HIT  // measurement builds only: the leaf / line gathers within 4 KB (wrong answers)
#ifdef MOSAIC_ABL_LMASK
        if (MOSAIC_ABL_GATHER_HIT & 1) roff &= (uint32_t)MOSAIC_ABL_LMASK;
#else
        if (MOSAIC_ABL_GATHER_HIT & 1) roff &= 0xff0u;
#endif
        if (MOSAIC_ABL_GATHER_HIT & 2) loff &= 0xffeu;
#endif
        z.leaf = gather_b16<0>(rblk, blk && !line, loff);
        z.lrec = gather_b128<0>(rblk, line, roff);
        z.code = line ? kPipeLine : (blk ? 0u : c);
    };
    // D: answers of the set's rows (group base wb)
    auto set_d = [&](CptSet& z, int64_t wb) {
        const uint32_t fb = (uint32_t)s.tsh + (uint32_t)F;
#ifdef MOSAIC_ABL_GATHER_HIT  // (measurement builds) wait for the gathers, then answer key 0
        __asm__ volatile("" ::"v"(z.lrec.x), "v"(z.lrec.y), "v"(z.lrec.z), "v"(z.lrec.w), "v"(z.leaf));
        if (MOSAIC_ABL_GATHER_HIT & 9) z.lrec = v4u{0u, 0u, __float_as_uint(2.0f), 0x00010001u};
        if (MOSAIC_ABL_GATHER_HIT & 10) z.leaf = z.code == kPipeLine ? z.leaf : 1u;
#endif
        const float u = (float)__builtin_amdgcn_ubfe(z.a, 0u, fb) * (1.0f / (float)(1 << F));
        const float v = (float)__builtin_amdgcn_ubfe(z.b, 0u, fb) * (1.0f / (float)(1 << F));
        const float sv = fmaf(__uint_as_float(z.lrec.x), u, fmaf(__uint_as_float(z.lrec.y), v, __uint_as_float(z.lrec.z)));
        const uint32_t pos = z.lrec.w & 0xffffu, neg = z.lrec.w >> 16;
        uint32_t lc = sv >= 1.0f ? pos : (uint32_t)tiles::kMixed;
        lc = sv <= -1.0f ? neg : lc;
        const uint32_t code = z.code == kPipeLine ? lc : (z.code | z.leaf);
        const uint32_t src = (z.a >> 24) & 63u, k = z.a >> 30;
        const int64_t row = wb + (int64_t)((k >> 1) * 128u + 2u * src + (k & 1u));
        answer(code, row);
        const bool m = code >= kPipeNonFinite;
        if (__ballot(m)) {
            const unsigned long long mm = __ballot(m);
            if (m) wq[wn + __popcll(mm & lt_mask)] = (uint32_t)(row - a.row_lo);
            wn += (uint32_t)__popcll(mm);
            stage_flush(a, wq, wn, lane, 64);  // the stage holds < 128
        }
    };
    // --- stage A of a group: LDS levels, resolved rows answered, pending rows compacted into z (the
    // first 64); more than 64 pending rows: the rest finished here
    auto stage_a = [&](const double* x, const double* y, const bool* live, bool valid, CptSet& z, CptSet& z2, bool& two,
                       int64_t wb) {
        uint32_t fa[4], fb[4], fc[4];
        bool pend[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t ixC = min(tiles::fix_cvt(fma(x[k], s.sxF, gx0v)), (uint32_t)s.gxmaxF);
            const uint32_t iyC = min(tiles::fix_cvt(fma(y[k], s.syF, gy0v)), (uint32_t)s.gymaxF);
            const uint32_t q0 = quad_lookup<F>(s, quad, qmask, qcode, ixC, iyC);
            const uint32_t q = valid && live[k] ? q0 : 0u;
            const uint32_t tile = mad_u24(iyC >> (s.tsh + F), (uint32_t)s.tnx, ixC >> (s.tsh + F));
            // resolved rows (codes < 0x8000: 0 or key + 1); pending rows add to the spill word now
            // and are counted when their answer is known
            if (LDS_COUNTS && !PAIRS) atomicAdd(&lds[min(q - 1u, spill)], 1u);
            else if (q - 1u < kPipeNonFinite - 1u) emit_hit<LDS_COUNTS, PAIRS>(a, wb + (k >> 1) * 128 + 2 * lane + (k & 1), q - 1u, lds);
            pend[k] = q >= 0x8000u;
            fa[k] = (ixC & lowm) | ((uint32_t)lane << 24) | ((uint32_t)k << 30);
            fb[k] = iyC & lowm;
            fc[k] = q | (tile << 16);
        }
        // compaction through the wave's LDS buffer: row slot k's pending rows take set slots base_k ..
        // base_k + n_k - 1; the rows of set sv (slots 64 sv .. 64 sv + 63) are stored, then read back
        // one per lane
        uint32_t ranks[4], bases[4];
        uint32_t base = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const unsigned long long m = __ballot(pend[k]);
            ranks[k] = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            bases[k] = base;
            base += (uint32_t)__popcll(m);
        }
        const uint32_t P = base;  // pending rows of the group (wave-uniform)
        auto gather_set = [&](uint32_t sv, CptSet& o) {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t slot = ranks[k] - 64u * sv;
                if (pend[k] && slot < 64u) {
                    cbuf[slot] = fa[k];
                    cbuf[64 + slot] = fb[k];
                    cbuf[128 + slot] = fc[k];
                }
            }
            __builtin_amdgcn_wave_barrier();
            const bool ok = 64u * sv + (uint32_t)lane < P;  // empty slots: quad entry 0, answer 0
            o.a = ok ? cbuf[lane] : 0u;
            o.b = ok ? cbuf[64 + lane] : 0u;
            o.c = ok ? cbuf[128 + lane] : 0u;
            __builtin_amdgcn_wave_barrier();
        };
        gather_set(0u, z);
        set_a(z);
        // a second set (65 - 128 pending rows, clustered input) is pipelined too
        two = P > 64u;
        if (two) {
            gather_set(1u, z2);
            set_a(z2);
        }
        if (P > (two ? 128u : 64u)) {  // (wave-uniform) the group's further sets, unpipelined
            for (uint32_t sv = two ? 2 : 1; sv * 64u < P; sv++) {
                CptSet o;
                gather_set(sv, o);
                set_a(o);
                set_b(o);
                set_d(o, wb);
            }
        }
    };
    struct Coords {
        v2d px[2], py[2];
    };
    auto load4 = [&](Coords& cb, int64_t wb, bool valid) {
        const int64_t r = valid ? wb + 2 * lane : wbase + 2 * lane;
        cb.px[0] = __builtin_nontemporal_load((const v2d*)(a.x + r));
        cb.px[1] = __builtin_nontemporal_load((const v2d*)(a.x + r + 128));
        cb.py[0] = __builtin_nontemporal_load((const v2d*)(a.y + r));
        cb.py[1] = __builtin_nontemporal_load((const v2d*)(a.y + r + 128));
    };
    CptSet z0, z1, y0, y1;  // y: the second set of the same group
    bool two0 = false, two1 = false;
    z0.a = z1.a = z0.b = z1.b = z0.c = z1.c = z0.code = z1.code = z0.leaf = z1.leaf = 0u;
    z0.lrec = z1.lrec = v4u{0u, 0u, 0u, 0u};
    // zfin (yfin): the set(s) of t - 2, refilled with group t; zadv (yadv): the set(s) of t - 1
    auto step = [&](auto VALID, int64_t t, CptSet& zfin, CptSet& yfin, bool& tfin, CptSet& zadv, CptSet& yadv, bool tadv,
                    Coords& cb, Coords& cn) {
        const bool all[4] = {true, true, true, true};
        if (t >= 2) {
            set_d(zfin, wbase + (t - 2) * stride);
            if (tfin) set_d(yfin, wbase + (t - 2) * stride);
        }
        set_b(zadv);
        if (tadv) set_b(yadv);
        const double x[4] = {cb.px[0].x, cb.px[0].y, cb.px[1].x, cb.px[1].y};
        const double y[4] = {cb.py[0].x, cb.py[0].y, cb.py[1].x, cb.py[1].y};
        stage_a(x, y, all, decltype(VALID)::value, zfin, yfin, tfin, wbase + t * stride);
        load4(cn, wbase + (t + 1) * stride, t + 1 < T);
    };
    if (T > 0) {
        Coords cb0, cb1;
        const std::true_type full;
        const std::false_type drain;
        int64_t t = 0;
        load4(cb0, wbase, true);
        for (; t + 2 <= T; t += 2) {
            step(full, t, z0, y0, two0, z1, y1, two1, cb0, cb1);
            step(full, t + 1, z1, y1, two1, z0, y0, two0, cb1, cb0);
        }
        if (t < T) {
            step(full, t, z0, y0, two0, z1, y1, two1, cb0, cb1);
            step(drain, t + 1, z1, y1, two1, z0, y0, two0, cb1, cb0);
            step(drain, t + 2, z0, y0, two0, z1, y1, two1, cb0, cb1);
        } else {
            step(drain, t, z0, y0, two0, z1, y1, two1, cb0, cb1);
            step(drain, t + 1, z1, y1, two1, z0, y0, two0, cb1, cb0);
        }
    }
    // the wave's partial group (rows past its last full group), unpipelined
    const int64_t wt = wbase + T * stride;
    if (wt < a.n) {
        double x[4], y[4];
        bool live[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int64_t r = wt + (k >> 1) * 128 + 2 * lane + (k & 1);
            live[k] = r < a.n;
            x[k] = live[k] ? a.x[r] : 0.0;
            y[k] = live[k] ? a.y[r] : 0.0;
        }
        CptSet z, z2;
        bool two = false;
        stage_a(x, y, live, true, z, z2, two, wt);
        set_b(z);
        set_d(z, wt);
        if (two) {
            set_b(z2);
            set_d(z2, wt);
        }
    }
    stage_flush(a, wq, wn, lane, 1);
    if (LDS_COUNTS) {
        __syncthreads();
        for (int k = threadIdx.x; k < a.n_polygons; k += blockDim.x)
            if (lds[k]) atomicAdd(&a.counts[k], (unsigned long long)lds[k]);
    }
}

// k_join_stream_bng: the dense table's answer for every point, branch-free, in the layout of
// k_join_stream (256 rows per wave and iteration, 1 KiB coalesced coordinate loads, the next
// iteration's coordinates loaded behind this iteration's gathers).  Per point: JVM toInt of both
// coordinates, the cell (exact quotients: (int)(a / div + 1e-7) from one f64 multiply-add -- for
// a < 1e7 and div <= 1e5 a non-integer quotient is >= 1 / div below the next integer, far more than
// the 2e-9 the reciprocal and the offset move it), one 4-byte cell gather and, in border cells, one
// 2-byte leaf gather, both through buffer descriptors (lanes that need none pass an out-of-range
// offset).  NaN coordinates set flags bit 0 (the reference throws IllegalStateException).
//
// LDS cell level (when the table is built with one and it fits the workgroup's LDS): one byte per
// 2^lsh x 2^lsh block of table cells, copied to LDS at kernel start -- 0: no chip cell in the block,
// 1..0xFE: every cell of the block is a pure cell whose answer is that code (key + 1), 0xFF: gather
// the cell's table entry.  Points in pure and empty cells then need no gather at all.
template <bool LDS_COUNTS, bool PAIRS, bool VEC>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4))) k_join_stream_bng(JoinArgs a, BngStreamArgs s) {
    extern __shared__ unsigned int lds[];
    const int ncw = LDS_COUNTS ? a.n_polygons + 64 : 0;
    uint32_t* stage = lds + ncw;
    uint32_t* lcw = stage + (int)(blockDim.x >> 6) * kStageWords;
    const uint8_t* lcell = (const uint8_t*)lcw;
    const bool use_lc = s.lcell_words > 0;  // (uniform)
    for (int k = threadIdx.x; k < ncw; k += blockDim.x) lds[k] = 0;
    lds_fill(lcw, s.lcell, s.lcell_words);
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rcell = stream_rsrc(s.cells, s.cells_bytes);
    const __amdgpu_buffer_rsrc_t rleaf = stream_rsrc(s.leaf, s.leaf_bytes);
    const int lane = (int)(threadIdx.x & 63);
    const unsigned long long lt_mask = (1ULL << lane) - 1ULL;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    uint32_t* wq = stage + wave * kStageWords;
    uint32_t wn = 0;
    bool nan_seen = false;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
    int64_t w0 = a.row_lo + ((int64_t)blockIdx.x * blockDim.x + (int64_t)wave * 64) * 4;
    auto row_of = [&](int64_t wb, int k) -> int64_t { return wb + (k >> 1) * 128 + 2 * lane + (k & 1); };
    v2d px[2], py[2];
    auto load4 = [&](int64_t wb) {
        const int64_t r = (wb + 256 <= a.n) ? wb + 2 * lane : a.row_lo;
        px[0] = __builtin_nontemporal_load((const v2d*)(a.x + r));
        px[1] = __builtin_nontemporal_load((const v2d*)(a.x + r + 128));
        py[0] = __builtin_nontemporal_load((const v2d*)(a.y + r));
        py[1] = __builtin_nontemporal_load((const v2d*)(a.y + r + 128));
    };
    if (VEC) load4(w0);
    const uint32_t C = (uint32_t)s.C;
    for (; w0 < a.n; w0 += stride) {
        const bool full = VEC && w0 + 256 <= a.n;
        double x[4], y[4];
        bool live[4];
        if (full) {
            x[0] = px[0].x, x[1] = px[0].y, x[2] = px[1].x, x[3] = px[1].y;
            y[0] = py[0].x, y[1] = py[0].y, y[2] = py[1].x, y[3] = py[1].y;
#pragma unroll
            for (int k = 0; k < 4; k++) live[k] = true;
        } else {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int64_t r = row_of(w0, k);
                live[k] = r < a.n;
                x[k] = live[k] ? a.x[r] : 0.0;
                y[k] = live[k] ? a.y[r] : 0.0;
            }
        }
        uint32_t code[4], e[4], loff[4];
        float gu[4], gv[4];
        bool inr[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const bool nan = x[k] != x[k] || y[k] != y[k];
            nan_seen |= live[k] && nan;
            const int32_t eI = bng::jvm_d2i(x[k]), nI = bng::jvm_d2i(y[k]);
            inr[k] = (uint32_t)eI < 10000000u && (uint32_t)nI < 10000000u;
            const double xe = (double)eI, ye = (double)nI;
            const int32_t qe = (int32_t)fma(xe, s.inv_div, 1e-7), qn = (int32_t)fma(ye, s.inv_div, 1e-7);
            const int32_t ce = qe - s.e0, cn = qn - s.n0;
            const bool cell_in = inr[k] && (uint32_t)ce < (uint32_t)s.ne && (uint32_t)cn < (uint32_t)s.nn;
            // LDS cell level first: only cells it marks kBngLdsGather gather their table entry
            const uint32_t li = cell_in ? __umul24((uint32_t)cn >> s.lsh, (uint32_t)s.lnx) + ((uint32_t)ce >> s.lsh) : 0u;
            const uint32_t lb = use_lc ? (uint32_t)lcell[li] : kBngLdsGather;
            const bool gth = cell_in && lb == kBngLdsGather;
            e[k] = __builtin_amdgcn_raw_buffer_load_b32(rcell, gth ? (uint32_t)(cn * s.ne + ce) << 2 : kNoLoad, 0, 0);
            e[k] = (gth || !cell_in) ? e[k] : (lb ? (kBngPure | lb) : 0u);
            // sub-cell of the point inside the cell [qe div, (qe + 1) div) x [qn div, (qn + 1) div):
            // the offset in the cell is (toInt(e) - qe div) (exact integer) + (e - toInt(e)) (exact in
            // f64), in f32 sub-cell units (relative error ~1e-7, far inside the builder's sub-cell
            // widening); one f64 add per axis instead of the f64 offset / scale / fract chain
            // (qe, qn < 2^24 wherever the cell is used: 24-bit multiplies)
            const float gxs = fmaf((float)(eI - (int32_t)__umul24((uint32_t)qe, (uint32_t)s.idiv)), s.ff, (float)(x[k] - xe) * s.ff);
            const float gys = fmaf((float)(nI - (int32_t)__umul24((uint32_t)qn, (uint32_t)s.idiv)), s.ff, (float)(y[k] - ye) * s.ff);
            int sx = (int)gxs, sy = (int)gys;
            sx = min(max(sx, 0), (int)C - 1);
            sy = min(max(sy, 0), (int)C - 1);
            gu[k] = gxs;  // offset in the cell (sub-cell units)
            gv[k] = gys;
            loff[k] = (uint32_t)(sy * (int)C + sx);
        }
        bool leafc[4], line[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            leafc[k] = (e[k] & (kBngPure | kBngLeaf)) == kBngLeaf;
            const uint32_t off = ((e[k] & ~kBngLeaf) + loff[k]) << 1;
            code[k] = __builtin_amdgcn_raw_buffer_load_b16(rleaf, leafc[k] ? off : kNoLoad, 0, 0);
        }
        v4u lrec[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            line[k] = leafc[k] && (code[k] & 0xC000u) == 0xC000u && code[k] != (uint32_t)tiles::kMixed;
            const uint32_t roff = ((e[k] & ~kBngLeaf) - 8u * ((code[k] & 0x3fffu) + 1u)) << 1;
            lrec[k] = __builtin_amdgcn_raw_buffer_load_b128(rleaf, line[k] ? roff : kNoLoad, 0, 0);
        }
        if (VEC) load4(w0 + stride);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            // tiles::line_code, as selects
            // (line records in the cell frame: the offsets from the cell's corner)
            const float lv = fmaf(__uint_as_float(lrec[k].x), gu[k], fmaf(__uint_as_float(lrec[k].y), gv[k], __uint_as_float(lrec[k].z)));
            uint32_t lc = lv >= 1.0f ? (lrec[k].w & 0xffffu) : (uint32_t)tiles::kMixed;
            lc = lv <= -1.0f ? (lrec[k].w >> 16) : lc;
            code[k] = line[k] ? lc : (code[k] - 0x8000u < 0x4000u ? (uint32_t)tiles::kMixed : code[k]);  // (wedges)
            uint32_t c = (e[k] & kBngPure) ? (e[k] & ~kBngPure) : ((e[k] & kBngLeaf) ? code[k] : (e[k] ? (uint32_t)tiles::kMixed : 0u));
            c = inr[k] ? c : (uint32_t)tiles::kMixed;      // outside the one-to-one range: generic path
            c = (x[k] != x[k] || y[k] != y[k]) ? 0u : c;  // NaN: flagged, no pair
            code[k] = live[k] ? c : 0u;
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (LDS_COUNTS && !PAIRS) {
                const uint32_t slot = code[k] - 1u < 0xfffeu ? code[k] - 1u : (uint32_t)(a.n_polygons + lane);
                atomicAdd(&lds[slot], 1u);
            } else if (code[k] - 1u < 0xfffeu) {
                emit_hit<LDS_COUNTS, PAIRS>(a, row_of(w0, k), code[k] - 1u, lds);
            }
        }
        const bool anym = code[0] == tiles::kMixed || code[1] == tiles::kMixed || code[2] == tiles::kMixed ||
                          code[3] == tiles::kMixed;
        if (__ballot(anym)) {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const bool m = code[k] == tiles::kMixed;
                const unsigned long long mm = __ballot(m);
                if (m) wq[wn + __popcll(mm & lt_mask)] = (uint32_t)(row_of(w0, k) - a.row_lo);
                wn += (uint32_t)__popcll(mm);
                stage_flush(a, wq, wn, lane, 64);  // the stage holds < 128
            }
        }
    }
    stage_flush(a, wq, wn, lane, 1);
    if (__ballot(nan_seen) && lane == 0) atomicOr(a.flags, 1u);
    if (LDS_COUNTS) {
        __syncthreads();
        for (int k = threadIdx.x; k < a.n_polygons; k += blockDim.x)
            if (lds[k]) atomicAdd(&a.counts[k], (unsigned long long)lds[k]);
    }
}


// ---- k_join_stream_bng_cpt: k_join_stream_bng with the rows that need gathers compacted (the H3
// k_join_stream_cpt scheme).  Stage A runs every row through the integer cell arithmetic and the LDS
// cell level; rows in empty or pure blocks (82 % of uniform C5 points), rows outside the one-to-one
// range (kMixed) and NaN rows (flagged) are answered there.  The others ("pending": in a border cell)
// go through a per-wave LDS buffer into one 64-lane set -- per row the cell index with the source
// lane and row slot, and the f32 sub-cell coordinates -- whose cell-entry + sub-block-level,
// sub-cell-code and line-record gathers and answers take one lane per pending row, as a four-stage
// software pipeline over the sets (iteration t: answers of the set of t - 3, line-record gathers of
// t - 2, sub-cell gathers of t - 1, group t's LDS level + compaction + cell-entry and level gathers,
// coordinates of t + 1).  The sub-block level (BngStreamArgs::lvl: per table cell one code per 4 x 4
// group of sub-cells, 128 B, read only for border cells, so the lines touched -- 2.6 MB for C5 --
// stay in L2) is gathered beside the cell entry, from the cell index alone; the 2-byte leaf code
// (2 KB leaf blocks over 41 MB) only for the rows whose group the level does not decide.
// More than 64 pending rows in a group are finished at once.  Needs ne nn < 2^24 (cell index in 24
// bits).  The sub-cell arithmetic is k_join_stream_bng's and a level code is the code of each
// sub-cell of its group, so the answers are the same point for point.
struct BngCptSet {
    uint32_t a;     // cell index | source lane << 24 | row slot k << 30
    uint32_t b, c;  // f32 sub-cell coordinates gxs, gys
    uint32_t e;     // A -> B: gathered cell entry; B -> C: the sub-cell code
    uint32_t l;     // A -> B: gathered sub-block level code
    uint32_t p;     // 0: empty slot; B -> C: the answer, or kBngLeaf; C -> D: the answer or kPipeLine
};
// (the cell's leaf base, B -> C, and the line record, C -> D, are held by one set at a time: one
// register copy each instead of one per set slot)

template <bool LDS_COUNTS, bool PAIRS>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4))) k_join_stream_bng_cpt(JoinArgs a, BngStreamArgs s) {
    extern __shared__ unsigned int lds[];
    const int nwaves = (int)(blockDim.x >> 6);
    const int ncw = LDS_COUNTS ? a.n_polygons + 64 : 0;
    uint32_t* stage = lds + ncw;
    uint32_t* cbuf_all = stage + nwaves * kStageWords;
    uint32_t* lcw = cbuf_all + nwaves * kCptBufWords;
    const uint8_t* lcell = (const uint8_t*)lcw;
    const bool use_lc = s.lcell_words > 0;  // (uniform)
    for (int k = threadIdx.x; k < ncw; k += blockDim.x) lds[k] = 0;
    lds_fill(lcw, s.lcell, s.lcell_words);
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rcell = stream_rsrc(s.cells, s.cells_bytes);
    const __amdgpu_buffer_rsrc_t rleaf = stream_rsrc(s.leaf, s.leaf_bytes);
    const __amdgpu_buffer_rsrc_t rlvl = stream_rsrc(s.lvl, s.lvl_bytes);
    const int lane = (int)(threadIdx.x & 63);
    const unsigned long long lt_mask = (1ULL << lane) - 1ULL;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    uint32_t* wq = stage + wave * kStageWords;
    uint32_t* cbuf = cbuf_all + wave * kCptBufWords;
    uint32_t wn = 0;
    bool nan_seen = false;
    const uint32_t C = (uint32_t)s.C;
    const uint32_t spill = (uint32_t)(a.n_polygons + lane);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
    const int64_t wbase = a.row_lo + ((int64_t)blockIdx.x * blockDim.x + (int64_t)wave * 64) * 4;
    const int64_t T = wbase + 256 <= a.n ? (a.n - 256 - wbase) / stride + 1 : 0;
    auto count = [&](uint32_t code, int64_t row) {
        if (LDS_COUNTS && !PAIRS) atomicAdd(&lds[min(code - 1u, spill)], 1u);  // 0 and kMixed: spill
        else if (code - 1u < 0xfffeu) emit_hit<LDS_COUNTS, PAIRS>(a, row, code - 1u, lds);
    };
    auto push_mixed = [&](bool m, int64_t row) {
        if (__ballot(m)) {
            const unsigned long long mm = __ballot(m);
            if (m) wq[wn + __popcll(mm & lt_mask)] = (uint32_t)(row - a.row_lo);
            wn += (uint32_t)__popcll(mm);
            stage_flush(a, wq, wn, lane, 64);  // the stage holds < 128
        }
    };
    // the sub-cell of set row z: index, and the offset in it (k_join_stream_bng's clamp)
    auto subcell = [&](const BngCptSet& z, float* su, float* sv) -> uint32_t {
        const float gxs = __uint_as_float(z.b), gys = __uint_as_float(z.c);
        int sx = (int)gxs, sy = (int)gys;
        sx = min(max(sx, 0), (int)C - 1);
        sy = min(max(sy, 0), (int)C - 1);
        *su = gxs - (float)sx;
        *sv = gys - (float)sy;
        return (uint32_t)(sy * (int)C + sx);
    };
    // A': cell-entry gathers
    auto set_a = [&](BngCptSet& z) {
        const uint32_t ci = z.a & 0xffffffu;
        z.e = gather_b32(rcell, z.p != 0u, ci << 2);
        const int sx = min(max((int)__uint_as_float(z.b), 0), (int)C - 1);  // (subcell's clamp)
        const int sy = min(max((int)__uint_as_float(z.c), 0), (int)C - 1);
        const uint32_t g = __umul24((uint32_t)sy >> tiles::kBngLvlShift, (uint32_t)s.lvl_cb) + ((uint32_t)sx >> tiles::kBngLvlShift);
        z.l = gather_b16<0>(rlvl, z.p != 0u, (ci * (uint32_t)s.lvl_stride + g) << 1);
    };
    // B': cell entry + level code -> sub-cell code gather (rows of undecided groups)
    auto set_b = [&](BngCptSet& z, uint32_t& base) {
        const uint32_t e = z.e;
        const bool leafc = z.p != 0u && (e & (kBngPure | kBngLeaf)) == kBngLeaf;
        base = e & ~kBngLeaf;
        float su, sv;
        const uint32_t q = subcell(z, &su, &sv);
        const bool see = leafc && z.l == (uint32_t)tiles::kSubBlock;  // the level does not decide
        const uint32_t v = gather_b16<0>(rleaf, see, (base + q) << 1);
        z.e = see ? v : z.l;
        z.p = z.p == 0u ? 0u : ((e & kBngPure) ? (e & ~kBngPure) : (leafc ? kBngLeaf : (e ? (uint32_t)tiles::kMixed : 0u)));
    };
    // C': sub-cell code -> line-record gather
    auto set_c = [&](BngCptSet& z, uint32_t base, v4u& lrec) {
        const uint32_t code = z.e;
        const bool leafc = z.p == kBngLeaf;
        const bool line = leafc && (code & 0xC000u) == 0xC000u && code != (uint32_t)tiles::kMixed;
        lrec = gather_b128<0>(rleaf, line, (base - 8u * ((code & 0x3fffu) + 1u)) << 1);
        // (wedge codes kSubBlock | n: the mixed queue, k_join_mixed_bng)
        z.p = line ? kPipeLine : (leafc ? (code - 0x8000u < 0x4000u ? (uint32_t)tiles::kMixed : code) : z.p);
    };
    // D': answers of the set's rows (group base wb)
    auto set_d = [&](BngCptSet& z, const v4u& lrec, int64_t wb) {
        // (line records in the cell frame: the offsets from the cell's corner)
        const float lv = fmaf(__uint_as_float(lrec.x), __uint_as_float(z.b), fmaf(__uint_as_float(lrec.y), __uint_as_float(z.c), __uint_as_float(lrec.z)));
        uint32_t lc = lv >= 1.0f ? (lrec.w & 0xffffu) : (uint32_t)tiles::kMixed;
        lc = lv <= -1.0f ? (lrec.w >> 16) : lc;
        const uint32_t code = z.p == kPipeLine ? lc : z.p;
        const uint32_t src = (z.a >> 24) & 63u, k = z.a >> 30;
        const int64_t row = wb + (int64_t)((k >> 1) * 128u + 2u * src + (k & 1u));
        count(code, row);
        push_mixed(code == (uint32_t)tiles::kMixed, row);
    };
    // A: a group through the cell arithmetic and the LDS level, resolved rows answered, pending rows
    // compacted into z (the first 64) through the wave's LDS buffer
    auto stage_a = [&](const double* x, const double* y, const bool* live, bool valid, BngCptSet& z, int64_t wb) {
        uint32_t fa[4], fb[4], fc[4];
        bool pend[4];
        uint32_t mixed_k = 0;  // row slots whose row goes to the mixed queue (outside the one-to-one range)
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const bool lv = valid && live[k];
            const bool nan = x[k] != x[k] || y[k] != y[k];
            nan_seen |= lv && nan;
            const int32_t eI = bng::jvm_d2i(x[k]), nI = bng::jvm_d2i(y[k]);
            const bool inr = (uint32_t)eI < 10000000u && (uint32_t)nI < 10000000u;
            const double xe = (double)eI, ye = (double)nI;
            const int32_t qe = (int32_t)fma(xe, s.inv_div, 1e-7), qn = (int32_t)fma(ye, s.inv_div, 1e-7);
            const int32_t ce = qe - s.e0, cn = qn - s.n0;
            const bool cell_in = inr && (uint32_t)ce < (uint32_t)s.ne && (uint32_t)cn < (uint32_t)s.nn;
            const uint32_t li = cell_in ? __umul24((uint32_t)cn >> s.lsh, (uint32_t)s.lnx) + ((uint32_t)ce >> s.lsh) : 0u;
            const uint32_t lb = use_lc ? (uint32_t)lcell[li] : kBngLdsGather;
            pend[k] = lv && !nan && cell_in && lb == kBngLdsGather;
            // resolved rows: outside the one-to-one range kMixed, else the LDS block's code (0 outside
            // the table); NaN and dead rows 0
            uint32_t code = !inr ? (uint32_t)tiles::kMixed : (cell_in ? (lb == kBngLdsGather ? 0u : lb) : 0u);
            code = (lv && !nan && !pend[k]) ? code : 0u;
            if (LDS_COUNTS && !PAIRS) atomicAdd(&lds[min(code - 1u, spill)], 1u);  // 0 and kMixed: spill
            else count(code, wb + (k >> 1) * 128 + 2 * lane + (k & 1));
            mixed_k |= (code == (uint32_t)tiles::kMixed ? 1u : 0u) << k;
            // k_join_stream_bng's f32 sub-cell coordinates
            const float gxs = fmaf((float)(eI - (int32_t)__umul24((uint32_t)qe, (uint32_t)s.idiv)), s.ff, (float)(x[k] - xe) * s.ff);
            const float gys = fmaf((float)(nI - (int32_t)__umul24((uint32_t)qn, (uint32_t)s.idiv)), s.ff, (float)(y[k] - ye) * s.ff);
            fa[k] = ((uint32_t)(cn * s.ne + ce) & 0xffffffu) | ((uint32_t)lane << 24) | ((uint32_t)k << 30);
            fb[k] = __float_as_uint(gxs);
            fc[k] = __float_as_uint(gys);
        }
        if (__ballot(mixed_k != 0u)) {  // (rare: one wave-uniform test per group)
            for (int k = 0; k < 4; k++) push_mixed((mixed_k >> k) & 1u, wb + (k >> 1) * 128 + 2 * lane + (k & 1));
        }
        uint32_t ranks[4];
        uint32_t P = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const unsigned long long m = __ballot(pend[k]);
            ranks[k] = P + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            P += (uint32_t)__popcll(m);
        }
        auto gather_set = [&](uint32_t sv, BngCptSet& o) {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t slot = ranks[k] - 64u * sv;
                if (pend[k] && slot < 64u) {
                    cbuf[slot] = fa[k];
                    cbuf[64 + slot] = fb[k];
                    cbuf[128 + slot] = fc[k];
                }
            }
            __builtin_amdgcn_wave_barrier();
            const bool ok = 64u * sv + (uint32_t)lane < P;
            o.a = ok ? cbuf[lane] : 0u;
            o.b = ok ? cbuf[64 + lane] : 0u;
            o.c = ok ? cbuf[128 + lane] : 0u;
            o.p = ok ? 1u : 0u;  // (a pending row: 1 until stage B' gives its answer)
            __builtin_amdgcn_wave_barrier();
        };
        gather_set(0u, z);
        set_a(z);
        if (P > 64u) {  // (wave-uniform) the group's further sets, unpipelined
            for (uint32_t sv = 1; sv * 64u < P; sv++) {
                BngCptSet o;
                uint32_t ob;
                v4u orec;
                gather_set(sv, o);
                set_a(o);
                set_b(o, ob);
                set_c(o, ob, orec);
                set_d(o, orec, wb);
            }
        }
    };
    struct Coords {
        v2d px[2], py[2];
    };
    auto load4 = [&](Coords& cb, int64_t wb, bool valid) {
        const int64_t r = valid ? wb + 2 * lane : wbase + 2 * lane;
        cb.px[0] = __builtin_nontemporal_load((const v2d*)(a.x + r));
        cb.px[1] = __builtin_nontemporal_load((const v2d*)(a.x + r + 128));
        cb.py[0] = __builtin_nontemporal_load((const v2d*)(a.y + r));
        cb.py[1] = __builtin_nontemporal_load((const v2d*)(a.y + r + 128));
    };
    BngCptSet z0, z1, z2;
    z0.a = z1.a = z2.a = z0.b = z1.b = z2.b = z0.c = z1.c = z2.c = 0u;
    z0.e = z1.e = z2.e = z0.p = z1.p = z2.p = z0.l = z1.l = z2.l = 0u;
    uint32_t base_bc = 0u;            // the leaf base of the set between stages B and C
    v4u lrec_cd = {0u, 0u, 0u, 0u};   // the line record of the set between stages C and D
    // zd: the set of t - 3, refilled with group t; zc: t - 2; zb: t - 1
    auto step = [&](bool valid, int64_t t, BngCptSet& zd, BngCptSet& zc, BngCptSet& zb, Coords& cb, Coords& cn) {
        const bool all[4] = {true, true, true, true};
        if (t >= 3) set_d(zd, lrec_cd, wbase + (t - 3) * stride);
        set_c(zc, base_bc, lrec_cd);
        set_b(zb, base_bc);
        const double x[4] = {cb.px[0].x, cb.px[0].y, cb.px[1].x, cb.px[1].y};
        const double y[4] = {cb.py[0].x, cb.py[0].y, cb.py[1].x, cb.py[1].y};
        stage_a(x, y, all, valid, zd, wbase + t * stride);
        load4(cn, wbase + (t + 1) * stride, t + 1 < T);
    };
    if (T > 0) {
        Coords cb0, cb1;
        load4(cb0, wbase, true);
        int64_t t = 0;
        for (; t + 6 <= T; t += 6) {
            step(true, t, z0, z1, z2, cb0, cb1);
            step(true, t + 1, z1, z2, z0, cb1, cb0);
            step(true, t + 2, z2, z0, z1, cb0, cb1);
            step(true, t + 3, z0, z1, z2, cb1, cb0);
            step(true, t + 4, z1, z2, z0, cb0, cb1);
            step(true, t + 5, z2, z0, z1, cb1, cb0);
        }
        // the remaining groups (<= 5) and the three drain steps, in the same slot sequence
#define MOSAIC_BCPT_TAIL(ZD, ZC, ZB, CB, CN) \
    if (t < T + 3) {                       \
        step(t < T, t, ZD, ZC, ZB, CB, CN); \
        t++;                               \
    }
        MOSAIC_BCPT_TAIL(z0, z1, z2, cb0, cb1)
        MOSAIC_BCPT_TAIL(z1, z2, z0, cb1, cb0)
        MOSAIC_BCPT_TAIL(z2, z0, z1, cb0, cb1)
        MOSAIC_BCPT_TAIL(z0, z1, z2, cb1, cb0)
        MOSAIC_BCPT_TAIL(z1, z2, z0, cb0, cb1)
        MOSAIC_BCPT_TAIL(z2, z0, z1, cb1, cb0)
        MOSAIC_BCPT_TAIL(z0, z1, z2, cb0, cb1)
        MOSAIC_BCPT_TAIL(z1, z2, z0, cb1, cb0)
#undef MOSAIC_BCPT_TAIL
    }
    // the wave's partial group, unpipelined
    const int64_t wt = wbase + T * stride;
    if (wt < a.n) {
        double x[4], y[4];
        bool live[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int64_t r = wt + (k >> 1) * 128 + 2 * lane + (k & 1);
            live[k] = r < a.n;
            x[k] = live[k] ? a.x[r] : 0.0;
            y[k] = live[k] ? a.y[r] : 0.0;
        }
        BngCptSet z;
        uint32_t zb;
        v4u zrec;
        stage_a(x, y, live, true, z, wt);
        set_b(z, zb);
        set_c(z, zb, zrec);
        set_d(z, zrec, wt);
    }
    stage_flush(a, wq, wn, lane, 1);
    if (__ballot(nan_seen) && lane == 0) atomicOr(a.flags, 1u);
    if (LDS_COUNTS) {
        __syncthreads();
        for (int k = threadIdx.x; k < a.n_polygons; k += blockDim.x)
            if (lds[k]) atomicAdd(&a.counts[k], (unsigned long long)lds[k]);
    }
}

// ---- k_join_leaf: the mixed queue's rows whose leaf cell is a leaf line (tiles.h leaf_is_line: the
// cell is split by one straight chip edge) are answered from the line record; the others -- the
// line's band, mixed leaf cells, line sub-blocks' bands, non-finite rows -- move to queue q2, which
// k_join_mixed then takes.  One lane per row: tiles::raster_code_fixed's chain from global memory
// (quad level, quad record, compact sub-block entry, tile base, leaf code, line record), the same
// fine cell and line offsets as the stream kernels.  ~95 % of NYC res-9 mixed leaf cells are leaf
// lines (tools/raster_stats.cpp), so the mixed kernel's H3 cell + chip loop runs on ~1/5 of the rows.
template <bool LDS_COUNTS, bool PAIRS>
__global__ void __launch_bounds__(256) k_join_leaf(JoinArgs a, StreamArgs s, uint32_t* q2, unsigned long long* q2_count) {
    extern __shared__ unsigned int lds[];
    if (LDS_COUNTS) {
        for (int k = threadIdx.x; k < a.n_polygons; k += blockDim.x) lds[k] = 0;
        __syncthreads();
    }
    // kept rows through a per-wave stage (one q2 atomic per >= 64 rows: a per-wave atomic on one
    // counter from every wave at once serialises the kernel)
    JoinArgs aq = a;
    aq.mixq = q2;
    aq.mixq_count = q2_count;
    uint32_t* wq = lds + (LDS_COUNTS ? a.n_polygons : 0) + (threadIdx.x >> 6) * kStageWords;
    uint32_t wn = 0;
    constexpr int F = tiles::kFixBits;
    const int lane = (int)(threadIdx.x & 63);
    const unsigned long long lt_mask = (1ULL << lane) - 1ULL;
    const uint16_t* quad = (const uint16_t*)s.quad;
    const uint32_t* qmask = s.qrec;
    const uint16_t* qcode = (const uint16_t*)(s.qrec + 2 * s.n_qrec);
    const uint32_t cs = (uint32_t)s.cs, qs = (uint32_t)s.qs, cm = (1u << cs) - 1u, qm = (1u << qs) - 1u;
    const unsigned long long total = *a.mixq_count;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    // wave-uniform loop (the q2 append is a wave ballot)
    for (unsigned long long t0 = (unsigned long long)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); t0 < total; t0 += stride) {
        const unsigned long long t = t0 + (unsigned long long)lane;
        const bool live = t < total;
        const uint32_t off = live ? a.mixq[t] : 0u;
        const int64_t row = a.row_lo + (int64_t)off;
        uint32_t code = tiles::kMixed;
        if (live) {
            const double x = a.x[row], y = a.y[row];
            if (isfinite(x + y)) {
                const uint32_t gix = min(tiles::fix_cvt(fma(x, s.sxF, s.gx0F)), (uint32_t)s.gxmaxF);
                const uint32_t giy = min(tiles::fix_cvt(fma(y, s.syF, s.gy0F)), (uint32_t)s.gymaxF);
                const uint32_t ixC = gix >> F, iyC = giy >> F, ix = ixC >> cs, iy = iyC >> cs;
                const uint32_t q = quad_lookup<F>(s, quad, qmask, qcode, gix, giy);
                const uint32_t e = q < 0x8000u ? q : s.csub[((q & 0x7fffu) << (2 * qs)) + (((iy & qm) << qs) | (ix & qm))];
                code = e;
                if (tiles::sub_is_block(e) && !(e & tiles::kLineBit)) {
                    const uint32_t tile = (iyC >> s.tsh) * (uint32_t)s.tnx + (ixC >> s.tsh);
                    const uint32_t base = s.tile_base[tile];
                    const uint32_t lc = s.blocks[base + ((e & 0x3fffu) << (2 * cs)) + (((iyC & cm) << cs) | (ixC & cm))];
                    code = lc;
                    if (tiles::leaf_is_line(lc)) {
                        const tiles::LineRec lr = s.llines[s.tile_lbase[tile] + (lc & 0x3fffu)];
                        const uint32_t fm = (1u << (cs + F)) - 1u;
                        const float sc = 1.0f / (float)(1 << F);
                        code = tiles::line_code(lr, (float)(gix & fm) * sc, (float)(giy & fm) * sc);
                    }
                } else if (tiles::sub_is_block(e)) {
                    code = tiles::kMixed;  // a line sub-block's band (the stream kernel's answer)
                }
            }
        }
        const bool keep = live && code >= 0x8000u;  // kMixed (or a code the chain cannot decide)
        if (live && !keep && code != 0u) {
            if (LDS_COUNTS && !PAIRS) atomicAdd(&lds[code - 1u], 1u);
            else emit_hit<LDS_COUNTS, PAIRS>(a, row, code - 1u, lds);
        }
        stage_push(wq, wn, keep, off, lt_mask);
        stage_flush(aq, wq, wn, lane, 64);
    }
    stage_flush(aq, wq, wn, lane, 1);
    if (LDS_COUNTS) {
        __syncthreads();
        for (int k = threadIdx.x; k < a.n_polygons; k += blockDim.x)
            if (lds[k]) atomicAdd(&a.counts[k], (unsigned long long)lds[k]);
    }
}

const void* leaf_kernel(bool lds, bool pairs) {
    if (pairs) return (const void*)k_join_leaf<false, true>;
    if (lds) return (const void*)k_join_leaf<true, false>;
    return (const void*)k_join_leaf<false, false>;
}

const void* stream_kernel_h3(int pipe, bool lds, bool pairs, bool vec) {
    if (pipe == 2 && vec) {
        if (pairs) return (const void*)k_join_stream_cpt<false, true>;
        if (lds) return (const void*)k_join_stream_cpt<true, false>;
        return (const void*)k_join_stream_cpt<false, false>;
    }
    if (pipe && vec) {
        if (pairs) return (const void*)k_join_stream_pipe<false, true>;
        if (lds) return (const void*)k_join_stream_pipe<true, false>;
        return (const void*)k_join_stream_pipe<false, false>;
    }
    if (pairs) return vec ? (const void*)k_join_stream<false, true, true> : (const void*)k_join_stream<false, true, false>;
    if (lds) return vec ? (const void*)k_join_stream<true, false, true> : (const void*)k_join_stream<true, false, false>;
    return vec ? (const void*)k_join_stream<false, false, true> : (const void*)k_join_stream<false, false, false>;
}

const void* stream_kernel_bng(bool lds, bool pairs, bool vec, bool cpt) {
    if (cpt && vec) {
        if (pairs) return (const void*)k_join_stream_bng_cpt<false, true>;
        if (lds) return (const void*)k_join_stream_bng_cpt<true, false>;
        return (const void*)k_join_stream_bng_cpt<false, false>;
    }
    if (pairs) return vec ? (const void*)k_join_stream_bng<false, true, true> : (const void*)k_join_stream_bng<false, true, false>;
    if (lds) return vec ? (const void*)k_join_stream_bng<true, false, true> : (const void*)k_join_stream_bng<true, false, false>;
    return vec ? (const void*)k_join_stream_bng<false, false, true> : (const void*)k_join_stream_bng<false, false, false>;
}

extern "C" uint64_t mosaic_layout_join_stream(void) { return mosaic_layout_fingerprint(); }
