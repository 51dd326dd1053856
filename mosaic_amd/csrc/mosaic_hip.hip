// libmosaic_hip.so: HIP kernels for gfx950 + the C ABI of include/mosaic_hip.h.
//
// Hot path (BASELINE.json north_star): per point
//   (a) cell = H3 / BNG point index         (h3_device.h fast path, bng_device.h)
//   (b) probe the chip hash table by cell    (open addressing, 16-byte entries, L2-resident)
//   (c) core chip -> accept; border chip -> JTS contains on the chip rings (pip_device.h)
//   and count accepted pairs per polygon key in LDS, flushed once per workgroup.
// (a)-(c) are fused in one grid-stride kernel so the 16 B/point coordinate stream is read once.
// Points whose H3 cell the fast path cannot certify are appended to a queue and finished by a
// second kernel running the exact H3 restatement (h3_exact).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <sys/mman.h>
#include <dirent.h>
#include <sys/prctl.h>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/mosaic_hip.h"
#include "bng_device.h"
#include "geom_build.h"
#include "h3_device.h"
#include "h3_geom.h"
#include "h3_grid.h"
#include "h3_neighbors.h"
#include "isect_geom.h"
#include "overlay.h"
#include "join_binned.h"
#include "join_common.h"
#include "pip_coop.h"
#include "pip_device.h"
#include "point_decode.h"
#include "raster.h"
#include "raster_build.h"
#include "tess_clip.h"
#include "tess_gpu.h"
#include "tiles.h"

using namespace mosaic;

// ------------------------------------------------------------------------------------------------
// errors
static thread_local std::string g_last_error;

// f(0) .. f(n - 1) on n host threads (the caller's thread runs f(0))
template <class F>
static void parallel_for(int n, F f) {
    std::vector<std::thread> pool;
    for (int k = 1; k < n; k++) pool.emplace_back(f, k);
    if (n > 0) f(0);
    for (auto& t : pool) t.join();
}

static int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define HIP_TRY(expr)                                                                                   \
    do {                                                                                                \
        hipError_t _e = (expr);                                                                         \
        if (_e != hipSuccess) return fail(MOSAIC_E_HIP, std::string(#expr ": ") + hipGetErrorString(_e)); \
    } while (0)

#include "join_chips.h"

namespace mosaic {
int kring_slow_host(uint64_t origin, int k, int loop, int64_t* out, int64_t* tab, int32_t* dist, uint64_t* stack);  // kring_host.cpp
}
// the other translation units' view of the shared structs (join_binned.h, tess_clip.h)
extern "C" uint64_t mosaic_layout_join_binned(void);
extern "C" uint64_t mosaic_layout_join_stream(void);
extern "C" uint64_t mosaic_layout_tess_clip(void);

template <int GRID, bool LDS_COUNTS, bool PAIRS>
__global__ void __launch_bounds__(256) k_join_raster(JoinArgs a) {
    extern __shared__ unsigned int lds[];
    __shared__ SlabItem items[4][16];
    counts_init<LDS_COUNTS>(a, lds);
    unsigned int tests = 0;
    bool nan_seen = false;
    const int lane = (int)(threadIdx.x & 63);
    const int wv = (int)(threadIdx.x >> 6) & 3;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x + (int64_t)(threadIdx.x & ~63u); base < a.n; base += stride) {
        int64_t i = base + lane;
        bool act = i < a.n && (!a.valid || a.valid[i]);
        double x = 0.0, y = 0.0;
        int64_t cell = kEmptyKey;
        if (act) {
            x = a.x[i];
            y = a.y[i];
            if (GRID == MOSAIC_GRID_H3) {
                bool amb;
                cell = (int64_t)h3::h3_fast(y, x, a.res, &amb);
                if (amb) {
                    unsigned long long q = atomicAdd(a.amb_count, 1ULL);
                    if (q < a.amb_cap) a.amb_queue[q] = (unsigned long long)i;
                    cell = kEmptyKey;
                }
            } else if (!bng::point_to_index(x, y, a.res, &cell)) {
                nan_seen = true;
                cell = kEmptyKey;
            }
        }
        uint32_t cur, end;
        probe(a, cell, cur, end);
        raster_chips<LDS_COUNTS, PAIRS>(a, i, cur, end, x, y, tests, lds, items[wv]);
    }
    if (nan_seen) atomicOr(a.flags, 1u);
    counts_flush<LDS_COUNTS>(a, lds, tests);
}

template <bool LDS_COUNTS, bool PAIRS>
__device__ inline void tiled_process(const JoinArgs& a, const TileQueue& q, int slot, bool live, unsigned int& tests,
                                     unsigned int* lds, SlabItem* items) {
    double x = 0.0, y = 0.0;
    int64_t i = -1;
    uint32_t cur = 0, end = 0;
    if (live) {
        x = q.x[slot];
        y = q.y[slot];
        i = q.row[slot];
        tiled_cell(a, i, x, y, q.code[slot], cur, end);
    }
    raster_chips<LDS_COUNTS, PAIRS>(a, i, cur, end, x, y, tests, lds, items);
}

template <bool LDS_COUNTS, bool PAIRS>
__global__ void __launch_bounds__(256) k_join_tiled(JoinArgs a) {
    extern __shared__ unsigned int lds[];
    __shared__ SlabItem items[4][16];
    __shared__ TileQueue queues[4];
    counts_init<LDS_COUNTS>(a, lds);
    unsigned int tests = 0;
    const int lane = (int)(threadIdx.x & 63);
    const int wv = (int)(threadIdx.x >> 6) & 3;
    const unsigned long long lt_mask = (1ULL << lane) - 1ULL;
    TileQueue& q = queues[wv];
    int qn = 0;  // wave-uniform fill level
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x + (int64_t)(threadIdx.x & ~63u); base < a.n; base += stride) {
        const int64_t i = base + lane;
        bool need = false;
        double x = 0.0, y = 0.0;
        uint32_t code = tiles::kSkip;
        if (i < a.n && (!a.valid || a.valid[i])) {
            x = a.x[i];
            y = a.y[i];
            code = tiles::tile_of(a.tgrid, a.tile_idx, x, y);
            need = code != tiles::kSkip;
        }
        const unsigned long long nm = __ballot(need);
        if (need) {
            const int s = qn + __popcll(nm & lt_mask);
            q.x[s] = x;
            q.y[s] = y;
            q.row[s] = i;
            q.code[s] = code;
        }
        qn += __popcll(nm);
        if (qn >= 64) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            qn -= 64;
            tiled_process<LDS_COUNTS, PAIRS>(a, q, qn + lane, true, tests, lds, items[wv]);
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (qn > 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        tiled_process<LDS_COUNTS, PAIRS>(a, q, lane, lane < qn, tests, lds, items[wv]);
    }
    counts_flush<LDS_COUNTS>(a, lds, tests);
}

// ---- point-raster build on the GPU: phase 1 of tiles::Builder::build_raster (tiles_build.cpp,
// classify_raster_host), the same classification with the same arithmetic (raster_build.h), so the
// raster is identical bit for bit.  k_raster_sub: one lane per sub-block of every tile record ->
// its code or kMixed; k_raster_line: one lane per mixed sub-block -> a line record, if one
// certifies; k_raster_cells: one lane per leaf cell of the other mixed sub-blocks.  Candidate
// hexagons are recomputed per lane (a window holds a few dozen).  The host assembles (phase 2).
struct RBuildArgs {
    const tiles::TileRec* recs;
    const int32_t* tile_of_rec;
    const tiles::TileCurv* rec_curv;
    const uint32_t* entries;  // tile-window entries: chip-hash slot + 1
    int32_t n_recs, tnx;
    double gx0, gy0, tw, th;
    int32_t S, C, N, res, lines;
    const HashEntry* table;
    const uint32_t* meta;
    pip::GeomStore store;
    rbuild::HexTable ht;
    uint16_t* code;             // n_recs x S x S
    const uint32_t* mixed;      // k_raster_line: mixed sub-blocks (index into code)
    int64_t n_mixed;
    uint8_t* kind;              // per mixed sub-block: 1 line record, 0 cells
    tiles::LineRec* line;
    const uint32_t* cell_sb;    // k_raster_cells: the kind-0 mixed sub-blocks (index into code)
    int64_t n_cell_sb;
    uint16_t* cells;            // n_cell_sb x C x C
};

struct RTile {  // one tile record, as the builder's per-record lambda sees it
    int face, wa, wb, a0, b0;
    uint32_t off;
    double lon0, lat0, exd, eyd;
    tiles::TileCurv cv;
};

__device__ inline bool rtile_of(const RBuildArgs& a, int r, RTile& t) {
    const tiles::TileRec tr = a.recs[r];
    const int ti_ = a.tile_of_rec[r];
    if (ti_ < 0 || tr.dims == 0) return false;
    const int ti = ti_ % a.tnx, tj = ti_ / a.tnx;
    t.face = (int)(tr.dims & 0xffu);
    t.wa = (int)((tr.dims >> 8) & 0xfffu);
    t.wb = (int)(tr.dims >> 20);
    t.a0 = tr.a0;
    t.b0 = tr.b0;
    t.off = tr.off;
    t.lon0 = a.gx0 + ti * a.tw;
    t.lat0 = a.gy0 + tj * a.th;
    t.cv = a.rec_curv[r];
    const double cell_deg_x = a.tw / a.N, cell_deg_y = a.th / a.N;
    t.exd = 1e-6 * cell_deg_x + 1e-12 * (fabs(t.lon0) + 1.0);
    t.eyd = 1e-6 * cell_deg_y + 1e-12 * (fabs(t.lat0) + 1.0);
    return true;
}

__device__ inline rbuild::P2 rimage(const RBuildArgs& a, const RTile& t, double i, double j) {
    double px, py, pz, vx, vy, b;
    h3::fast_unit(t.lat0 + a.th * j / a.N, t.lon0 + a.tw * i / a.N, &px, &py, &pz);
    h3::fast_plane(px, py, pz, t.face, a.res, &vx, &vy, &b);
    return rbuild::P2{vx, vy};
}

__device__ inline rbuild::P2 rhex_centre(const RTile& t, int k) {
    const int ra = k / t.wb, rb = k - ra * t.wb;
    const int aa = t.a0 + ra, bb = t.b0 + rb;
    return rbuild::P2{(double)aa - 0.5 * (double)bb, (double)bb * rbuild::kS60};
}

// The answer of window hexagon k's points in a region: the keys of its core chips plus those of
// its border chips containing (cx, cy) -- as (count, key of a single one) -- or -1 when a border
// chip's boundary meets the region (rect: [x0, x1] x [y0, y1]; poly: ll[n] within eps).
__device__ inline int rhex_answer(const RBuildArgs& a, const RTile& t, int k, bool poly, double x0, double y0,
                                  double x1, double y1, const rbuild::P2* ll, int n, double eps, double cx, double cy,
                                  int* key) {
    const uint32_t e = a.entries[t.off + (uint32_t)k];
    int cnt = 0;
    *key = -1;
    if (!e) return 0;
    const HashEntry he = a.table[e - 1];
    for (uint32_t c = he.first; c < he.first + he.count; c++) {
        const uint32_t m = a.meta[c];
        if (!(m & 1u)) {
            const pip::Box bx = a.store.geom_bbox[c];
            const bool meets_box = poly ? !(bx.maxx < x0 - eps || bx.minx > x1 + eps || bx.maxy < y0 - eps || bx.miny > y1 + eps)
                                        : !(bx.maxx < x0 || bx.minx > x1 || bx.maxy < y0 || bx.miny > y1);
            if (meets_box) {
                for (uint32_t p = a.store.geom_part[c]; p < a.store.geom_part[c + 1]; p++)
                    for (uint32_t r = a.store.part_ring[p]; r < a.store.part_ring[p + 1]; r++)
                        for (uint32_t v = a.store.ring_start[r] + 1; v < a.store.ring_start[r + 1]; v++) {
                            const pip::Vec2 s0 = a.store.verts[v - 1], s1 = a.store.verts[v];
                            const bool hit = poly ? rbuild::seg_meets_poly(rbuild::P2{s0.x, s0.y}, rbuild::P2{s1.x, s1.y}, ll, n, eps)
                                                  : raster::seg_meets_rect(s0.x, s0.y, s1.x, s1.y, x0, y0, x1, y1);
                            if (hit) return -1;
                        }
            }
            if (!pip::contains(a.store, c, cx, cy)) continue;
        }
        if (cnt == 0) *key = (int)(m >> 1);
        cnt++;
    }
    return cnt;
}

// tiles_build.cpp classify(): the code of fine-lattice rectangle [i0, i1] x [j0, j1] with corner
// images q; candidates: window hexagons meeting q (and, for cells, meeting the sub-block quad sq
// with the sub-block's tolerance).
__device__ inline uint16_t rclassify_rect(const RBuildArgs& a, const RTile& t, int i0, int j0, int i1, int j1,
                                          const rbuild::P2* q, const rbuild::P2* sq, double stol) {
    const double cell_deg_x = a.tw / a.N, cell_deg_y = a.th / a.N;
    const double ex = 1e-6 * cell_deg_x + 1e-12 * (fabs(t.lon0) + 1.0);
    const double ey = 1e-6 * cell_deg_y + 1e-12 * (fabs(t.lat0) + 1.0);
    const double tol = tiles::rect_tol(t.cv, cell_deg_x * (i1 - i0), cell_deg_y * (j1 - j0), rbuild::dmax(ex, ey));
    const double x0 = t.lon0 + a.tw * i0 / a.N - ex, x1 = t.lon0 + a.tw * i1 / a.N + ex;
    const double y0 = t.lat0 + a.th * j0 / a.N - ey, y1 = t.lat0 + a.th * j1 / a.N + ey;
    const double cxm = t.lon0 + a.tw * (i0 + i1) / (2.0 * a.N), cym = t.lat0 + a.th * (j0 + j1) / (2.0 * a.N);
    bool any = false;
    int acnt = 0, akey = -1;
    for (int k = 0; k < t.wa * t.wb; k++) {
        const rbuild::P2 c = rhex_centre(t, k);
        if (sq && !rbuild::poly_meets_hex(sq, 4, c, stol, a.ht)) continue;
        if (!rbuild::poly_meets_hex(q, 4, c, tol, a.ht)) continue;
        int key;
        const int cnt = rhex_answer(a, t, k, false, x0, y0, x1, y1, nullptr, 0, 0.0, cxm, cym, &key);
        if (cnt < 0 || cnt > 1) return tiles::kMixed;
        if (!any) {
            any = true;
            acnt = cnt;
            akey = key;
        } else if (cnt != acnt || key != akey) {
            return tiles::kMixed;
        }
    }
    if (!any) return tiles::kMixed;
    return acnt == 0 ? (uint16_t)0 : (uint16_t)(akey + 1);
}

// the sub-block quad (corner images) of sub-block (si, sj) and its tolerance
__device__ inline double rsub_quad(const RBuildArgs& a, const RTile& t, int si, int sj, rbuild::P2* q) {
    const int C = a.C;
    q[0] = rimage(a, t, si * C, sj * C);
    q[1] = rimage(a, t, (si + 1) * C, sj * C);
    q[2] = rimage(a, t, (si + 1) * C, (sj + 1) * C);
    q[3] = rimage(a, t, si * C, (sj + 1) * C);
    const double cell_deg_x = a.tw / a.N, cell_deg_y = a.th / a.N;  // (as the host's classify)
    return tiles::rect_tol(t.cv, cell_deg_x * C, cell_deg_y * C, rbuild::dmax(t.exd, t.eyd));
}

// tiles_build.cpp classify_poly(): convex region uv[n] of sub-block (si, sj), candidates those
// of the sub-block (sq, stol)
__device__ inline uint16_t rclassify_poly(const RBuildArgs& a, const RTile& t, int si, int sj, const rbuild::P2* uv,
                                          int n, const rbuild::P2* sq, double stol) {
    using rbuild::dmax;
    using rbuild::dmin;
    rbuild::P2 img[8], ll[8];
    double u0 = INFINITY, u1 = -INFINITY, v0 = INFINITY, v1 = -INFINITY;
    double x0 = INFINITY, x1 = -INFINITY, y0 = INFINITY, y1 = -INFINITY, mx = 0.0, my = 0.0;
    const int S = a.S, C = a.C;
    for (int v = 0; v < n; v++) {
        img[v] = rimage(a, t, (si + uv[v].x) * C, (sj + uv[v].y) * C);
        ll[v] = rbuild::P2{t.lon0 + a.tw * (si + uv[v].x) / S, t.lat0 + a.th * (sj + uv[v].y) / S};
        u0 = dmin(u0, uv[v].x);
        u1 = dmax(u1, uv[v].x);
        v0 = dmin(v0, uv[v].y);
        v1 = dmax(v1, uv[v].y);
        x0 = dmin(x0, ll[v].x);
        x1 = dmax(x1, ll[v].x);
        y0 = dmin(y0, ll[v].y);
        y1 = dmax(y1, ll[v].y);
        mx += ll[v].x;
        my += ll[v].y;
    }
    mx /= n;
    my /= n;
    const double eps = dmax(t.exd, t.eyd);
    const double tol = tiles::poly_tol(t.cv, a.tw * (u1 - u0) / S, a.th * (v1 - v0) / S, eps);
    bool any = false;
    int acnt = 0, akey = -1;
    for (int k = 0; k < t.wa * t.wb; k++) {
        const rbuild::P2 c = rhex_centre(t, k);
        if (!rbuild::poly_meets_hex(sq, 4, c, stol, a.ht)) continue;
        if (!rbuild::poly_meets_hex(img, n, c, tol, a.ht)) continue;
        int key;
        const int cnt = rhex_answer(a, t, k, true, x0, y0, x1, y1, ll, n, eps, mx, my, &key);
        if (cnt < 0 || cnt > 1) return tiles::kMixed;
        if (!any) {
            any = true;
            acnt = cnt;
            akey = key;
        } else if (cnt != acnt || key != akey) {
            return tiles::kMixed;
        }
    }
    if (!any) return tiles::kMixed;
    return acnt == 0 ? (uint16_t)0 : (uint16_t)(akey + 1);
}

__global__ void __launch_bounds__(256) k_raster_sub(RBuildArgs a) {
    const int64_t SS = (int64_t)a.S * a.S;
    const int64_t total = (int64_t)a.n_recs * SS;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total; g += (int64_t)gridDim.x * blockDim.x) {
        const int r = (int)(g / SS), sb = (int)(g - (int64_t)r * SS), sj = sb / a.S, si = sb - sj * a.S;
        RTile t;
        uint16_t code = 0;
        if (rtile_of(a, r, t)) {
            rbuild::P2 q[4];
            rsub_quad(a, t, si, sj, q);
            code = rclassify_rect(a, t, si * a.C, sj * a.C, (si + 1) * a.C, (sj + 1) * a.C, q, nullptr, 0.0);
        }
        a.code[g] = code;
    }
}

// tiles_build.cpp try_line()
__device__ inline bool rtry_line(const RBuildArgs& a, const RTile& t, int si, int sj, const rbuild::P2* sq, double stol,
                                 tiles::LineRec& out) {
    const int S = a.S;
    const double wR = a.tw / S, hR = a.th / S;
    const double lonR0 = t.lon0 + a.tw * si / S, latR0 = t.lat0 + a.th * sj / S;
    const double exu = t.exd / wR, eyv = t.eyd / hR;
    const double bx0 = lonR0 - t.exd, bx1 = lonR0 + wR + t.exd, by0 = latR0 - t.eyd, by1 = latR0 + hR + t.eyd;
    // pass 0: the longest clipped border-chip segment; pass 1: the largest distance of any clipped
    // end from its line
    double best = 0.0, dev_max = 0.0, la = 0.0, lb = 0.0, lc = 0.0;
    rbuild::P2 ta{0, 0}, tb{0, 0};  // the longest piece's whole segment, tile frame
    for (int pass = 0; pass < 2; pass++) {
        for (int k = 0; k < t.wa * t.wb; k++) {
            if (!rbuild::poly_meets_hex(sq, 4, rhex_centre(t, k), stol, a.ht)) continue;
            const uint32_t e = a.entries[t.off + (uint32_t)k];
            if (!e) continue;
            const HashEntry he = a.table[e - 1];
            for (uint32_t c = he.first; c < he.first + he.count; c++) {
                if (a.meta[c] & 1u) continue;
                const pip::Box bx = a.store.geom_bbox[c];
                if (bx.maxx < bx0 || bx.minx > bx1 || bx.maxy < by0 || bx.miny > by1) continue;
                for (uint32_t p = a.store.geom_part[c]; p < a.store.geom_part[c + 1]; p++)
                    for (uint32_t r = a.store.part_ring[p]; r < a.store.part_ring[p + 1]; r++)
                        for (uint32_t v = a.store.ring_start[r] + 1; v < a.store.ring_start[r + 1]; v++) {
                            const pip::Vec2 s0 = a.store.verts[v - 1], s1 = a.store.verts[v];
                            double ax = (s0.x - lonR0) / wR, ay = (s0.y - latR0) / hR;
                            double qx = (s1.x - lonR0) / wR, qy = (s1.y - latR0) / hR;
                            if (!rbuild::clip_seg(ax, ay, qx, qy, -exu, -eyv, 1.0 + exu, 1.0 + eyv)) continue;
                            if (pass == 0) {
                                const double l2 = (qx - ax) * (qx - ax) + (qy - ay) * (qy - ay);
                                if (l2 > best) {
                                    best = l2;
                                    ta = rbuild::P2{(s0.x - t.lon0) / wR, (s0.y - t.lat0) / hR};
                                    tb = rbuild::P2{(s1.x - t.lon0) / wR, (s1.y - t.lat0) / hR};
                                }
                            } else {
                                dev_max = rbuild::dmax(dev_max, fabs(la * (ax + si) + lb * (ay + sj) + lc));
                                dev_max = rbuild::dmax(dev_max, fabs(la * (qx + si) + lb * (qy + sj) + lc));
                            }
                        }
            }
        }
        if (pass == 0) {
            if (!(best > 1e-6)) return false;
            const double lt = sqrt((tb.x - ta.x) * (tb.x - ta.x) + (tb.y - ta.y) * (tb.y - ta.y));
            la = -(tb.y - ta.y) / lt;
            lb = (tb.x - ta.x) / lt;
            lc = -(la * 0.5 * (ta.x + tb.x) + lb * 0.5 * (ta.y + tb.y));
        }
    }
    const rbuild::P2 sqb[4] = {{-exu, -eyv}, {1.0 + exu, -eyv}, {1.0 + exu, 1.0 + eyv}, {-exu, 1.0 + eyv}};
    for (int mk = 0; mk < 4; mk++) {
        const double margin = rbuild::line_margin(mk);
        if (dev_max > margin - 2.0 * tiles::kLineSlack) continue;
        out.a = (float)(la / margin);
        out.b = (float)(lb / margin);
        out.c = (float)(lc / margin);
        const double A = out.a, B = out.b;
        const double Cf = (double)out.c + A * si + B * sj;
        const double m = 1.0 - rbuild::line_slack_tile(A, B, out.c, S, tiles::kLineSlack);
        rbuild::P2 hp[8], hn[8];
        const int np = rbuild::clip_half(sqb, 4, A, B, Cf - m, hp), nn = rbuild::clip_half(sqb, 4, -A, -B, -Cf - m, hn);
        const uint16_t cp = np >= 3 ? rclassify_poly(a, t, si, sj, hp, np, sq, stol) : (uint16_t)0;
        if (cp == tiles::kMixed) continue;
        const uint16_t cn = nn >= 3 ? rclassify_poly(a, t, si, sj, hn, nn, sq, stol) : (uint16_t)0;
        if (cn == tiles::kMixed) continue;
        out.pos = cp;
        out.neg = cn;
        out.a = (float)((double)out.a / a.C);
        out.b = (float)((double)out.b / a.C);
        return true;
    }
    return false;
}

__global__ void __launch_bounds__(256) k_raster_line(RBuildArgs a) {
    const int64_t SS = (int64_t)a.S * a.S;
    for (int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; m < a.n_mixed; m += (int64_t)gridDim.x * blockDim.x) {
        const int64_t g = a.mixed[m];
        const int r = (int)(g / SS), sb = (int)(g - (int64_t)r * SS), sj = sb / a.S, si = sb - sj * a.S;
        RTile t;
        tiles::LineRec lr{0, 0, 0, 0, 0};
        bool ok = false;
        if (a.lines && rtile_of(a, r, t)) {
            rbuild::P2 sq[4];
            const double stol = rsub_quad(a, t, si, sj, sq);
            ok = rtry_line(a, t, si, sj, sq, stol, lr);
        }
        a.kind[m] = ok ? 1 : 0;
        a.line[m] = ok ? lr : tiles::LineRec{0, 0, 0, 0, 0};
    }
}

// ---- k_raster_line_wave: k_raster_line with one wave per mixed sub-block -- the candidate
// hexagons, chips and rings wave-uniform, their segments spread over the lanes (ballot for "any
// segment meets", wave reductions for the longest clipped segment and the largest deviation,
// coop_contains for JTS contains).  Every decision is order-independent or reduced in the
// sequential order, so the line records are those of k_raster_line / try_line, bit for bit.
__device__ inline double wave_max_f64(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = rbuild::dmax(v, __shfl_xor(v, o, 64));
    return v;
}

// rhex_answer for a convex region ll[n] (within eps), wave-uniform result
__device__ inline int rhex_answer_wave(const RBuildArgs& a, const RTile& t, int k, double x0, double y0, double x1,
                                       double y1, const rbuild::P2* ll, int n, double eps, double cx, double cy, int* key) {
    const uint32_t e = a.entries[t.off + (uint32_t)k];
    int cnt = 0;
    *key = -1;
    if (!e) return 0;
    const HashEntry he = a.table[e - 1];
    const int lane = (int)(threadIdx.x & 63);
    for (uint32_t c = he.first; c < he.first + he.count; c++) {
        const uint32_t m = a.meta[c];
        if (!(m & 1u)) {
            const pip::Box bx = a.store.geom_bbox[c];
            if (!(bx.maxx < x0 - eps || bx.minx > x1 + eps || bx.maxy < y0 - eps || bx.miny > y1 + eps)) {
                for (uint32_t p = a.store.geom_part[c]; p < a.store.geom_part[c + 1]; p++)
                    for (uint32_t r = a.store.part_ring[p]; r < a.store.part_ring[p + 1]; r++) {
                        const uint32_t v0 = a.store.ring_start[r] + 1, v1 = a.store.ring_start[r + 1];
                        for (uint32_t base = v0; base < v1; base += 64) {
                            const uint32_t v = base + (uint32_t)lane;
                            bool hit = false;
                            if (v < v1) {
                                const pip::Vec2 s0 = a.store.verts[v - 1], s1 = a.store.verts[v];
                                hit = rbuild::seg_meets_poly(rbuild::P2{s0.x, s0.y}, rbuild::P2{s1.x, s1.y}, ll, n, eps);
                            }
                            if (__ballot(hit)) return -1;
                        }
                    }
            }
            if (!pip::coop_contains(a.store, c, cx, cy)) continue;
        }
        if (cnt == 0) *key = (int)(m >> 1);
        cnt++;
    }
    return cnt;
}

// (qc, ctol): for a leaf line, the leaf cell's corner images and tolerance -- the candidates are then
// those of the cell (tiles_build.cpp classify's cand2), as try_line's cin
__device__ inline uint16_t rclassify_poly_wave(const RBuildArgs& a, const RTile& t, int si, int sj, const rbuild::P2* uv,
                                               int n, const rbuild::P2* sq, double stol, const rbuild::P2* qc = nullptr,
                                               double ctol = 0.0, int nc = -1, int ck = 0) {
    using rbuild::dmax;
    using rbuild::dmin;
    rbuild::P2 img[8], ll[8];
    double u0 = INFINITY, u1 = -INFINITY, v0 = INFINITY, v1 = -INFINITY;
    double x0 = INFINITY, x1 = -INFINITY, y0 = INFINITY, y1 = -INFINITY, mx = 0.0, my = 0.0;
    const int S = a.S, C = a.C;
    for (int v = 0; v < n; v++) {
        img[v] = rimage(a, t, (si + uv[v].x) * C, (sj + uv[v].y) * C);
        ll[v] = rbuild::P2{t.lon0 + a.tw * (si + uv[v].x) / S, t.lat0 + a.th * (sj + uv[v].y) / S};
        u0 = dmin(u0, uv[v].x);
        u1 = dmax(u1, uv[v].x);
        v0 = dmin(v0, uv[v].y);
        v1 = dmax(v1, uv[v].y);
        x0 = dmin(x0, ll[v].x);
        x1 = dmax(x1, ll[v].x);
        y0 = dmin(y0, ll[v].y);
        y1 = dmax(y1, ll[v].y);
        mx += ll[v].x;
        my += ll[v].y;
    }
    mx /= n;
    my /= n;
    const double eps = dmax(t.exd, t.eyd);
    const double tol = tiles::poly_tol(t.cv, a.tw * (u1 - u0) / S, a.th * (v1 - v0) / S, eps);
    bool any = false;
    int acnt = 0, akey = -1;
    const int W = t.wa * t.wb, lane = (int)(threadIdx.x & 63);
    // nc >= 0: the candidates are given (lane j < nc holds window hexagon ck, ascending), the sq / qc
    // filters already applied
    const bool listm = nc >= 0;
    for (int k0 = 0; k0 < (listm ? 1 : W); k0 += 64) {
        // the window hexagons of this chunk that are candidates, one lane each, in order
        const int kl = listm ? (lane < nc ? ck : -1) : k0 + lane;
        bool is_c = false;
        if (listm ? kl >= 0 : kl < W) {
            const rbuild::P2 c = rhex_centre(t, kl);
            is_c = (listm || (rbuild::poly_meets_hex(sq, 4, c, stol, a.ht) && (!qc || rbuild::poly_meets_hex(qc, 4, c, ctol, a.ht)))) &&
                   rbuild::poly_meets_hex(img, n, c, tol, a.ht);
        }
        for (unsigned long long mask = __ballot(is_c); mask; mask &= mask - 1) {
            const int k = listm ? __shfl(ck, __builtin_ctzll(mask), 64) : k0 + __builtin_ctzll(mask);
            int key;
            const int cnt = rhex_answer_wave(a, t, k, x0, y0, x1, y1, ll, n, eps, mx, my, &key);
            if (cnt < 0 || cnt > 1) return tiles::kMixed;
            if (!any) {
                any = true;
                acnt = cnt;
                akey = key;
            } else if (cnt != acnt || key != akey) {
                return tiles::kMixed;
            }
        }
    }
    if (!any) return tiles::kMixed;
    return acnt == 0 ? (uint16_t)0 : (uint16_t)(akey + 1);
}

// tiles_build.cpp try_line() over the box [u0, u1] x [v0, v1] (sub-block units; the whole sub-block
// or, for a leaf line, one leaf cell whose corner images and tolerance are qc, ctol), margins
// 0 .. mk_end - 1
__device__ inline bool rtry_line_wave(const RBuildArgs& a, const RTile& t, int si, int sj, const rbuild::P2* sq,
                                      double stol, tiles::LineRec& out, double u0 = 0.0, double v0 = 0.0,
                                      double u1 = 1.0, double v1 = 1.0, int mk_end = 4, const rbuild::P2* qc = nullptr,
                                      double ctol = 0.0, int nc = -1, int ck = 0, bool tf = true) {
    // tf: a sub-block line, tile frame (rbuild::line_slack_tile); else a leaf line, sub-block frame
    const bool listm = nc >= 0;  // the candidates given (rclassify_poly_wave's nc, ck)
    const int S = a.S, lane = (int)(threadIdx.x & 63);
    const double wR = a.tw / S, hR = a.th / S;
    const double lonR0 = t.lon0 + a.tw * si / S, latR0 = t.lat0 + a.th * sj / S;
    const double exu = t.exd / wR, eyv = t.eyd / hR;
    const double bx0 = lonR0 + wR * u0 - t.exd, bx1 = lonR0 + wR * u1 + t.exd, by0 = latR0 + hR * v0 - t.eyd,
                 by1 = latR0 + hR * v1 + t.eyd;
    // pass 0: this lane's longest clipped segment (first in (hexagon, vertex) order on ties); pass
    // 1: this lane's largest deviation; then wave reductions
    double best = 0.0, dev_max = 0.0, la = 0.0, lb = 0.0, lc = 0.0;
    uint64_t best_key = ~0ull;
    rbuild::P2 pa{0, 0}, pb{0, 0}, ta{0, 0}, tb{0, 0};
    const int W = t.wa * t.wb;
    if (W <= 0) return false;
    for (int pass = 0; pass < 2; pass++)
        for (int k0 = 0; k0 < (listm ? 1 : W); k0 += 64) {
        const int kl = listm ? (lane < nc ? ck : -1) : k0 + lane;
        const bool is_c = (listm ? kl >= 0 : kl < W) && a.entries[t.off + (uint32_t)kl] &&
                          (listm || (rbuild::poly_meets_hex(sq, 4, rhex_centre(t, kl), stol, a.ht) &&
                                     (!qc || rbuild::poly_meets_hex(qc, 4, rhex_centre(t, kl), ctol, a.ht))));
        for (unsigned long long mask = __ballot(is_c); mask; mask &= mask - 1) {
            const int k = listm ? __shfl(ck, __builtin_ctzll(mask), 64) : k0 + __builtin_ctzll(mask);
            const uint32_t e = a.entries[t.off + (uint32_t)k];
            const HashEntry he = a.table[e - 1];
            for (uint32_t c = he.first; c < he.first + he.count; c++) {
                if (a.meta[c] & 1u) continue;
                const pip::Box bx = a.store.geom_bbox[c];
                if (bx.maxx < bx0 || bx.minx > bx1 || bx.maxy < by0 || bx.miny > by1) continue;
                for (uint32_t p = a.store.geom_part[c]; p < a.store.geom_part[c + 1]; p++)
                    for (uint32_t r = a.store.part_ring[p]; r < a.store.part_ring[p + 1]; r++) {
                        const uint32_t vend = a.store.ring_start[r + 1];
                        for (uint32_t v = a.store.ring_start[r] + 1 + (uint32_t)lane; v < vend; v += 64) {
                            const pip::Vec2 s0 = a.store.verts[v - 1], s1 = a.store.verts[v];
                            double ax = (s0.x - lonR0) / wR, ay = (s0.y - latR0) / hR;
                            double qx = (s1.x - lonR0) / wR, qy = (s1.y - latR0) / hR;
                            if (!rbuild::clip_seg(ax, ay, qx, qy, u0 - exu, v0 - eyv, u1 + exu, v1 + eyv)) continue;
                            if (pass == 0) {
                                const double l2 = (qx - ax) * (qx - ax) + (qy - ay) * (qy - ay);
                                if (l2 > best) {  // a lane's segments come in increasing order
                                    best = l2;
                                    best_key = ((uint64_t)(uint32_t)k << 32) | v;
                                    pa = rbuild::P2{ax, ay};
                                    pb = rbuild::P2{qx, qy};
                                    ta = rbuild::P2{(s0.x - t.lon0) / wR, (s0.y - t.lat0) / hR};
                                    tb = rbuild::P2{(s1.x - t.lon0) / wR, (s1.y - t.lat0) / hR};
                                }
                            } else if (tf) {
                                dev_max = rbuild::dmax(dev_max, fabs(la * (ax + si) + lb * (ay + sj) + lc));
                                dev_max = rbuild::dmax(dev_max, fabs(la * (qx + si) + lb * (qy + sj) + lc));
                            } else {
                                dev_max = rbuild::dmax(dev_max, fabs(la * ax + lb * ay + lc));
                                dev_max = rbuild::dmax(dev_max, fabs(la * qx + lb * qy + lc));
                            }
                        }
                    }
            }
        }
        if (pass == 0 && (listm || k0 + 64 >= W)) {
            // the sequential choice: the largest l2, and of equal ones the first in order
            double bl = best;
            uint64_t bk = best_key;
            int bw = lane;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) {
                const double ol = __shfl_xor(bl, o, 64);
                const uint64_t ok = __shfl_xor(bk, o, 64);
                const int ow = __shfl_xor(bw, o, 64);
                if (ol > bl || (ol == bl && ok < bk)) {
                    bl = ol;
                    bk = ok;
                    bw = ow;
                }
            }
            best = bl;
            if (!(best > 1e-6)) return false;
            if (tf) {
                ta = rbuild::P2{__shfl(ta.x, bw, 64), __shfl(ta.y, bw, 64)};
                tb = rbuild::P2{__shfl(tb.x, bw, 64), __shfl(tb.y, bw, 64)};
                const double lt = sqrt((tb.x - ta.x) * (tb.x - ta.x) + (tb.y - ta.y) * (tb.y - ta.y));
                la = -(tb.y - ta.y) / lt;
                lb = (tb.x - ta.x) / lt;
                lc = -(la * 0.5 * (ta.x + tb.x) + lb * 0.5 * (ta.y + tb.y));
            } else {
                pa = rbuild::P2{__shfl(pa.x, bw, 64), __shfl(pa.y, bw, 64)};
                pb = rbuild::P2{__shfl(pb.x, bw, 64), __shfl(pb.y, bw, 64)};
                const double l = sqrt(best);
                la = -(pb.y - pa.y) / l;
                lb = (pb.x - pa.x) / l;
                lc = -(la * 0.5 * (pa.x + pb.x) + lb * 0.5 * (pa.y + pb.y));
            }
        }
    }
    dev_max = wave_max_f64(dev_max);
    const rbuild::P2 sqb[4] = {{u0 - exu, v0 - eyv}, {u1 + exu, v0 - eyv}, {u1 + exu, v1 + eyv}, {u0 - exu, v1 + eyv}};
    for (int mk = 0; mk < mk_end; mk++) {
        const double margin = rbuild::line_margin(mk);
        if (dev_max > margin - 2.0 * tiles::kLineSlack) continue;
        out.a = (float)(la / margin);
        out.b = (float)(lb / margin);
        out.c = (float)(lc / margin);
        const double A = out.a, B = out.b;
        const double Cf = tf ? (double)out.c + A * si + B * sj : (double)out.c;
        const double m = 1.0 - (tf ? rbuild::line_slack_tile(A, B, out.c, S, tiles::kLineSlack) : tiles::kLineSlack / margin);
        rbuild::P2 hp[8], hn[8];
        const int np = rbuild::clip_half(sqb, 4, A, B, Cf - m, hp), nn = rbuild::clip_half(sqb, 4, -A, -B, -Cf - m, hn);
        const uint16_t cp = np >= 3 ? rclassify_poly_wave(a, t, si, sj, hp, np, sq, stol, qc, ctol, nc, ck) : (uint16_t)0;
        if (cp == tiles::kMixed) continue;
        const uint16_t cn = nn >= 3 ? rclassify_poly_wave(a, t, si, sj, hn, nn, sq, stol, qc, ctol, nc, ck) : (uint16_t)0;
        if (cn == tiles::kMixed) continue;
        out.pos = cp;
        out.neg = cn;
        out.a = (float)((double)out.a / a.C);
        out.b = (float)((double)out.b / a.C);
        return true;
    }
    return false;
}

// (measurement builds may constrain the raster classification kernels' occupancy: MOSAIC_RASTER_WAVES)
#if defined(MOSAIC_RASTER_WAVES)
#define MOSAIC_RASTER_ATTR __attribute__((amdgpu_waves_per_eu(MOSAIC_RASTER_WAVES)))
#else
#define MOSAIC_RASTER_ATTR
#endif
// one wave per mixed sub-block (waves past the end exit together)
__global__ void __launch_bounds__(256) MOSAIC_RASTER_ATTR k_raster_line_wave(RBuildArgs a) {
    const int64_t SS = (int64_t)a.S * a.S;
    const int64_t m = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (m >= a.n_mixed) return;
    const int64_t g = a.mixed[m];
    const int r = (int)(g / SS), sb = (int)(g - (int64_t)r * SS), sj = sb / a.S, si = sb - sj * a.S;
    RTile t;
    tiles::LineRec lr{0, 0, 0, 0, 0};
    bool ok = false;
    if (a.lines && rtile_of(a, r, t)) {
        rbuild::P2 sq[4];
        const double stol = rsub_quad(a, t, si, sj, sq);
        ok = rtry_line_wave(a, t, si, sj, sq, stol, lr);
    }
    if ((threadIdx.x & 63) == 0) {
        a.kind[m] = ok ? 1 : 0;
        a.line[m] = ok ? lr : tiles::LineRec{0, 0, 0, 0, 0};
    }
}

__global__ void __launch_bounds__(256) MOSAIC_RASTER_ATTR k_raster_cells(RBuildArgs a) {
    const int64_t SS = (int64_t)a.S * a.S, CC = (int64_t)a.C * a.C;
    const int64_t total = a.n_cell_sb * CC;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < total; w += (int64_t)gridDim.x * blockDim.x) {
        const int64_t m = w / CC;
        const int cc = (int)(w - m * CC), cj = cc / a.C, ci = cc - cj * a.C;
        const int64_t g = a.cell_sb[m];
        const int r = (int)(g / SS), sb = (int)(g - (int64_t)r * SS), sj = sb / a.S, si = sb - sj * a.S;
        RTile t;
        uint16_t code = tiles::kMixed;
        if (rtile_of(a, r, t)) {
            rbuild::P2 sq[4];
            const double stol = rsub_quad(a, t, si, sj, sq);
            const int i0 = si * a.C + ci, j0 = sj * a.C + cj;
            const rbuild::P2 qc[4] = {rimage(a, t, i0, j0), rimage(a, t, i0 + 1, j0), rimage(a, t, i0 + 1, j0 + 1),
                                      rimage(a, t, i0, j0 + 1)};
            code = rclassify_rect(a, t, i0, j0, i0 + 1, j0 + 1, qc, sq, stol);
        }
        a.cells[w] = code;
    }
}

// Leaf lines (tiles_build.cpp, the cell loop of classify_raster_host).  mlist: the kMixed leaf
// cells (index in `cells`, ascending).  k_sub_cands: one wave per kind-0 sub-block, its candidate
// hexagons (the window hexagons meeting the sub-block quad, as classify's `cand`) into
// cands[64 msb ..], their number in ncand[msb] (-1: more than 64).  k_raster_cell_lines: one wave
// per mixed cell, the cell's candidates among its sub-block's (cand2, ascending) and the line fit of
// k_raster_line_wave over the cell's box with those; ok[m] = 1 and out[m] = the record when one
// certifies.  (One wave per sub-block for all its cells measured slower: 83 ms for NYC res 9, the
// sub-blocks with hundreds of mixed cells serialise.)
__global__ void __launch_bounds__(256) k_sub_cands(RBuildArgs a, int32_t* cands, int32_t* ncand) {
    __shared__ int cbuf[4][64];
    const int64_t msb = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (msb >= a.n_cell_sb) return;
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6) & 3;
    const unsigned long long lt_mask = (1ULL << lane) - 1ULL;
    const int64_t SS = (int64_t)a.S * a.S;
    const int64_t g = a.cell_sb[msb];
    const int r = (int)(g / SS), sb = (int)(g - (int64_t)r * SS), sj = sb / a.S, si = sb - sj * a.S;
    RTile t;
    int nsc = 0;
    bool over = false;
    if (rtile_of(a, r, t)) {
        rbuild::P2 sq[4];
        const double stol = rsub_quad(a, t, si, sj, sq);
        const int W = t.wa * t.wb;
        for (int k0 = 0; k0 < W && !over; k0 += 64) {
            const int kl = k0 + lane;
            const bool is_c = kl < W && rbuild::poly_meets_hex(sq, 4, rhex_centre(t, kl), stol, a.ht);
            const unsigned long long mk = __ballot(is_c);
            const int cnt = __popcll(mk);
            if (nsc + cnt > 64) {
                over = true;
            } else {
                if (is_c) cbuf[wv][nsc + __popcll(mk & lt_mask)] = kl;
                nsc += cnt;
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    if (!over && lane < nsc) cands[msb * 64 + lane] = cbuf[wv][lane];
    if (lane == 0) ncand[msb] = over ? -1 : nsc;
}

// (occupancy 4, spilling, instead of the 256 VGPRs the compiler picks unconstrained: the leaf-line fits
// are chains of dependent chip / vertex loads, 63 -> ~33 ms for the NYC res-9 raster's 1 M mixed leaf
// cells, gpurun_out/r06w, profiles/r06_mixed/leaf_lines_occupancy.txt)
#if !defined(MOSAIC_CELL_LINES_WAVES)
#define MOSAIC_CELL_LINES_WAVES 4
#endif
#define MOSAIC_CELL_LINES_ATTR __attribute__((amdgpu_waves_per_eu(MOSAIC_CELL_LINES_WAVES)))
__global__ void __launch_bounds__(256) MOSAIC_CELL_LINES_ATTR k_raster_cell_lines(RBuildArgs a, const uint32_t* mlist, int64_t n_ml,
                                                           const int32_t* cands, const int32_t* ncand, uint8_t* ok,
                                                           tiles::LineRec* out) {
    __shared__ int cbuf[4][64];
    const int64_t m = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (m >= n_ml) return;
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6) & 3;
    const unsigned long long lt_mask = (1ULL << lane) - 1ULL;
    const int64_t SS = (int64_t)a.S * a.S, CC = (int64_t)a.C * a.C;
    const int64_t w = mlist[m];
    const int64_t msb = w / CC;
    const int cc = (int)(w - msb * CC), cj = cc / a.C, ci = cc - cj * a.C;
    const int64_t g = a.cell_sb[msb];
    const int r = (int)(g / SS), sb = (int)(g - (int64_t)r * SS), sj = sb / a.S, si = sb - sj * a.S;
    RTile t;
    tiles::LineRec lr{0, 0, 0, 0, 0};
    bool found = false;
    if (rtile_of(a, r, t)) {
        rbuild::P2 sq[4];
        const double stol = rsub_quad(a, t, si, sj, sq);
        const int i0 = si * a.C + ci, j0 = sj * a.C + cj;
        const rbuild::P2 qc[4] = {rimage(a, t, i0, j0), rimage(a, t, i0 + 1, j0), rimage(a, t, i0 + 1, j0 + 1),
                                  rimage(a, t, i0, j0 + 1)};
        // the cell's tolerance as rclassify_rect computes it (tiles_build.cpp classify)
        const double cell_deg_x = a.tw / a.N, cell_deg_y = a.th / a.N;
        const double ex = 1e-6 * cell_deg_x + 1e-12 * (fabs(t.lon0) + 1.0);
        const double ey = 1e-6 * cell_deg_y + 1e-12 * (fabs(t.lat0) + 1.0);
        const double ctol = tiles::rect_tol(t.cv, cell_deg_x * 1, cell_deg_y * 1, rbuild::dmax(ex, ey));
        const double u0 = (double)ci / a.C, v0 = (double)cj / a.C, u1 = (double)(ci + 1) / a.C, v1 = (double)(cj + 1) / a.C;
        const int nsc = ncand[msb];
        if (nsc < 0) {
            found = rtry_line_wave(a, t, si, sj, sq, stol, lr, u0, v0, u1, v1, tiles::kLeafLineMargins, qc, ctol, -1, 0, false);
        } else {
            // the cell's candidates: the sub-block's that meet the cell quad, ascending
            const int sck = lane < nsc ? cands[msb * 64 + lane] : -1;
            const bool cin = lane < nsc && rbuild::poly_meets_hex(qc, 4, rhex_centre(t, sck), ctol, a.ht);
            const unsigned long long mk = __ballot(cin);
            if (cin) cbuf[wv][__popcll(mk & lt_mask)] = sck;
            __builtin_amdgcn_wave_barrier();
            const int ncc = __popcll(mk);
            const int cck = lane < ncc ? cbuf[wv][lane] : -1;
            found = rtry_line_wave(a, t, si, sj, sq, stol, lr, u0, v0, u1, v1, tiles::kLeafLineMargins, qc, ctol, ncc, cck, false);
        }
    }
    if (lane == 0) {
        ok[m] = found ? 1 : 0;
        out[m] = found ? lr : tiles::LineRec{0, 0, 0, 0, 0};
    }
}

struct RasterMixedCell {  // hipcub select predicate: leaf cell w is kMixed
    const uint16_t* cells;
    __host__ __device__ bool operator()(uint32_t w) const { return cells[w] == tiles::kMixed; }
};

// ---- st_intersects_aggregate over the chip join of two chip tables ----------------------------
// ST_IntersectsAggregate.update (expressions/geometry/ST_IntersectsAggregate.scala:28-39) folds
// `left.is_core || right.is_core || left.wkb intersects right.wkb` with OR over the rows of a
// (left key, right key) group, the rows being the equi-join of the two chip sets on index_id
// (ST_IntersectsBehaviors.scala:34-47).  One wave per cell of the left table: it probes the right
// table for the cell and folds every (left chip, right chip) pair of the cell into its group, held
// in a device hash keyed by (left key << 32 | right key).  A group already true skips the geometry
// test (the reference's `accumulator || ...`).  The geometry test spreads the segment pairs of two
// rings over the wave's lanes (any hit ends it), then the shell-vertex containments.
static const unsigned long long kEmptyGroup = ~0ULL;
struct IsectArgs {
    const HashEntry* ta;
    uint64_t capa;
    const uint32_t* meta_a;
    pip::GeomStore sa;
    const HashEntry* tb;
    uint64_t maskb;
    const uint32_t* meta_b;
    pip::GeomStore sb;
    int pass;                          // 0: count chip pairs, 1: fold them into groups
    unsigned long long* pair_count;    // pass 0
    unsigned long long* gkey;          // pass 1: group hash (kEmptyGroup = free)
    uint32_t* gflag;
    uint64_t gmask;
    int* overflow;
};

__device__ bool wave_intersects(const pip::GeomStore& sa, uint32_t a, const pip::GeomStore& sb, uint32_t b, int lane) {
    if (sa.geom_part[a + 1] <= sa.geom_part[a] || sb.geom_part[b + 1] <= sb.geom_part[b]) return false;
    if (!pip::boxes_meet(sa.geom_bbox[a], sb.geom_bbox[b])) return false;
    const uint32_t ra0 = sa.part_ring[sa.geom_part[a]], ra1 = sa.part_ring[sa.geom_part[a + 1]];
    const uint32_t rb0 = sb.part_ring[sb.geom_part[b]], rb1 = sb.part_ring[sb.geom_part[b + 1]];
    for (uint32_t ra = ra0; ra < ra1; ra++) {
        if (!pip::boxes_meet(sa.ring_bbox[ra], sb.geom_bbox[b])) continue;
        const uint32_t ia = sa.ring_start[ra], na = sa.ring_start[ra + 1] - ia;
        if (na < 2) continue;
        for (uint32_t rb = rb0; rb < rb1; rb++) {
            if (!pip::boxes_meet(sa.ring_bbox[ra], sb.ring_bbox[rb])) continue;
            const uint32_t ib = sb.ring_start[rb], nb = sb.ring_start[rb + 1] - ib;
            if (nb < 2) continue;
            const uint64_t total = (uint64_t)(na - 1) * (nb - 1);
            for (uint64_t base = 0; base < total; base += 64) {  // wave-uniform trip count
                const uint64_t k = base + (uint64_t)lane;
                bool hit = false;
                if (k < total) {
                    const uint32_t i = (uint32_t)(k / (nb - 1)), j = (uint32_t)(k - (uint64_t)i * (nb - 1));
                    hit = pip::segments_intersect(sa.verts[ia + i], sa.verts[ia + i + 1], sb.verts[ib + j],
                                                  sb.verts[ib + j + 1]);
                }
                if (__ballot(hit)) return true;
            }
        }
    }
    return pip::shell_vertex_in(sb, b, sa, a) || pip::shell_vertex_in(sa, a, sb, b);
}

__device__ inline uint64_t group_slot(const IsectArgs& a, unsigned long long key) {
    uint64_t s = mix64(key) & a.gmask;
    for (uint64_t probes = 0; probes <= a.gmask; probes++) {
        const unsigned long long prev = atomicCAS(&a.gkey[s], kEmptyGroup, key);
        if (prev == kEmptyGroup || prev == key) return s;
        s = (s + 1) & a.gmask;
    }
    atomicExch(a.overflow, 1);
    return ~0ULL;
}

__global__ void __launch_bounds__(256) k_isect_agg(IsectArgs a) {
    const int lane = (int)(threadIdx.x & 63);
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t slot = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; slot < a.capa; slot += nw) {
        const HashEntry e = a.ta[slot];
        if (e.key == kEmptyKey) continue;
        uint32_t fb = 0, eb = 0;
        for (uint64_t s = mix64((uint64_t)e.key) & a.maskb;; s = (s + 1) & a.maskb) {
            const HashEntry f = a.tb[s];
            if (f.key == e.key) {
                fb = f.first;
                eb = f.first + f.count;
                break;
            }
            if (f.key == kEmptyKey) break;
        }
        if (eb == fb) continue;
        if (a.pass == 0) {
            if (lane == 0) atomicAdd(a.pair_count, (unsigned long long)e.count * (eb - fb));
            continue;
        }
        for (uint32_t ca = e.first; ca < e.first + e.count; ca++)
            for (uint32_t cb = fb; cb < eb; cb++) {
                const uint32_t ma = a.meta_a[ca], mb = a.meta_b[cb];
                const unsigned long long key = ((unsigned long long)(ma >> 1) << 32) | (unsigned long long)(mb >> 1);
                uint64_t gs = 0;
                uint32_t done = 0;
                if (lane == 0) {
                    gs = group_slot(a, key);
                    done = gs == ~0ULL ? 1u : __hip_atomic_load(&a.gflag[gs], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                done = __shfl(done, 0, 64);
                if (done) continue;
                const bool hit = ((ma | mb) & 1u) || wave_intersects(a.sa, ca, a.sb, cb, lane);
                if (lane == 0 && hit) atomicOr(&a.gflag[gs], 1u);
            }
    }
}


// ---- st_intersection_aggregate's union by cell (overlay.h): units = (group, left cell slot) ----
// A unit holds the group's chip pairs of one cell.  Its piece of the union the reference folds is
// the cell for a (core, core) pair, else (the group's left chips in the cell, or the whole cell when
// one of them is core) n (its right chips, likewise).  k_isect_units lists the units (one wave per
// left cell slot, as k_isect_agg; lane 0 writes) with their edge counts, which size each unit's
// scratch; k_isect_overlay runs overlay::unit_boundary one lane per unit.
struct IsectUnit {
    uint32_t gs, slot, fb, eb;
    uint32_t flags;    // bit 0: a (core, core) pair; bit 1: a left core chip; bit 2: a right core chip
    uint32_t n_edges;  // edges of the chips the overlay reads (0 for a (core, core) unit)
    uint32_t n_parts, pad;
};

__device__ uint32_t chip_edges(const pip::GeomStore& s, uint32_t g, uint32_t* parts) {
    uint32_t n = 0;
    for (uint32_t p = s.geom_part[g]; p < s.geom_part[g + 1]; p++) n += (uint32_t)overlay::part_edges(s, p);
    *parts += s.geom_part[g + 1] - s.geom_part[g];
    return n;
}

__global__ void __launch_bounds__(256) k_isect_units(IsectArgs a, IsectUnit* units, unsigned long long* n_units,
                                                     unsigned long long cap) {
    const int lane = (int)(threadIdx.x & 63);
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t slot = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; slot < a.capa; slot += nw) {
        if (lane != 0) continue;
        const HashEntry e = a.ta[slot];
        if (e.key == kEmptyKey) continue;
        uint32_t fb = 0, eb = 0;
        for (uint64_t s = mix64((uint64_t)e.key) & a.maskb;; s = (s + 1) & a.maskb) {
            const HashEntry f = a.tb[s];
            if (f.key == e.key) {
                fb = f.first;
                eb = f.first + f.count;
                break;
            }
            if (f.key == kEmptyKey) break;
        }
        for (uint32_t ca = e.first; ca < e.first + e.count; ca++)
            for (uint32_t cb = fb; cb < eb; cb++) {
                const uint32_t L = a.meta_a[ca] >> 1, R = a.meta_b[cb] >> 1;
                // first pair of its group in this cell?
                bool first = true;
                for (uint32_t ca2 = e.first; ca2 <= ca && first; ca2++)
                    for (uint32_t cb2 = fb; cb2 < eb; cb2++) {
                        if (ca2 == ca && cb2 >= cb) break;
                        if ((a.meta_a[ca2] >> 1) == L && (a.meta_b[cb2] >> 1) == R) {
                            first = false;
                            break;
                        }
                    }
                if (!first) continue;
                uint32_t acore = 0, bcore = 0;
                for (uint32_t c = e.first; c < e.first + e.count; c++)
                    if ((a.meta_a[c] >> 1) == L) acore |= a.meta_a[c] & 1u;
                for (uint32_t c = fb; c < eb; c++)
                    if ((a.meta_b[c] >> 1) == R) bcore |= a.meta_b[c] & 1u;
                const bool cc = acore && bcore;
                uint32_t ne = 0, np = 0;
                if (!cc) {
                    if (!acore)
                        for (uint32_t c = e.first; c < e.first + e.count; c++)
                            if ((a.meta_a[c] >> 1) == L) ne += chip_edges(a.sa, c, &np);
                    if (!bcore)
                        for (uint32_t c = fb; c < eb; c++)
                            if ((a.meta_b[c] >> 1) == R) ne += chip_edges(a.sb, c, &np);
                }
                const uint64_t gs = group_slot(a, ((unsigned long long)L << 32) | R);
                if (gs == ~0ULL) continue;
                const unsigned long long u = atomicAdd(n_units, 1ULL);
                if (u < cap) {
                    IsectUnit x;
                    x.gs = (uint32_t)gs;
                    x.slot = (uint32_t)slot;
                    x.fb = fb;
                    x.eb = eb;
                    x.flags = (cc ? 1u : 0u) | (acore ? 2u : 0u) | (bcore ? 4u : 0u);
                    x.n_edges = ne;
                    x.n_parts = np;
                    x.pad = 0;
                    units[u] = x;
                }
            }
    }
}

struct OverlayArgs {
    IsectArgs base;
    const IsectUnit* units;
    const uint32_t* order;  // processing order: largest units first
    uint64_t n_units;
    const int64_t* scratch_off;  // bytes into scratch, per unit
    char* scratch;
    const int64_t* out_off;  // edges into out, per unit
    double* out;             // 4 doubles per edge
    int32_t* out_count;      // edges, -1: a capacity exceeded
    double* out_area;
    int grid, jdk;
};

__device__ int cell_ring(int grid, int64_t id, int jdk, double* xy) {  // indexToGeometry's ring, open, ccw
    int n = 0;
    if (grid == MOSAIC_GRID_BNG) {
        int r;
        int32_t e, x, y;
        if (!bng::cell_origin(id, &r, &e, &x, &y)) return 0;
        const double X = x, Y = y, E = e;
        const double v[8] = {X, Y, X + E, Y, X + E, Y + E, X, Y + E};
        for (int i = 0; i < 8; i++) xy[i] = v[i];
        return 4;
    }
    double v[20];
    n = h3geom::h3_to_geo_boundary((uint64_t)id, v);
    if (n <= 0) return 0;
    for (int k = 0; k < n; k++) xy[2 * k] = h3geom::to_degrees(v[2 * k + 1], jdk), xy[2 * k + 1] = h3geom::to_degrees(v[2 * k], jdk);
    double s = 0;
    for (int k = 0; k < n; k++) {
        const int j = k + 1 == n ? 0 : k + 1;
        s += (xy[2 * k] - xy[0]) * (xy[2 * j + 1] - xy[1]) - (xy[2 * j] - xy[0]) * (xy[2 * k + 1] - xy[1]);
    }
    if (s < 0)
        for (int k = 0; k < n / 2; k++) {
            const double tx = xy[2 * k], ty = xy[2 * k + 1];
            xy[2 * k] = xy[2 * (n - 1 - k)], xy[2 * k + 1] = xy[2 * (n - 1 - k) + 1];
            xy[2 * (n - 1 - k)] = tx, xy[2 * (n - 1 - k) + 1] = ty;
        }
    return n;
}

// one unit per wave (lane 0): a unit's overlay is sequential, data-dependent work, so units that
// shared a wave would serialise behind its largest; largest units first, for the tail
// the largest unit (edges of its chip parts) one lane overlays: 16384^2 noding steps, ~1.5 s -- above
// every unit of the 263 NYC zones against a translated copy down to res 5 (15,358 edges; 4,096, the
// round-5 limit, refused 6 groups at res 7, the reference's test resolution, and 147 at res 5)
static constexpr uint32_t kMaxUnitEdges = 16384;
__global__ void __launch_bounds__(64) k_isect_overlay(OverlayArgs x) {
    const IsectArgs& a = x.base;
    if ((threadIdx.x & 63) != 0) return;
    const uint64_t step = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < x.n_units; i += step) {
        const uint64_t u = x.order[i];
        const IsectUnit un = x.units[u];
        double* out = x.out + 4 * x.out_off[u];
        const int out_cap = (int)(x.out_off[u + 1] - x.out_off[u]);
        const HashEntry e = a.ta[un.slot];
        if (un.flags & 1u) {
            double xy[20];
            const int n = cell_ring(x.grid, e.key, x.jdk, xy);
            double acc = 0;
            for (int k = 0; k < n && k < out_cap; k++) {
                const int j = k + 1 == n ? 0 : k + 1;
                out[4 * k] = xy[2 * k], out[4 * k + 1] = xy[2 * k + 1], out[4 * k + 2] = xy[2 * j], out[4 * k + 3] = xy[2 * j + 1];
                acc += (xy[2 * k] - xy[0]) * (xy[2 * j + 1] - xy[1]) - (xy[2 * j] - xy[0]) * (xy[2 * k + 1] - xy[1]);
            }
            x.out_count[u] = n > 0 && n <= out_cap ? n : -1;
            x.out_area[u] = 0.5 * acc;
            continue;
        }
        if (un.n_edges > kMaxUnitEdges) {
            // one lane's noding is O(E^2) dependent steps: a unit beyond the limit is not answered
            // (count -1: its group gets status 1, area NaN) instead of holding the lane for seconds
            x.out_count[u] = -1;
            x.out_area[u] = NAN;
            continue;
        }
        const unsigned long long key = a.gkey[un.gs];
        const uint32_t L = (uint32_t)(key >> 32), R = (uint32_t)key;
        char* base = x.scratch + x.scratch_off[u];
        overlay::PartRef* parts = (overlay::PartRef*)base;
        int np = 0;
        if (!(un.flags & 2u))
            for (uint32_t c = e.first; c < e.first + e.count; c++)
                if ((a.meta_a[c] >> 1) == L)
                    for (uint32_t p = a.sa.geom_part[c]; p < a.sa.geom_part[c + 1]; p++) parts[np++] = overlay::PartRef{p, 0, 0, 0};
        if (!(un.flags & 4u))
            for (uint32_t c = un.fb; c < un.eb; c++)
                if ((a.meta_b[c] >> 1) == R)
                    for (uint32_t p = a.sb.geom_part[c]; p < a.sb.geom_part[c + 1]; p++) parts[np++] = overlay::PartRef{p, 1, 0, 0};
        overlay::Scratch sc = overlay::make_scratch(base + (((int64_t)un.n_parts * sizeof(overlay::PartRef) + 63) & ~(int64_t)63),
                                                    un.n_edges);
        const pip::GeomStore st[2] = {a.sa, a.sb};
        const int need = ((un.flags & 2u) ? 0 : overlay::kNeedA) | ((un.flags & 4u) ? 0 : overlay::kNeedB);
        double area = 0;
        x.out_count[u] = overlay::unit_boundary(st, parts, np, need, sc, out, out_cap, &area);
        x.out_area[u] = area;
    }
}


// ---- grid_cellkring / grid_cellkloop over a BNG cell column (BNGIndexSystem.kRing / kLoop,
// BNGIndexSystem.scala:216-246): one lane per row writes its cells to a fixed-stride slot
// (8k for a loop, 1 + 4k(k + 1) for a ring) and the count; null rows get count -1 (NullIntolerant).
struct KringArgs {
    const int64_t* cells;
    const uint8_t* valid;
    int64_t n;
    int k, loop;
    int64_t stride;
    int64_t* out;
    int32_t* count;
    unsigned int* flags;  // bit 0: an id the reference cannot decode
};
__global__ void __launch_bounds__(256) k_bng_kring(KringArgs a) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    bool bad = false;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += step) {
        if (a.valid && !a.valid[i]) {
            a.count[i] = -1;
            continue;
        }
        int64_t* o = a.out + i * a.stride;
        const int m = a.loop ? bng::kloop(a.cells[i], a.k, o) : bng::kring(a.cells[i], a.k, o);
        if (m < 0) bad = true;
        a.count[i] = m < 0 ? 0 : m;
    }
    if (bad) atomicOr(a.flags, 1u);
}

// grid_cellkring / grid_cellkloop over H3 cells (h3_neighbors.h): one lane per row, H3's hexRange /
// hexRing walk; rows where H3 meets a pentagon get count -3 and are finished by k_h3_kring_slow
// (H3's _kRingInternal; the reference's set-difference fallback for kLoop); invalid ids -2.
__global__ void __launch_bounds__(256) k_h3_kring(KringArgs a) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += step) {
        if (a.valid && !a.valid[i]) {
            a.count[i] = -1;
            continue;
        }
        a.count[i] = h3nb::kring_fast((uint64_t)a.cells[i], a.k, a.loop, a.out + i * a.stride);
    }
}

// the -3 rows of k_h3_kring (rows[0 .. n_rows)), with per-row scratch (tables, distances, the
// depth-first stack), `lanes` rows per 64-lane workgroup: 64 for small k, 1 for large k (H3's
// search makes ~5 k^3 dependent visits per row, so rows sharing a wave would serialise)
__global__ void __launch_bounds__(64) k_h3_kring_slow(KringArgs a, const int64_t* rows, int64_t n_rows, int lanes,
                                                      int64_t* tab, int64_t tab_stride, int32_t* dist,
                                                      int64_t dist_stride, uint64_t* stack) {
    if ((int)threadIdx.x >= lanes) return;
    const int64_t t = (int64_t)blockIdx.x * lanes + threadIdx.x;
    if (t >= n_rows) return;
    const int64_t i = rows[t];
    a.count[i] = h3nb::kring_slow((uint64_t)a.cells[i], a.k, a.loop, a.out + i * a.stride, tab + t * tab_stride,
                                  dist + t * dist_stride, stack + t * (int64_t)(a.k + 1));
}


// ---- serializeCellId for BNG (IndexSystem.scala:37-46 -> BNGIndexSystem.format :114-129) over a
// cell column, output in Arrow utf8 layout: k_bng_format_len writes each row's length (0 for null
// rows) to offsets[i + 1], an inclusive scan turns them into offsets, k_bng_format_write writes the
// characters.  Ids the reference cannot format set flags bit 0.
struct FormatArgs {
    const int64_t* ids;
    const uint8_t* valid;
    int64_t n;
    int64_t* offsets;  // n + 1
    char* chars;
    unsigned int* flags;
};
__global__ void __launch_bounds__(256) k_bng_format_len(FormatArgs a) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    bool bad = false;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += step) {
        int len = 0;
        if (!a.valid || a.valid[i]) {
            len = bng::format_id(a.ids[i], nullptr);
            if (len < 0) {
                bad = true;
                len = 0;
            }
        }
        a.offsets[i + 1] = len;
    }
    if (bad) atomicOr(a.flags, 1u);
}
__global__ void __launch_bounds__(256) k_bng_format_write(FormatArgs a) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += step) {
        if (a.valid && !a.valid[i]) continue;
        char buf[16];
        const int len = bng::format_id(a.ids[i], buf);
        char* o = a.chars + a.offsets[i];
        int j = 0;
        // whole aligned 4-byte words where the row's start allows (a column of one resolution has
        // equal lengths, so its rows start 4-aligned whenever the length is a multiple of 4)
        if ((((uintptr_t)o) & 3) == 0)
            for (; j + 4 <= len; j += 4) {
                uint32_t w = (uint32_t)(uint8_t)buf[j] | ((uint32_t)(uint8_t)buf[j + 1] << 8) |
                             ((uint32_t)(uint8_t)buf[j + 2] << 16) | ((uint32_t)(uint8_t)buf[j + 3] << 24);
                *(uint32_t*)(o + j) = w;
            }
        for (; j < len; j++) o[j] = buf[j];
    }
}
__global__ void k_add_prev(int64_t* first, const int64_t* prev_total) { *first += *prev_total; }

// BNGIndexSystem.parse over a string column (Arrow utf8 / large_utf8): one lane per row, the row's
// characters read from global memory (ids are <= 16 characters).  Rows the reference cannot parse
// get id 0 and set flags bit 0; null rows (valid[i] == 0) get 0.
struct ParseArgs {
    const void* offsets;
    int off64;
    const uint8_t* chars;
    const uint8_t* valid;
    int64_t n;
    int64_t* ids;
    unsigned long long* first_bad;  // smallest unparseable row (atomicMin), ~0 if none
};
__global__ void __launch_bounds__(256) k_bng_parse(ParseArgs a) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += step) {
        int64_t id = 0;
        if (!a.valid || a.valid[i]) {
            const int64_t o0 = a.off64 ? ((const int64_t*)a.offsets)[i] : ((const int32_t*)a.offsets)[i];
            const int64_t o1 = a.off64 ? ((const int64_t*)a.offsets)[i + 1] : ((const int32_t*)a.offsets)[i + 1];
            char buf[24];
            const int len = (int)(o1 - o0);
            bool ok = len >= 0 && len <= 24;
            if (ok) {
                for (int j = 0; j < len; j++) buf[j] = (char)a.chars[o0 + j];
                ok = bng::parse(buf, len, &id);
            }
            if (!ok) {
                id = 0;
                atomicMin(a.first_bad, (unsigned long long)i);
            }
        }
        a.ids[i] = id;
    }
}

// The COORDS form of a point (InternalGeometryType, core/types/model/InternalGeometry.scala,
// the output of st_point: expressions/constructors/ST_Point.scala:27-32) as Arrow columns:
// type_id[n] (int32), boundaries list offsets bnd[n + 1] (rows -> boundaries), ring offsets
// ring[] (boundaries -> coordinates), coordinate offsets crd[] (coordinates -> values), values
// (float64).  MosaicPointJTS.fromInternal (core/geometry/point/MosaicPointJTS.scala:82-89) reads
// boundaries.head.head: x = values[0], y = values[1] of the first coordinate of the first
// boundary; InternalCoord(ArrayData) (InternalCoord.scala) needs 2 values, or >= 3 (z ignored).
// Rows of other types (their centroid) and rows the reference would throw on (no boundary, no
// coordinate, a 1-value coordinate) go to the row path.
struct CoordsArgs {
    const int32_t* type_id;
    const int32_t* bnd;
    const int32_t* ring;
    const int32_t* crd;
    const double* values;
    const uint8_t* valid;
    int64_t n, n_bnd, n_ring, n_values;  // lengths of ring[] and crd[] offset arrays (+1), values
    double* x;
    double* y;
    uint8_t* status;
    unsigned long long* n_rowpath;
};
__global__ void __launch_bounds__(256) k_decode_coords(CoordsArgs a) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    unsigned int rowpath = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += step) {
        uint8_t st = MOSAIC_ROW_NULL;
        double x = 0.0, y = 0.0;
        if (!a.valid || a.valid[i]) {
            st = MOSAIC_ROW_PATH;
            if (a.type_id[i] == 1) {  // GeometryTypeEnum.POINT
                const int64_t b0 = a.bnd[i], b1 = a.bnd[i + 1];
                if (b1 > b0 && b0 >= 0 && b0 + 1 < a.n_bnd) {
                    const int64_t r0 = a.ring[b0], r1 = a.ring[b0 + 1];
                    if (r1 > r0 && r0 >= 0 && r0 + 1 < a.n_ring) {
                        const int64_t c0 = a.crd[r0], c1 = a.crd[r0 + 1];
                        const int64_t len = c1 - c0;
                        if ((len == 2 || len >= 3) && c0 >= 0 && c0 + 1 < a.n_values) {
                            x = a.values[c0];
                            y = a.values[c0 + 1];
                            st = MOSAIC_ROW_OK;
                        }
                    }
                }
            }
        }
        rowpath += st == MOSAIC_ROW_PATH;
        a.x[i] = x;
        a.y[i] = y;
        a.status[i] = st;
    }
    for (int off = 32; off > 0; off >>= 1) rowpath += __shfl_down(rowpath, off, 64);
    if ((threadIdx.x & 63) == 0 && rowpath) atomicAdd(a.n_rowpath, (unsigned long long)rowpath);
}


// ---- grid_boundaryaswkb over a BNG cell column (IndexGeometry -> BNGIndexSystem.indexToGeometry,
// toWKB): 93 bytes per row at out + 93 i; null rows are left untouched (the caller's validity).
__global__ void __launch_bounds__(256) k_bng_cell_wkb(const int64_t* ids, const uint8_t* valid, int64_t n,
                                                      uint8_t* out, unsigned int* flags) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    bool bad = false;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
        if (valid && !valid[i]) continue;
        if (!bng::cell_wkb(ids[i], out + i * bng::kCellWkbBytes)) bad = true;
    }
    if (bad) atomicOr(flags, 1u);
}

// ---- H3 cell geometry over a cell column (h3_geom.h): mode 0 h3ToGeo centres, 1 h3ToGeoBoundary
// vertices, 2 grid_boundaryaswkb (IndexGeometry -> H3IndexSystem.indexToGeometry -> toWKB: the
// boundary closed with its first vertex, JTS big-endian 2D WKB, x = lng, y = lat in degrees through
// java.lang.Math.toDegrees).  One lane per row; invalid ids set flags bit 0.
static const int kH3WkbStride = 13 + 16 * 11;  // <= 10 boundary vertices + the closing point
__global__ void __launch_bounds__(256) k_h3_geom(const int64_t* ids, const uint8_t* valid, int64_t n, int mode,
                                                 int jdk, void* out, int32_t* count, unsigned int* flags) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    bool bad = false;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
        if (valid && !valid[i]) {
            count[i] = -1;
            continue;
        }
        double v[20];
        int nv;
        if (mode == 0) {
            nv = h3geom::h3_to_geo((uint64_t)ids[i], &v[0], &v[1]) ? 1 : -1;
        } else {
            nv = h3geom::h3_to_geo_boundary((uint64_t)ids[i], v);
        }
        if (nv < 0) {
            bad = true;
            count[i] = 0;
            continue;
        }
        if (mode < 2) {
            double* o = (double*)out + (mode == 0 ? 2 : 20) * i;
            for (int k = 0; k < nv; k++) {
                o[2 * k] = h3geom::to_degrees(v[2 * k + 1], jdk);  // x = lng
                o[2 * k + 1] = h3geom::to_degrees(v[2 * k], jdk);  // y = lat
            }
            count[i] = nv;
        } else {
            uint8_t* o = (uint8_t*)out + (int64_t)kH3WkbStride * i;
            o[0] = 0;  // big-endian
            bng::put_be_u32(o + 1, 3);
            bng::put_be_u32(o + 5, 1);
            bng::put_be_u32(o + 9, (uint32_t)(nv + 1));
            for (int k = 0; k <= nv; k++) {
                const int q = k == nv ? 0 : k;
                bng::put_be_f64(o + 13 + 16 * k, h3geom::to_degrees(v[2 * q + 1], jdk));
                bng::put_be_f64(o + 21 + 16 * k, h3geom::to_degrees(v[2 * q], jdk));
            }
            count[i] = 13 + 16 * (nv + 1);
        }
    }
    if (bad) atomicOr(flags, 1u);
}

// Rows of the BNG dense table's mixed sub-cells (and rows outside its one-to-one range), R rows per
// lane: coordinates, cell (BNGIndexSystem.pointToIndex), first hash probe of all R rows issued
// together (R independent chains per lane, as k_join_mixed), then the raster chip loop per row slot.
template <bool LDS_COUNTS, bool PAIRS, int R>
__global__ void __launch_bounds__(256) k_join_mixed_bng(JoinArgs a) {
    extern __shared__ unsigned int lds[];
    __shared__ SlabItem items[4][16];
    counts_init<LDS_COUNTS>(a, lds);
    unsigned int tests = 0;
    const int lane = (int)(threadIdx.x & 63);
    const int wv = (int)(threadIdx.x >> 6) & 3;
    const unsigned long long total = *a.mixq_count;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x * R;
    for (unsigned long long w0 = ((unsigned long long)blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) * R; w0 < total;
         w0 += stride) {
        int64_t row[R], cell[R];
        double x[R], y[R];
        bool live[R];
        uint32_t cur[R], end[R];
        uint64_t slot[R];
#pragma unroll
        for (int k = 0; k < R; k++) {
            const unsigned long long t = w0 + (unsigned long long)(k * 64 + lane);
            live[k] = t < total;
            row[k] = a.row_lo + (live[k] ? (int64_t)a.mixq[t] : 0);
        }
#pragma unroll
        for (int k = 0; k < R; k++) {
            x[k] = a.x[row[k]];
            y[k] = a.y[row[k]];
        }
        // wedge sub-cells (tiles.h bng_leaf_blocks wedges): the stream kernels' cell and sub-cell
        // arithmetic, the leaf code, and for a wedge code the two records -- a point outside both
        // bands is answered here and skips the chip loop
        bool done[R];
#pragma unroll
        for (int k = 0; k < R; k++) {
            done[k] = false;
            if (!a.bng_wedge || !live[k] || x[k] != x[k] || y[k] != y[k]) continue;
            const int32_t eI = bng::jvm_d2i(x[k]), nI = bng::jvm_d2i(y[k]);
            if (!((uint32_t)eI < 10000000u && (uint32_t)nI < 10000000u)) continue;
            const double xe = (double)eI, ye = (double)nI, inv_div = 1.0 / (double)a.bng_div;
            const int32_t qe = (int32_t)fma(xe, inv_div, 1e-7), qn = (int32_t)fma(ye, inv_div, 1e-7);
            const int32_t ce = qe - a.bng_e0, cn = qn - a.bng_n0;
            if (!((uint32_t)ce < (uint32_t)a.bng_ne && (uint32_t)cn < (uint32_t)a.bng_nn)) continue;
            const uint32_t e = a.bng_cells[(int64_t)cn * a.bng_ne + ce];
            if ((e & (kBngPure | kBngLeaf)) != kBngLeaf) continue;
            const uint32_t base = e & ~kBngLeaf;
            const float ff = (float)((double)a.bng_C / (double)a.bng_div);
            const float gxs = fmaf((float)(eI - (int32_t)__umul24((uint32_t)qe, (uint32_t)a.bng_div)), ff, (float)(x[k] - xe) * ff);
            const float gys = fmaf((float)(nI - (int32_t)__umul24((uint32_t)qn, (uint32_t)a.bng_div)), ff, (float)(y[k] - ye) * ff);
            const int sx = min(max((int)gxs, 0), a.bng_C - 1), sy = min(max((int)gys, 0), a.bng_C - 1);
            const uint32_t code = a.bng_leaf[base + (uint32_t)(sy * a.bng_C + sx)];
            if (code - 0x8000u >= 0x4000u) continue;
            const uint32_t nrec = code & 0x3fffu;
            const tiles::LineRec r1 = *(const tiles::LineRec*)(a.bng_leaf + base - 8u * (nrec + 1u));
            const tiles::LineRec r2 = *(const tiles::LineRec*)(a.bng_leaf + base - 8u * (nrec + 2u));
            const uint32_t w = tiles::bng_wedge_code(r1, r2, gxs, gys);
            if (w == (uint32_t)tiles::kMixed) continue;
            if (w) emit_hit<LDS_COUNTS, PAIRS>(a, row[k], w - 1u, lds);
            done[k] = true;
        }
#pragma unroll
        for (int k = 0; k < R; k++) {
            // NaN: flagged by the stream kernel, no pair
            if (!live[k] || done[k] || !bng::point_to_index(x[k], y[k], a.res, &cell[k])) cell[k] = kEmptyKey;
            slot[k] = mix64((uint64_t)cell[k]) & a.mask;
        }
        HashEntry he[R];
#pragma unroll
        for (int k = 0; k < R; k++) he[k] = a.table[slot[k]];
#pragma unroll
        for (int k = 0; k < R; k++) {
            cur[k] = end[k] = 0;
            if (cell[k] == kEmptyKey) continue;
            while (he[k].key != cell[k] && he[k].key != kEmptyKey) {  // linear probing (rare)
                slot[k] = (slot[k] + 1) & a.mask;
                he[k] = a.table[slot[k]];
            }
            if (he[k].key == cell[k]) {
                cur[k] = he[k].first;
                end[k] = he[k].first + he[k].count;
            }
        }
#pragma unroll
        for (int k = 0; k < R; k++)
            raster_chips<LDS_COUNTS, PAIRS>(a, live[k] ? row[k] : -1, cur[k], end[k], x[k], y[k], tests, lds, items[wv]);
    }
    counts_flush<LDS_COUNTS>(a, lds, tests);
}

// Rows of mixed raster cells (the dense queue mixq), R rows per lane: their chip ranges are found
// stage by stage for all R rows at once (coordinate gathers, tile codes, tile records, projection,
// window entries, hash entries -- R independent chains in flight per lane instead of one), then the
// raster chip loop runs once per row slot (wave-cooperative, so wave-uniform).  Rows the fast path
// cannot certify, kFull tiles and window misses take tiled_cell (the generic path).
template <bool LDS_COUNTS, bool PAIRS, int R>
#if !defined(MOSAIC_MIXED_WAVES)
#define MOSAIC_MIXED_WAVES 4
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MOSAIC_MIXED_WAVES))) k_join_mixed(JoinArgs a) {
    extern __shared__ unsigned int lds[];
    __shared__ SlabItem items[4][16];
    counts_init<LDS_COUNTS>(a, lds);
    unsigned int tests = 0;
    const int lane = (int)(threadIdx.x & 63);
    const int wv = (int)(threadIdx.x >> 6) & 3;
    const unsigned long long total = *a.mixq_count;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x * R;
    // wave-uniform loop: the wave's rows are [w0, w0 + 64 R), slot k of lane l is w0 + k * 64 + l
    for (unsigned long long w0 = ((unsigned long long)blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) * R; w0 < total;
         w0 += stride) {
        int64_t row[R];
        double x[R], y[R];
        bool live[R];
        uint32_t code[R], cur[R], end[R];
#pragma unroll
        for (int k = 0; k < R; k++) {
            const unsigned long long t = w0 + (unsigned long long)(k * 64 + lane);
            live[k] = t < total;
            row[k] = a.row_lo + (live[k] ? (int64_t)a.mixq[t] : 0);
        }
#pragma unroll
        for (int k = 0; k < R; k++) {
            x[k] = a.x[row[k]];
            y[k] = a.y[row[k]];
        }
#pragma unroll
        for (int k = 0; k < R; k++) code[k] = tiles::tile_of(a.tgrid, a.tile_idx, x[k], y[k]);
        tiles::TileRec rec[R];
#pragma unroll
        for (int k = 0; k < R; k++) rec[k] = a.tile_rec[code[k] >= 2 ? code[k] - 2 : 0];
        uint32_t ent_idx[R];
        bool fast[R];
#pragma unroll
        for (int k = 0; k < R; k++) {
            fast[k] = false;
            ent_idx[k] = 0;
            if (live[k] && code[k] >= 2) {
                const int face = (int)(rec[k].dims & 0xffu);
                const int wa = (int)((rec[k].dims >> 8) & 0xfffu), wb = (int)(rec[k].dims >> 20);
                double px, py, pz, vx, vy, best;
                h3::fast_unit(y[k], x[k], &px, &py, &pz);
                h3::fast_plane(px, py, pz, face, a.res, &vx, &vy, &best);
                int ba, bb;
                if (h3::fast_hex(vx, vy, a.res, &ba, &bb)) {
                    const int ra = ba - rec[k].a0, rb = bb - rec[k].b0;
                    if ((unsigned)ra < (unsigned)wa && (unsigned)rb < (unsigned)wb) {
                        fast[k] = true;
                        ent_idx[k] = rec[k].off + (uint32_t)(ra * wb + rb);
                    }
                }
            }
        }
        uint32_t ent[R];
#pragma unroll
        for (int k = 0; k < R; k++) ent[k] = a.tile_ent[ent_idx[k]];
        HashEntry he[R];
#pragma unroll
        for (int k = 0; k < R; k++) he[k] = a.table[fast[k] && ent[k] ? ent[k] - 1 : 0];
#pragma unroll
        for (int k = 0; k < R; k++) {
            cur[k] = end[k] = 0;
            if (!live[k]) continue;
            if (fast[k]) {
                if (ent[k]) {
                    cur[k] = he[k].first;
                    end[k] = he[k].first + he[k].count;
                }
            } else {
                tiled_cell(a, row[k], x[k], y[k], code[k], cur[k], end[k]);
            }
        }
#pragma unroll
        for (int k = 0; k < R; k++) {
            raster_chips<LDS_COUNTS, PAIRS>(a, live[k] ? row[k] : -1, cur[k], end[k], x[k], y[k], tests, lds, items[wv]);
        }
    }
    counts_flush<LDS_COUNTS>(a, lds, tests);
}

// Exact H3 for the queued rows (or for every row when all_rows is set: queue overflow fallback).
template <bool PAIRS>
__global__ void __launch_bounds__(256) k_join_h3_exact(JoinArgs a, int all_rows) {
    unsigned int tests = 0;
    unsigned long long total = all_rows ? (unsigned long long)a.n : min(*a.amb_count, a.amb_cap);
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    for (unsigned long long t = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
        int64_t i = all_rows ? (int64_t)t : (int64_t)a.amb_queue[t];
        if (a.valid && !a.valid[i]) continue;
        const int64_t k = i * a.cstride;
        double x = a.x[k], y = a.y[k];
        int64_t cell = (int64_t)h3::h3_exact(h3::to_radians(y, a.jdk), h3::to_radians(x, a.jdk), a.res);
        join_point<false, PAIRS>(a, a.rowmap ? (int64_t)a.rowmap[k] : i, x, y, cell, nullptr, tests);
    }
    counts_flush<false>(a, nullptr, tests);
}

struct CellArgs {
    const double* x;
    const double* y;
    const uint8_t* valid;
    const uint8_t* status;  // decoded point rows (k_decode_points): present iff status == kRowOk
    int64_t n;
    int res, jdk;
    long long* out;
    uint8_t* out_valid;
    unsigned long long* amb_queue;
    unsigned long long* amb_count;
    unsigned long long amb_cap;
    unsigned int* flags;
    int vec;  // x, y, out 16-byte aligned: two rows per lane as 16-byte loads / stores
};

__device__ __forceinline__ bool cell_row_present(const CellArgs& a, int64_t i) {
    return (!a.valid || a.valid[i]) && (!a.status || a.status[i] == 1);
}

// rows per lane of k_cell_h3 (compile-time; 2 unless a measurement build sets MOSAIC_CELL_ROWS)
#if defined(MOSAIC_CELL_ROWS)
static constexpr int kCellRows = MOSAIC_CELL_ROWS;
#else
static constexpr int kCellRows = 2;
#endif
// digits four levels per step (h3::kAxialQuads) in k_cell_h3 (compile-time; a measurement build may set
// MOSAIC_CELL_QUAD=0 for the pair steps alone)
#if defined(MOSAIC_CELL_QUAD)
static constexpr bool kCellQuad = MOSAIC_CELL_QUAD != 0;
#else
static constexpr bool kCellQuad = true;
#endif
// grid_longlatascellid / grid_pointascellid's cell step: two consecutive rows per lane (16-byte loads
// of x and y, one 16-byte store), the two fast paths interleaved (h3::h3_fastk_tab); rows the fast path
// cannot certify are queued for k_cell_h3_exact.
#if defined(MOSAIC_CELL_WAVES)
#define MOSAIC_CELL_ATTR __attribute__((amdgpu_waves_per_eu(MOSAIC_CELL_WAVES, MOSAIC_CELL_WAVES)))
#else
#define MOSAIC_CELL_ATTR
#endif
__global__ void __launch_bounds__(256) MOSAIC_CELL_ATTR k_cell_h3(CellArgs a) {
    // the digit tables read from LDS (12.8 vs 13.6 ms per 1e9 points for the pair table from the
    // constant table: gpurun_out/r06f, profiles/r06_cell_*), the four-level table of res's parity too
    __shared__ h3::AxialPairTab lpairs;
    __shared__ uint32_t lquad[kCellQuad ? 2401 : 1];
    for (int k = threadIdx.x; k < 98; k += blockDim.x) (&lpairs.v[0][0])[k] = (&h3::kAxialPairs.v[0][0])[k];
    if (kCellQuad) {
        const uint32_t* gq = h3::kAxialQuads.v[a.res & 1];
        for (int k = threadIdx.x; k < 2401; k += blockDim.x) lquad[k] = gq[k];
    }
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    constexpr int R = kCellRows;
    const int64_t np = (a.n + R - 1) / R;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < np; p += stride) {
        const int64_t i = R * p;
        const bool full = i + R <= a.n;
        double lat[R], lon[R];
        if (full && a.vec) {
#pragma unroll
            for (int h = 0; h < R / 2; h++) {
                const v2d xv = __builtin_nontemporal_load((const v2d*)(a.x + i) + h);
                const v2d yv = __builtin_nontemporal_load((const v2d*)(a.y + i) + h);
                lon[2 * h] = xv.x, lon[2 * h + 1] = xv.y, lat[2 * h] = yv.x, lat[2 * h + 1] = yv.y;
            }
        } else {
#pragma unroll
            for (int k = 0; k < R; k++) {
                lon[k] = i + k < a.n ? a.x[i + k] : 0.0;
                lat[k] = i + k < a.n ? a.y[i + k] : 0.0;
            }
        }
        uint64_t cell[R];
        bool amb[R], rare[R];
        h3::h3_fastk_tab<R, kCellQuad>(lat, lon, a.res, cell, amb, rare, lpairs, lquad);
#pragma unroll
        for (int k = 0; k < R; k++) {
            if (i + k >= a.n) continue;
            const bool v = cell_row_present(a, i + k);
            if (a.out_valid) a.out_valid[i + k] = v;
            if (!v) {
                cell[k] = 0;
            } else if (amb[k] || rare[k]) {
                // (rare rows -- off the face table, beyond the table sine, non-finite -- get h3_fast in
                // k_cell_h3_exact, then h3_exact if that is ambiguous too)
                unsigned long long q = atomicAdd(a.amb_count, 1ULL);
                if (q < a.amb_cap) a.amb_queue[q] = (unsigned long long)(i + k);
                else atomicOr(a.flags, 2u);
            }
        }
        if (full && a.vec) {
            typedef long long v2ll __attribute__((ext_vector_type(2)));
#pragma unroll
            for (int h = 0; h < R / 2; h++) {
                v2ll o;
                o.x = (long long)cell[2 * h];
                o.y = (long long)cell[2 * h + 1];
                __builtin_nontemporal_store(o, (v2ll*)(a.out + i) + h);
            }
        } else {
#pragma unroll
            for (int k = 0; k < R; k++)
                if (i + k < a.n) a.out[i + k] = (long long)cell[k];
        }
    }
}

__global__ void __launch_bounds__(256) k_cell_h3_exact(CellArgs a, int all_rows) {
    unsigned long long total = all_rows ? (unsigned long long)a.n : min(*a.amb_count, a.amb_cap);
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    for (unsigned long long t = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
        int64_t i = all_rows ? (int64_t)t : (int64_t)a.amb_queue[t];
        if (!cell_row_present(a, i)) continue;
        // queued rows: k_cell_h3's rare rows take the full fast path first (face search, glibc sincos)
        bool amb = true;
        uint64_t cell = all_rows ? 0 : h3::h3_fast(a.y[i], a.x[i], a.res, &amb);
        if (amb) cell = h3::h3_exact(h3::to_radians(a.y[i], a.jdk), h3::to_radians(a.x[i], a.jdk), a.res);
        a.out[i] = (long long)cell;
    }
}

// Diagnostics (mosaic_diag_libm): the exact path's libm restatement (glibc_math.h) per row.
__global__ void __launch_bounds__(256) k_diag_libm(int fn, const double* a, const double* b, int64_t n, double* out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        double s, c, r = 0.0;
        switch (fn) {
            case 0: glibc::sincos(a[i], &s, &c); r = s; break;
            case 1: glibc::sincos(a[i], &s, &c); r = c; break;
            case 2: r = glibc::tan(a[i]); break;
            case 3: r = glibc::acos(a[i]); break;
            default: r = glibc::atan2(a[i], b[i]); break;
        }
        out[i] = r;
    }
}

__global__ void __launch_bounds__(256) k_cell_bng(CellArgs a) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    bool nan_seen = false;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
        bool v = cell_row_present(a, i);
        if (a.out_valid) a.out_valid[i] = v;
        int64_t cell = 0;
        if (v && !bng::point_to_index(a.x[i], a.y[i], a.res, &cell)) nan_seen = true;
        a.out[i] = v ? cell : 0;
    }
    if (nan_seen) atomicOr(a.flags, 1u);
}

// ---- point geometry column -> coordinates (grid_pointascellid over WKB / WKT / hex rows) ----
// One lane per row; rows are [offsets[i], offsets[i+1]) of the value buffer (Arrow binary / utf8
// layout, 32- or 64-bit offsets).  Status per row: 0 null, 1 decoded, 2 row path (point_decode.h).
struct DecodeArgs {
    const void* offsets;
    int off64;
    const uint8_t* data;
    const uint8_t* valid;
    int64_t n;
    int format;
    double* x;
    double* y;
    uint8_t* status;
    unsigned long long* n_rowpath;
};

// Each wave takes 64 consecutive rows.  Their value bytes -- one contiguous span -- are copied
// to the wave's LDS slice with coalesced 16-byte loads, and every lane parses its row from LDS
// (ds_read_u8 at LDS latency instead of a chain of dependent global byte loads).  A wave whose
// span exceeds the slice parses from global memory.  The copy reads the 16-byte aligned granules
// around the span: no page is touched that does not hold a byte of the span.
static const int kDecodeWaveBytes = 4096;

__device__ __forceinline__ int64_t decode_offset(const DecodeArgs& a, int64_t i) {
    return a.off64 ? ((const int64_t*)a.offsets)[i] : (int64_t)((const int32_t*)a.offsets)[i];
}

__global__ void __launch_bounds__(256) k_decode_points(DecodeArgs a) {
    __shared__ uint4 stage[4][kDecodeWaveBytes / 16];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    unsigned int rowpath = 0;
    for (int64_t w0 = (int64_t)blockIdx.x * blockDim.x + wave * 64; w0 < a.n; w0 += stride) {  // wave-uniform
        const int64_t i = w0 + lane;
        const bool act = i < a.n;
        const int64_t wend = w0 + 64 < a.n ? w0 + 64 : a.n;
        const int64_t sb = decode_offset(a, w0), se = decode_offset(a, wend);
        const uintptr_t gb = ((uintptr_t)(a.data + sb)) & ~(uintptr_t)15;
        const int64_t nchunk = se > sb ? (int64_t)(((uintptr_t)(a.data + se) - gb + 15) >> 4) : 0;
        const bool staged = se >= sb && nchunk <= kDecodeWaveBytes / 16;
        __builtin_amdgcn_wave_barrier();
        if (staged) {
            const uint4* g = (const uint4*)gb;
            for (int64_t k = lane; k < nchunk; k += 64) stage[wave][k] = g[k];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        double px = 0.0, py = 0.0;
        uint8_t st = 0;
        if (act && (!a.valid || a.valid[i])) {
            const int64_t b = decode_offset(a, i), e = decode_offset(a, i + 1);
            int rc = decode::kBadWkb;
            if (e >= b && b >= sb && e <= se) {
                if (staged) {
                    const uint8_t* row = (const uint8_t*)stage[wave] + ((uintptr_t)(a.data + b) - gb);
                    rc = decode::decode_row(a.format, row, e - b, &px, &py);
                } else {
                    rc = decode::decode_row(a.format, a.data + b, e - b, &px, &py);
                }
            }
            st = rc == decode::kOk ? 1 : 2;
            if (st == 2) {
                px = py = 0.0;
                rowpath++;
            }
        }
        if (act) {
            a.x[i] = px;
            a.y[i] = py;
            a.status[i] = st;
        }
    }
    if (rowpath) atomicAdd(a.n_rowpath, (unsigned long long)rowpath);
}

struct ContainsArgs {
    pip::GeomStore store;
    int64_t n_geoms;
    const int* geom_index;
    const double* px;
    const double* py;
    int64_t n;
    uint8_t* out;
};

__global__ void __launch_bounds__(256) k_st_contains(ContainsArgs a) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
        int g = a.geom_index[i];
        a.out[i] = (g >= 0 && g < a.n_geoms) ? (uint8_t)pip::contains(a.store, (uint32_t)g, a.px[i], a.py[i]) : 0;
    }
}

// ------------------------------------------------------------------------------------------------
// host side
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    int reserve(size_t n) {
        if (n <= bytes) return MOSAIC_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        if (hipMalloc(&p, n) != hipSuccess) return fail(MOSAIC_E_NOMEM, "hipMalloc(" + std::to_string(n) + ") failed");
        bytes = n;
        return MOSAIC_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

// Pinned host staging for the table build's host <-> device copies (h2d / d2h below).  A copy
// from or to pageable memory of a megabyte or more makes the HIP runtime pin that memory (a
// user-pointer registration with the kernel driver); when the range is later invalidated -- the
// vector freed, its pages moved or collapsed into a huge page -- the driver evicts every queue of
// the process, restores them tens of ms later, and whatever kernel was running stretches by that
// much.  Measured: the raster classification kernels' active cycles identical in every build
// (GRBM_GUI_ACTIVE, profiles/r05_build_var_pmc/), their wall time 6 ms in a process's first build
// and 32-42 ms in later ones, the 5 MB k_raster_sub copy 3 -> 30 ms.  Two 8 MB buffers allocated
// once per thread state, used in turn (an event per buffer), so no build copy touches pageable
// memory on the device side.
struct HostStage {
    static const size_t kBytes = (size_t)8 << 20;
    void* p[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool busy[2] = {false, false};
    int next = 0;  // the buffer the next chunk takes
    int ensure() {
        if (p[0]) return MOSAIC_OK;
        for (int k = 0; k < 2; k++) {
            if (hipHostMalloc(&p[k], kBytes, hipHostMallocDefault) != hipSuccess) {
                p[k] = nullptr;
                release();
                return fail(MOSAIC_E_NOMEM, "hipHostMalloc(staging) failed");
            }
            if (hipEventCreateWithFlags(&ev[k], hipEventDisableTiming) != hipSuccess) {
                ev[k] = nullptr;
                release();
                return fail(MOSAIC_E_HIP, "hipEventCreate(staging) failed");
            }
        }
        return MOSAIC_OK;
    }
    // wait until buffer k's last copy has finished
    int wait(int k) {
        if (busy[k]) {
            busy[k] = false;
            if (hipEventSynchronize(ev[k]) != hipSuccess) return fail(MOSAIC_E_HIP, "staging event");
        }
        return MOSAIC_OK;
    }
    void release() {
        for (int k = 0; k < 2; k++) {
            if (busy[k] && ev[k]) (void)hipEventSynchronize(ev[k]);
            busy[k] = false;
            if (ev[k]) (void)hipEventDestroy(ev[k]);
            if (p[k]) (void)hipHostFree(p[k]);
            ev[k] = nullptr;
            p[k] = nullptr;
        }
    }
};

// Scope guards of entry points: staged buffers and timing events are released
// on every return path (errors after allocation included)
struct DevBufGuard {
    std::vector<DevBuf*> bufs;
    ~DevBufGuard() {
        for (DevBuf* b : bufs) b->release();
    }
};
struct EventGuard {
    hipEvent_t e[2] = {nullptr, nullptr};
    ~EventGuard() {
        for (hipEvent_t x : e)
            if (x) (void)hipEventDestroy(x);
    }
};

// Options of a context (mosaic_set_option).  Every call copies them once at entry, so a call runs
// with one consistent set even while another thread changes them.
struct Options {
    int jdk = 8;
    int async = 0;
    int block = 256;
    int blocks_per_cu = 8;
    int raster = 16;          // ray-parity raster cells per side of a border chip (chip tables built later)
    int raster_adaptive = 1;  // fewer raster cells for rings with few segments
    int raster_min_segments = 0;  // rings with fewer segments get no chip raster (direct segment test)
    int lane_edges = 0;       // raster cell lists up to this long are evaluated by the owning lane
    int tiles = 1;            // build / use the H3 tile directory (tiles.h)
    int point_raster = 1;     // build / use the point raster over the tile directory (tiles.h)
    int raster_sub = 64;      // point raster: sub-blocks per tile side (a power of two)
    int raster_cell = 16;     // point raster: leaf cells per sub-block side (a power of two)
    int raster_quad = 1;      // point raster: LDS quad level
    int raster_lines = 1;     // point raster: line records for single-edge sub-blocks
    int raster_tb_lds = 1;    // tile bases in the stream kernels' LDS: 1 up to 1/3 of it, 2 only when small (1/16), 0 never
    int raster_leaf_lines = 1;  // point raster: line records for single-edge leaf cells (leaf lines; default since round 6)
    int leaf_join = 1;        // k_join_leaf answers the mixed queue's leaf-line rows before k_join_mixed
    int leaf_blocks_per_cu = 2;  // k_join_leaf grid
    int exact_defer = 0;      // stream joins: uncertified rows to k_join_h3_exact after k_join_mixed
    int raster_build = 1;     // point raster classification: 1 on the GPU (k_raster_*), 0 on host threads
    int raster_quad_records = 1;  // point raster: LDS quad records beside the quad level
    int stream_block = 1024;  // k_join_stream workgroup size (a multiple of 64, <= 1024)
    int bng_cpt = 1;          // k_join_stream_bng_cpt (rows needing gathers compacted) where it applies
    int stream_pipe = 2;      // 1: k_join_stream_pipe (software-pipelined), 2: k_join_stream_cpt (+ compacted gathers)
    int bng_lds = 1;          // BNG dense table: LDS cell level for k_join_stream_bng (chip tables built later)
    int bng_cell = 32;        // BNG dense table: sub-cells per border cell side (a power of two)
    int bng_group_lines = 1;  // BNG levels carry a line code where one line record decides a whole group
    int bng_wedges = 1;       // BNG tables: wedge records for sub-cells split at a chip vertex
    int cell_blocks_per_cu = 256;  // k_cell_h3 grid: n_cu x this, grid-strided (0 = one lane per group of kCellRows rows)
    int mixed_blocks_per_cu = 16;  // k_join_mixed(_bng) grid (16 since round 6: BNG mixed 0.68 -> 0.59 ms at C5, H3 unchanged; gpurun_out/r06bm2)
    int mixed_rows = 1;  // k_join_mixed rows per lane (1 since round 6: 0.278 -> 0.235 ms at C2 on the reference's chips, gpurun_out/r06mr2)
    // host-resident coordinates (mosaic_pip_join_count): chunks of host_chunk rows, the next chunk's
    // copy on copy_stream overlapping the current chunk's join (0: stage the whole batch first)
    int64_t host_chunk = (int64_t)1 << 25;
    int timing = 0;           // HIP events bracket each fused join kernel on the calling thread's stream
    // a calling thread keeps its scratch (queues, staging) between calls up to this many bytes; above
    // it the scratch is freed when the call returns (0: always kept, the default)
    int64_t scratch_limit = 0;
    // the binned join (join_binned.hip) for tile-directory tables without a usable point raster
    // (border-chip-heavy chip sets): points sorted by tile before the chip loop; rows per sort chunk
    int bin_points = 1;
    int64_t bin_min_rows = (int64_t)1 << 18;
    int64_t bin_chunk = (int64_t)1 << 28;
    // per-tile chip images in LDS for the binned join: 0 off, 1 for tables without a point raster
    // (built with the table; joins use them when present), 2 built for every tile-directory table
    int tile_images = 1;
    // exact-H3 queue capacity in rows (0: the default, max(n / 8, 2^20) capped at n); a small value
    // exercises the overflow -> rerun path
    int64_t exact_cap = 0;
    // k_bin_cover's look-back poll limit (< 0: the uncompacted fallback at once, for its test)
    int bin_spin_cap = 1 << 20;
};

// Execution state of one calling thread on one context: its HIP stream (created on first use, or
// set with mosaic_set_stream), its scratch buffers, counters, deferred errors and timing events.
// Threads never share one, so concurrent calls on a context do not touch each other's scratch
// ("Concurrent callers are multiplexed onto per-thread HIP streams").
struct ThreadCtx : Options {
    int device = 0;
    int n_cu = 256;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    const char* last_kernel = "";      // the dominant kernel of the last join call (mosaic_last_kernel)
    double last_tess_classify_ms = 0;  // classification kernel (k_bng_tess_classify / k_tess_classify_poly) of the
                                       // last mosaic_tessellate_gpu; 0 when it had no candidates
    DevBuf amb_queue, mix_queue, mix_queue2, scalars, stage_x, stage_y, stage_v, stage_out, stage_out2, stage_idx;
    DevBuf geo_off, geo_data, dec_x, dec_y, dec_status;  // point geometry decode
    DevBuf ov[8];  // st_intersection_aggregate's cell overlay (run_unit_overlay)
    HostStage hstage;  // pinned staging of the table build's copies (h2d / d2h)
    DevBuf rbuild[14];  // the raster classification's device scratch, kept between builds (raster_classify_gpu)
    hipStream_t copy_stream = nullptr;
    DevBuf hx[2], hy[2], hcounts;
    binned::Scratch bins;  // the binned join's keys, sorted points and sort temp
    int64_t stats[3] = {0, 0, 0};
    int64_t binned_rows = 0;  // rows the last join's binned path sorted (mosaic_last_binned_rows)
    unsigned int deferred_flags = 0;
    uint64_t last_qcap = 0;  // the exact-H3 queue capacity of the last join (sync_impl's overflow test)
    std::vector<hipEvent_t> ev_start, ev_stop;
    size_t ev_used = 0;
    // the scratch buffers sized by the calls (not `scalars`, which every call needs)
    std::vector<DevBuf*> scratch() {
        return {&amb_queue, &mix_queue, &mix_queue2, &stage_x, &stage_y, &stage_v, &stage_out, &stage_out2, &stage_idx, &geo_off,
                &geo_data, &dec_x, &dec_y, &dec_status, &hx[0], &hx[1], &hy[0], &hy[1], &hcounts,
                &ov[0], &ov[1], &ov[2], &ov[3], &ov[4], &ov[5], &ov[6], &ov[7], &rbuild[0], &rbuild[1], &rbuild[2],
                &rbuild[3], &rbuild[4], &rbuild[5], &rbuild[6], &rbuild[7], &rbuild[8], &rbuild[9], &rbuild[10],
                &rbuild[11], &rbuild[12], &rbuild[13]};
    }
    size_t held() {
        size_t n = 0;
        for (DevBuf* b : scratch()) n += b->bytes;
        return n + bins.held();
    }
    // free the scratch once the thread's queued work is done (scratch_limit)
    void trim() {
        (void)hipSetDevice(device);
        if (stream) (void)hipStreamSynchronize(stream);
        if (copy_stream) (void)hipStreamSynchronize(copy_stream);
        for (DevBuf* b : scratch()) b->release();
        bins.release();
    }
    void release() {
        (void)hipSetDevice(device);
        if (stream) (void)hipStreamSynchronize(stream);
        if (copy_stream) (void)hipStreamSynchronize(copy_stream);
        for (DevBuf* b : scratch()) b->release();
        bins.release();
        scalars.release();
        hstage.release();
        if (copy_stream) (void)hipStreamDestroy(copy_stream);
        for (size_t i = 0; i < ev_start.size(); i++) {
            (void)hipEventDestroy(ev_start[i]);
            (void)hipEventDestroy(ev_stop[i]);
        }
        if (own_stream && stream) (void)hipStreamDestroy(stream);
    }
};

// The ABI handle: a device, the shared options and the per-thread execution states.  Chip tables
// are immutable after mosaic_chip_table_create and may be joined from any number of threads.
struct mosaic_ctx {
    int device = 0;
    int n_cu = 256;
    uint64_t serial = 0;  // unique per context for the process's lifetime (never reused, unlike pointers)
    std::mutex mu;
    Options opt;
    // keyed by the thread's serial (this_thread_serial), never by pthread / std::thread ids, which
    // the runtime reuses: a new thread must not inherit a dead thread's state (its stream)
    std::unordered_map<uint64_t, std::unique_ptr<ThreadCtx>> threads;
};

// join scalars: [0] exact-queue rows, [1] pairs, [2] contains tests, [3] flags, [4] mixed-queue rows,
// [5] exact rows summed over the binned join's chunks, [6] a binned chunk overflowed the exact queue
static const int kScalars = 8;  // [7]: k_join_leaf's second queue count
// the join's counts and scalars zeroed by one launch (two hipMemsetAsync calls of odd sizes took four
// fill kernels, ~20 us per call on the stream)
__global__ void __launch_bounds__(256) k_zero_join(unsigned long long* counts, int64_t n_counts, unsigned long long* scalars) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_counts + kScalars; k += (int64_t)gridDim.x * blockDim.x) {
        if (k < n_counts) counts[k] = 0ull;
        else scalars[k - n_counts] = 0ull;
    }
}

// After a binned chunk's exact pass: its queue rows are added to scalars[5], an overflow is noted in
// scalars[6], and the queue starts over for the next chunk (whose sorted positions reuse the buffers).
__global__ void k_amb_roll(unsigned long long* sc, unsigned long long cap) {
    const unsigned long long q = sc[0];
    sc[5] += q;
    if (q > cap) sc[6] = 1;
    sc[0] = 0;
}
// After the last binned chunk: scalars[0] holds the rows of all chunks, or cap + 1 when one chunk
// overflowed, so an async caller's sync (mosaic_sync, the host-chunked join) sees the overflow.
__global__ void k_amb_final(unsigned long long* sc, unsigned long long cap) { sc[0] = sc[6] ? cap + 1 : sc[5]; }

// Lifetime of per-thread states.  A thread's state on a context is freed by mosaic_thread_release,
// by mosaic_destroy, or when the thread exits (ThreadExit below) -- so an executor whose worker pool
// retires threads does not accumulate streams and scratch.  Live contexts are registered by serial;
// lock order: g_live_mu, then ctx->mu.
static std::mutex g_live_mu;
static std::unordered_map<mosaic_ctx*, uint64_t> g_live;
static std::atomic<uint64_t> g_serial{1};

static uint64_t this_thread_serial() {
    static thread_local uint64_t id = g_serial.fetch_add(1);
    return id;
}

struct ThreadExit {
    std::vector<std::pair<mosaic_ctx*, uint64_t>> ctxs;  // contexts this thread entered
    ~ThreadExit() {
        // the process's main thread exits with the process: its states go with mosaic_destroy or the
        // process, never from a thread_local destructor racing the HIP runtime's own teardown
        if ((pid_t)syscall(SYS_gettid) == getpid()) return;
        const uint64_t me = this_thread_serial();
        std::lock_guard<std::mutex> live(g_live_mu);
        for (auto& e : ctxs) {
            auto it = g_live.find(e.first);
            if (it == g_live.end() || it->second != e.second) continue;  // destroyed since
            std::unique_ptr<ThreadCtx> t;
            {
                std::lock_guard<std::mutex> lock(e.first->mu);
                auto f = e.first->threads.find(me);
                if (f == e.first->threads.end()) continue;
                t = std::move(f->second);
                e.first->threads.erase(f);
            }
            t->release();
        }
    }
};
static thread_local ThreadExit g_thread_exit;

// The calling thread's execution state, options refreshed from the context (created on first use).
static ThreadCtx* enter(mosaic_ctx* ctx) {
    if (!ctx) return nullptr;
    const uint64_t me = this_thread_serial();
    std::lock_guard<std::mutex> lock(ctx->mu);
    std::unique_ptr<ThreadCtx>& t = ctx->threads[me];
    if (!t) {
        std::unique_ptr<ThreadCtx> n(new ThreadCtx());
        n->device = ctx->device;
        n->n_cu = ctx->n_cu;
        if (hipSetDevice(ctx->device) != hipSuccess ||
            hipStreamCreateWithFlags(&n->stream, hipStreamNonBlocking) != hipSuccess) {
            fail(MOSAIC_E_HIP, "hipStreamCreate failed");
            ctx->threads.erase(me);
            return nullptr;
        }
        n->own_stream = true;
        if (n->scalars.reserve(kScalars * 8)) {
            n->release();
            ctx->threads.erase(me);
            return nullptr;
        }
        t = std::move(n);
        auto& v = g_thread_exit.ctxs;
        v.erase(std::remove_if(v.begin(), v.end(), [&](const std::pair<mosaic_ctx*, uint64_t>& e) {
                    return e.first == ctx;
                }), v.end());
        v.emplace_back(ctx, ctx->serial);
    }
    static_cast<Options&>(*t) = ctx->opt;
    return t.get();
}

// Frees the calling thread's scratch on the way out of an entry point when it holds more than the
// option scratch_limit (bytes; 0 keeps it).
struct ScratchTrim {
    ThreadCtx* c;
    ~ScratchTrim() {
        if (c && c->scratch_limit > 0 && (int64_t)c->held() > c->scratch_limit) c->trim();
    }
};
#define ENTER(CTX)                                                                 \
    ThreadCtx* c = enter(CTX);                                                     \
    if (!c) return (CTX) ? MOSAIC_E_HIP : fail(MOSAIC_E_ARG, "null context");      \
    ScratchTrim scratch_trim_{c};

static int timing_begin(ThreadCtx* c, hipEvent_t* stop_out) {
    *stop_out = nullptr;
    if (!c->timing) return MOSAIC_OK;
    if (c->ev_used == c->ev_start.size()) {
        if (c->ev_used >= 4096) return MOSAIC_OK;  // bounded; extra calls are not timed
        hipEvent_t a, b;
        HIP_TRY(hipEventCreate(&a));
        HIP_TRY(hipEventCreate(&b));
        c->ev_start.push_back(a);
        c->ev_stop.push_back(b);
    }
    HIP_TRY(hipEventRecord(c->ev_start[c->ev_used], c->stream));
    *stop_out = c->ev_stop[c->ev_used];
    c->ev_used++;
    return MOSAIC_OK;
}

static int h2d(ThreadCtx* c, void* dst, const void* src, size_t n);

struct GeomStoreDev {
    DevBuf verts, ring_start, ring_bbox, part_ring, geom_part, geom_bbox;
    pip::GeomStore view() const {
        pip::GeomStore s;
        s.verts = (const pip::Vec2*)verts.p;
        s.ring_start = (const uint32_t*)ring_start.p;
        s.ring_bbox = (const pip::Box*)ring_bbox.p;
        s.part_ring = (const uint32_t*)part_ring.p;
        s.geom_part = (const uint32_t*)geom_part.p;
        s.geom_bbox = (const pip::Box*)geom_bbox.p;
        return s;
    }
    int upload(const GeomBuilder& b, ThreadCtx* c, size_t* total) {
        auto up = [&](DevBuf& d, const void* src, size_t bytes) -> int {
            int rc = d.reserve(std::max<size_t>(bytes, 16));
            if (rc) return rc;
            if ((rc = h2d(c, d.p, src, bytes))) return rc;
            *total += bytes;
            return MOSAIC_OK;
        };
        int rc;
        if ((rc = up(verts, b.verts.data(), b.verts.size() * sizeof(pip::Vec2)))) return rc;
        if ((rc = up(ring_start, b.ring_start.data(), b.ring_start.size() * 4))) return rc;
        if ((rc = up(ring_bbox, b.ring_bbox.data(), b.ring_bbox.size() * sizeof(pip::Box)))) return rc;
        if ((rc = up(part_ring, b.part_ring.data(), b.part_ring.size() * 4))) return rc;
        if ((rc = up(geom_part, b.geom_part.data(), b.geom_part.size() * 4))) return rc;
        if ((rc = up(geom_bbox, b.geom_bbox.data(), b.geom_bbox.size() * sizeof(pip::Box)))) return rc;
        HIP_TRY(hipStreamSynchronize(c->stream));
        return MOSAIC_OK;
    }
    void release() {
        verts.release();
        ring_start.release();
        ring_bbox.release();
        part_ring.release();
        geom_part.release();
        geom_bbox.release();
    }
};

struct mosaic_chips {
    int grid = 0, res = 0, device = 0;
    int64_t n_chips = 0, n_cells = 0, n_border = 0, n_vertices = 0, n_rings = 0;
    int32_t n_polygons = 0;
    uint64_t capacity = 0;
    size_t device_bytes = 0;
    DevBuf table, meta, hdr, cells, rast_edges;
    int raster = 0;  // raster dims the table was built with (0: none)
    int64_t raster_cells = 0, raster_pure = 0, raster_records = 0;
    GeomStoreDev store;
    // H3 tile directory (tiles.h); tiles_ok == false: none
    bool tiles_ok = false;
    tiles::Grid tgrid{};
    DevBuf tile_idx, tile_rec, tile_ent;
    int64_t tile_stats[6] = {0, 0, 0, 0, 0, 0};  // nx, ny, records, entries, kFull tiles, rings
    bool bng_ok = false;  // BNG dense cell table (k_join_stream_bng)
    int32_t bng_e0 = 0, bng_n0 = 0, bng_ne = 0, bng_nn = 0, bng_div = 1, bng_C = 0;
    DevBuf bng_cells, bng_leaf, bng_lcell, bng_lvl;
    size_t bng_leaf_bytes = 0, bng_lvl_bytes = 0;  // bng_lvl: sub-block levels (tiles.h bng_level_code); 0: none
    bool bng_cpt_ok = false;  // levels built, or no border cell has a leaf block (k_join_stream_bng_cpt applies)
    int32_t bng_lwords = 0, bng_lsh = 0, bng_lnx = 0;  // LDS cell level (BngStreamArgs::lcell); 0 words: none
    int64_t bng_sub_stats[2] = {0, 0};                 // border-cell sub-cells: kMixed, line records
    int bng_wedges = 0;                                // leaf blocks carry wedge codes (tiles.h)
    bool raster_ok = false;                       // point raster (tiles.h)
    tiles::PointRaster praster{};
    bool stream_ok = false;  // k_join_stream can run on the raster (quad level with compact copies, clamp-safe edges)
    StreamArgs stream{};
    DevBuf rsub, rmid, rblocks, rquad, rqrec;  // rmid: per-tile leaf block bases; rqrec: quad records
    DevBuf rlbase, rllines;                    // leaf lines: per-tile first record, the records
    // per-tile chip images of the binned join (tile_images.h ImageSet); empty: none
    DevBuf img_words, img_off, img_rec, img_binmap;
    uint32_t img_max_words = 0;
    int64_t img_records = 0;  // images built (parts of tile records; tile_images.h)
    int64_t img_count = 0;    // image keys (with the parts that have no image)
    bool tb_lds_budget = true;  // the build's LDS budget left room for the tile bases (k_join_stream_*)
    int64_t raster_stats[7] = {0, 0, 0, 0, 0, 0, 0};  // S, C, pure sub-blocks, mixed sub-blocks, mixed cells,
                                                      // line sub-blocks, leaf lines
    // build cost (ms): chip table core (hash, geometry, chip rasters), tile directory, point-raster
    // classification (GPU or host), point-raster assembly; FNV-1a digest of the point raster
    double build_ms[4] = {0, 0, 0, 0};
    uint64_t raster_digest = 0;  // computed on first request (mosaic_chip_table_build_info), not in the build
    size_t raster_parts[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // bytes of sub, blocks, tile_base, quad, qrec masks, qrec
                                                        // codes, leaf-line bases, leaf lines
    void release_all() {
        for (DevBuf* b : {&table, &meta, &hdr, &cells, &rast_edges,
                          &tile_idx, &tile_rec, &tile_ent, &rsub, &rmid, &rblocks, &rquad, &rqrec, &rlbase, &rllines, &bng_cells, &bng_leaf, &bng_lcell, &bng_lvl,
                          &img_words, &img_off, &img_rec, &img_binmap})
            b->release();
        store.release();
    }
};

// pointer residency: returns true if p is device-accessible memory of the current device
static bool is_device_ptr(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

// Make `src` (n_bytes) available on the device: returns the pointer to use.
static int to_device(ThreadCtx* c, DevBuf& stage, const void* src, size_t n_bytes, const void** out) {
    if (!src) {
        *out = nullptr;
        return MOSAIC_OK;
    }
    if (is_device_ptr(src)) {
        *out = src;
        return MOSAIC_OK;
    }
    int rc = stage.reserve(std::max<size_t>(n_bytes, 16));
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(stage.p, src, n_bytes, hipMemcpyHostToDevice, c->stream));
    *out = stage.p;
    return MOSAIC_OK;
}

static int grid_size(ThreadCtx* c, int64_t n) {
    int64_t want = (n + c->block - 1) / c->block;
    int64_t cap = (int64_t)c->n_cu * c->blocks_per_cu;
    return (int)std::max<int64_t>(1, std::min(want, cap));
}

static int res_error(int grid, int res) {
    if (grid == MOSAIC_GRID_H3)
        return fail(MOSAIC_E_RES, "H3 resolution has to be between 0 and 15; found " + std::to_string(res));
    return fail(MOSAIC_E_RES, "BNG resolution not supported; found " + std::to_string(res));
}

static bool valid_res(int grid, int res) {
    if (grid == MOSAIC_GRID_H3) return res >= 0 && res <= 15;
    return bng::valid_resolution(res);
}

// scalars buffer layout (unsigned long long): [0] amb_count, [1] pair_count, [2] tests, [3] flags,
// [4] mixed-raster-cell queue length

// Large host arrays whose release (munmap of tens of MB) would sit on the build's critical path are
// freed on a detached thread instead.
template <class T>
static void defer_free(T&& obj) {
    T* p = new T(std::move(obj));
    std::thread([p]() { delete p; }).detach();
}

extern "C" {

int mosaic_tess_fail(int code, const char* msg) { return fail(code, msg); }

int mosaic_ctx_exec(mosaic_ctx* ctx, int* device, void** stream, int* jdk, int* n_cu) {
    ENTER(ctx);
    HIP_TRY(hipSetDevice(c->device));
    *device = c->device;
    *stream = (void*)c->stream;
    *jdk = c->jdk;
    *n_cu = c->n_cu;
    return MOSAIC_OK;
}

int mosaic_abi_version(void) { return MOSAIC_ABI_VERSION; }
const char* mosaic_last_error(void) { return g_last_error.c_str(); }

// Context entry pays the device's one-time costs so that the first table build and join do not: a
// 4 MB pageable upload (the HIP runtime's setup for megabyte-sized pageable copies, 5.5 ms on its
// first use in a process) and ~3 ms of work on every CU (the GPU leaves its idle clock state; the
// build's first kernels ran up to 5x slower on a fresh box without it).  Bounded: s_memrealtime
// runs at 100 MHz, and the loop stops after 2^22 reads whatever the clock says.
__global__ void __launch_bounds__(256) k_warm_up(unsigned long long ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned int spins = 0; spins < (1u << 22) && __builtin_amdgcn_s_memrealtime() - t0 < ticks; spins++) {
    }
}

// Host -> device through the pinned staging buffers, ordered on c->stream: `src` may be freed or
// reused as soon as this returns (its bytes are in a staging buffer or already copied).
static int h2d(ThreadCtx* c, void* dst, const void* src, size_t n) {
    if (!n) return MOSAIC_OK;
    HostStage& h = c->hstage;
    int e;
    if ((e = h.ensure())) return e;
    for (size_t off = 0; off < n; off += HostStage::kBytes) {
        const size_t m = std::min(HostStage::kBytes, n - off);
        const int k = h.next;
        h.next ^= 1;
        if ((e = h.wait(k))) return e;
        memcpy(h.p[k], (const char*)src + off, m);
        HIP_TRY(hipMemcpyAsync((char*)dst + off, h.p[k], m, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipEventRecord(h.ev[k], c->stream));
        h.busy[k] = true;
    }
    return MOSAIC_OK;
}

// Device -> host through the pinned staging buffers after the work queued on c->stream; returns
// when `dst` holds the bytes.  Chunk i + 1's copy runs while chunk i is copied out on the host.
static int d2h(ThreadCtx* c, void* dst, const void* src, size_t n) {
    if (!n) return MOSAIC_OK;
    HostStage& h = c->hstage;
    int e;
    if ((e = h.ensure())) return e;
    int pk = -1;
    size_t poff = 0, pm = 0;
    for (size_t off = 0;; off += HostStage::kBytes) {
        const bool more = off < n;
        int k = -1;
        size_t m = 0;
        if (more) {
            m = std::min(HostStage::kBytes, n - off);
            k = h.next;
            h.next ^= 1;
            if ((e = h.wait(k))) return e;
            HIP_TRY(hipMemcpyAsync(h.p[k], (const char*)src + off, m, hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(hipEventRecord(h.ev[k], c->stream));
            h.busy[k] = true;
        }
        if (pk >= 0) {
            if ((e = h.wait(pk))) return e;
            memcpy((char*)dst + poff, h.p[pk], pm);
        }
        if (!more) break;
        pk = k;
        poff = off;
        pm = m;
    }
    return MOSAIC_OK;
}

// On the creating thread's own stream (never the null stream: context creation must not wait for
// other contexts' or torch's queued work); MOSAIC_NO_WARMUP=1 in the environment skips it.
static void warm_up(ThreadCtx* t) {
    const char* off = getenv("MOSAIC_NO_WARMUP");
    if (off && off[0] == '1') return;
    const size_t bytes = (size_t)4 << 20;
    void* d = nullptr;
    if (hipMalloc(&d, bytes) != hipSuccess) return;
    std::vector<uint8_t> h(bytes, 0);
    (void)h2d(t, d, h.data(), bytes);  // (allocates the build's pinned staging)
    hipLaunchKernelGGL(k_warm_up, dim3((unsigned)std::max(1, t->n_cu * 4)), dim3(256), 0, t->stream, 300000ULL);
    (void)hipGetLastError();
    (void)hipStreamSynchronize(t->stream);
    (void)hipFree(d);
}

// Transparent huge pages off for the process (unless MOSAIC_THP=1): khugepaged collapsing pages of a
// range the GPU driver tracks evicts every queue of the process for tens of ms -- measured on the
// table build (build side: 21.6-23.4 ms raster classification without, 70-84 ms with
// huge pages; the first geometry upload 0.5 vs 12.5 ms).  Boxes whose kernel setting is "always"
// would collapse pages without any advice, so the process opts out once, at its first context.
static void thp_off_once() {
    static std::once_flag once;
    std::call_once(once, []() {
        const char* e = getenv("MOSAIC_THP");
        if (!(e && e[0] == '1')) (void)prctl(PR_SET_THP_DISABLE, 1, 0, 0, 0);
    });
}

int mosaic_init(int device, mosaic_ctx** out) {
    if (!out) return fail(MOSAIC_E_ARG, "out is null");
    // objects compiled against different revisions of the shared headers (a hand-linked A/B library)
    // would pass structs with shifted fields between translation units: refuse to run
    if (mosaic_layout_join_binned() != mosaic_layout_fingerprint() || mosaic_layout_join_stream() != mosaic_layout_fingerprint() ||
        mosaic_layout_tess_clip() != mosaic::tessll::layout_fingerprint())
        return fail(MOSAIC_E_ARG, "libmosaic_hip.so links objects built against different struct layouts (rebuild every object)");
    thp_off_once();
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return fail(MOSAIC_E_HIP, "no HIP device available");
    if (device < 0 || device >= count) return fail(MOSAIC_E_ARG, "device ordinal out of range");
    HIP_TRY(hipSetDevice(device));
    mosaic_ctx* c = new mosaic_ctx();
    c->device = device;
    c->serial = g_serial.fetch_add(1);
    {
        std::lock_guard<std::mutex> live(g_live_mu);
        g_live[c] = c->serial;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->n_cu = prop.multiProcessorCount;
    ThreadCtx* t = enter(c);
    if (!t) {  // the creating thread's state: fails early if the device cannot make a stream
        mosaic_destroy(c);
        return MOSAIC_E_HIP;
    }
    warm_up(t);
    *out = c;
    return MOSAIC_OK;
}

int mosaic_destroy(mosaic_ctx* ctx) {
    if (!ctx) return MOSAIC_OK;
    {
        std::lock_guard<std::mutex> live(g_live_mu);  // waits for an exiting thread's release
        g_live.erase(ctx);
    }
    {
        std::lock_guard<std::mutex> lock(ctx->mu);
        for (auto& kv : ctx->threads) kv.second->release();
        ctx->threads.clear();
    }
    delete ctx;
    return MOSAIC_OK;
}

int mosaic_thread_release(mosaic_ctx* ctx) {
    if (!ctx) return fail(MOSAIC_E_ARG, "null context");
    std::unique_ptr<ThreadCtx> t;
    {
        std::lock_guard<std::mutex> lock(ctx->mu);
        auto f = ctx->threads.find(this_thread_serial());
        if (f == ctx->threads.end()) return MOSAIC_OK;
        t = std::move(f->second);
        ctx->threads.erase(f);
    }
    t->release();
    auto& v = g_thread_exit.ctxs;
    v.erase(std::remove_if(v.begin(), v.end(), [&](const std::pair<mosaic_ctx*, uint64_t>& e) { return e.first == ctx; }),
            v.end());
    return MOSAIC_OK;
}

int mosaic_thread_count(mosaic_ctx* ctx, int64_t* n_threads, int64_t* scratch_bytes) {
    if (!ctx || !n_threads) return fail(MOSAIC_E_ARG, "null argument");
    std::lock_guard<std::mutex> lock(ctx->mu);
    *n_threads = (int64_t)ctx->threads.size();
    if (scratch_bytes) {
        int64_t b = 0;
        for (auto& kv : ctx->threads) b += (int64_t)kv.second->held();
        *scratch_bytes = b;
    }
    return MOSAIC_OK;
}

int mosaic_set_option(mosaic_ctx* ctx, const char* key, int64_t v) {
    if (!ctx || !key) return fail(MOSAIC_E_ARG, "null argument");
    std::string k(key);
    Options o;
    {
        std::lock_guard<std::mutex> lock(ctx->mu);
        o = ctx->opt;
    }
    auto pow2 = [](int64_t x) { return x > 0 && (x & (x - 1)) == 0; };
    if (k == "jdk") {
        if (v < 8) return fail(MOSAIC_E_ARG, "jdk must be >= 8");
        o.jdk = (int)v;
    } else if (k == "async") {
        o.async = v ? 1 : 0;
    } else if (k == "block") {
        if (v < 64 || v > 256 || v % 64) return fail(MOSAIC_E_ARG, "block must be 64, 128, 192 or 256");
        o.block = (int)v;
    } else if (k == "blocks_per_cu") {
        if (v < 1 || v > 64) return fail(MOSAIC_E_ARG, "blocks_per_cu must be in [1, 64]");
        o.blocks_per_cu = (int)v;
    } else if (k == "cell_blocks_per_cu") {
        if (v < 0 || v > 4096) return fail(MOSAIC_E_ARG, "cell_blocks_per_cu must be in [0, 4096]");
        o.cell_blocks_per_cu = (int)v;
    } else if (k == "raster") {
        if (v < 1 || v > 64) return fail(MOSAIC_E_ARG, "raster must be in [1, 64]");
        o.raster = (int)v;
    } else if (k == "lane_edges") {
        if (v < 0 || v > 32) return fail(MOSAIC_E_ARG, "lane_edges must be in [0, 32]");
        o.lane_edges = (int)v;
    } else if (k == "tiles") {
        o.tiles = v ? 1 : 0;
    } else if (k == "point_raster") {
        o.point_raster = v ? 1 : 0;
    } else if (k == "raster_sub") {
        if (v > 64 || !pow2(v)) return fail(MOSAIC_E_ARG, "raster_sub must be a power of two in [1, 64]");
        o.raster_sub = (int)v;
    } else if (k == "raster_cell") {
        if (v > 32 || !pow2(v)) return fail(MOSAIC_E_ARG, "raster_cell must be a power of two in [1, 32]");
        o.raster_cell = (int)v;
    } else if (k == "mixed_rows") {
        if (v != 1 && v != 2 && v != 4) return fail(MOSAIC_E_ARG, "mixed_rows must be 1, 2 or 4");
        o.mixed_rows = (int)v;
    } else if (k == "mixed_blocks_per_cu") {
        if (v < 1 || v > 64) return fail(MOSAIC_E_ARG, "mixed_blocks_per_cu must be in [1, 64]");
        o.mixed_blocks_per_cu = (int)v;
    } else if (k == "raster_quad") {
        if (v < 0 || v > tiles::kQuadLimit)
            return fail(MOSAIC_E_ARG, "raster_quad must be 0 (off), 1 (default size) or an entry budget <= " +
                                          std::to_string(tiles::kQuadLimit));
        o.raster_quad = (int)v;
    } else if (k == "raster_adaptive") {
        o.raster_adaptive = v ? 1 : 0;
    } else if (k == "raster_min_segments") {
        if (v < 0 || v > 1000000) return fail(MOSAIC_E_ARG, "raster_min_segments must be in [0, 1e6]");
        o.raster_min_segments = (int)v;
    } else if (k == "raster_lines") {
        o.raster_lines = v ? 1 : 0;
    } else if (k == "raster_tb_lds") {
        if (v < 0 || v > 2) return fail(MOSAIC_E_ARG, "raster_tb_lds must be 0, 1 or 2");
        o.raster_tb_lds = (int)v;
    } else if (k == "raster_leaf_lines") {
        o.raster_leaf_lines = v ? 1 : 0;
    } else if (k == "leaf_join") {
        o.leaf_join = v ? 1 : 0;
    } else if (k == "exact_defer") {
        o.exact_defer = v ? 1 : 0;
    } else if (k == "leaf_blocks_per_cu") {
        if (v < 1 || v > 64) return fail(MOSAIC_E_ARG, "leaf_blocks_per_cu must be in [1, 64]");
        o.leaf_blocks_per_cu = (int)v;
    } else if (k == "raster_quad_records") {
        o.raster_quad_records = v ? 1 : 0;
    } else if (k == "raster_build") {
        if (v < 0 || v > 2) return fail(MOSAIC_E_ARG, "raster_build must be 0 (host), 1 (GPU) or 2 (GPU, lane-per-sub-block lines)");
        o.raster_build = (int)v;
    } else if (k == "host_chunk") {
        if (v < 0) return fail(MOSAIC_E_ARG, "host_chunk must be >= 0");
        o.host_chunk = v;
    } else if (k == "stream_block") {
        if (v < 64 || v > 1024 || v % 64) return fail(MOSAIC_E_ARG, "stream_block must be a multiple of 64 in [64, 1024]");
        o.stream_block = (int)v;
    } else if (k == "stream_pipe") {
        if (v < 0 || v > 2) return fail(MOSAIC_E_ARG, "stream_pipe must be 0, 1 or 2");
        o.stream_pipe = (int)v;
    } else if (k == "bng_cpt") {
        o.bng_cpt = v ? 1 : 0;
    } else if (k == "bng_lds") {
        o.bng_lds = v ? 1 : 0;
    } else if (k == "bng_cell") {
        if (v > 64 || !pow2(v)) return fail(MOSAIC_E_ARG, "bng_cell must be a power of two in [1, 64]");
        o.bng_cell = (int)v;
    } else if (k == "bng_group_lines") {
        o.bng_group_lines = v ? 1 : 0;
    } else if (k == "bng_wedges") {
        o.bng_wedges = v ? 1 : 0;
    } else if (k == "timing") {
        if (v < 0 || v > 2) return fail(MOSAIC_E_ARG, "timing must be 0, 1 or 2");
        o.timing = (int)v;
    } else if (k == "bin_points") {
        o.bin_points = v ? 1 : 0;
    } else if (k == "tile_images") {
        if (v < 0 || v > 2) return fail(MOSAIC_E_ARG, "tile_images must be 0, 1 or 2");
        o.tile_images = (int)v;
    } else if (k == "bin_min_rows") {
        if (v < 0) return fail(MOSAIC_E_ARG, "bin_min_rows must be >= 0");
        o.bin_min_rows = v;
    } else if (k == "bin_chunk") {
        if (v < 1024 || v > ((int64_t)1 << 30)) return fail(MOSAIC_E_ARG, "bin_chunk must be in [1024, 2^30]");
        o.bin_chunk = v;
    } else if (k == "scratch_limit") {
        if (v < 0) return fail(MOSAIC_E_ARG, "scratch_limit must be >= 0");
        o.scratch_limit = v;
    } else if (k == "bin_spin_cap") {
        o.bin_spin_cap = (int)std::max<int64_t>(-1, std::min<int64_t>(v, (int64_t)1 << 30));
    } else if (k == "exact_cap") {
        if (v < 0) return fail(MOSAIC_E_ARG, "exact_cap must be >= 0");
        o.exact_cap = v;
    } else {
        return fail(MOSAIC_E_ARG, "unknown option " + k);
    }
    {
        std::lock_guard<std::mutex> lock(ctx->mu);
        ctx->opt = o;
    }
    if (k == "timing") {  // the calling thread's timed-call list starts over
        ENTER(ctx);
        c->ev_used = 0;
    }
    return MOSAIC_OK;
}

int mosaic_get_stream(mosaic_ctx* ctx, void** s) {
    if (!ctx || !s) return fail(MOSAIC_E_ARG, "null argument");
    ENTER(ctx);
    *s = (void*)c->stream;
    return MOSAIC_OK;
}

int mosaic_set_stream(mosaic_ctx* ctx, void* s) {
    ENTER(ctx);
    if (c->own_stream) {
        (void)hipStreamSynchronize(c->stream);
        (void)hipStreamDestroy(c->stream);
    }
    c->stream = (hipStream_t)s;
    c->own_stream = false;
    return MOSAIC_OK;
}

int mosaic_stream_wait_event(mosaic_ctx* ctx, void* ev) {
    ENTER(ctx);
    if (!ev) return fail(MOSAIC_E_ARG, "null event");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamWaitEvent(c->stream, (hipEvent_t)ev, 0));
    return MOSAIC_OK;
}

static int sync_impl(ThreadCtx* c);
int mosaic_sync(mosaic_ctx* ctx) {
    ENTER(ctx);
    return sync_impl(c);
}

static int sync_impl(ThreadCtx* c) {
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    unsigned long long s[kScalars];
    HIP_TRY(hipMemcpy(s, c->scalars.p, sizeof s, hipMemcpyDeviceToHost));
    unsigned int flags = c->deferred_flags | (unsigned int)s[3];
    c->deferred_flags = 0;
    if (flags & 1u) return fail(MOSAIC_E_NAN, "NaN coordinates are not supported.");
    if ((flags & 2u) || s[0] > c->last_qcap)
        return fail(MOSAIC_E_CAPACITY, "exact-path queue overflowed in an async call; rerun synchronously");
    return MOSAIC_OK;
}

int mosaic_kernel_times(mosaic_ctx* ctx, double* out_ms, int64_t cap, int64_t* n_out) {
    if (!ctx || !n_out || (cap > 0 && !out_ms)) return fail(MOSAIC_E_ARG, "null argument");
    ENTER(ctx);
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    int64_t n = (int64_t)c->ev_used;
    for (int64_t i = 0; i < n && i < cap; i++) {
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, c->ev_start[i], c->ev_stop[i]));
        out_ms[i] = ms;
    }
    *n_out = n;
    c->ev_used = 0;
    return MOSAIC_OK;
}

const char* mosaic_last_kernel(mosaic_ctx* ctx) {
    ThreadCtx* c = ctx ? enter(ctx) : nullptr;
    return c ? c->last_kernel : "";
}

int mosaic_last_binned_rows(mosaic_ctx* ctx, int64_t* out) {
    if (!ctx || !out) return fail(MOSAIC_E_ARG, "null argument");
    ENTER(ctx);
    *out = c->binned_rows;
    return MOSAIC_OK;
}

int mosaic_last_stats(mosaic_ctx* ctx, int64_t* out3) {
    if (!ctx || !out3) return fail(MOSAIC_E_ARG, "null argument");
    ENTER(ctx);
    for (int i = 0; i < 3; i++) out3[i] = c->stats[i];
    return MOSAIC_OK;
}

int mosaic_resolution(int grid, int res, int* out) {
    if (!out) return fail(MOSAIC_E_ARG, "out is null");
    if (grid != MOSAIC_GRID_H3 && grid != MOSAIC_GRID_BNG) return fail(MOSAIC_E_ARG, "unknown grid");
    if (!valid_res(grid, res)) return res_error(grid, res);
    *out = res;
    return MOSAIC_OK;
}

int mosaic_resolution_str(int grid, const char* s, int* out) {
    if (!out || !s) return fail(MOSAIC_E_ARG, "null argument");
    std::string v(s);
    if (grid == MOSAIC_GRID_H3) {
        // H3IndexSystem.getResolution: s.toInt (NumberFormatException propagates in the reference)
        char* end = nullptr;
        long r = strtol(s, &end, 10);
        if (v.empty() || *end) return fail(MOSAIC_E_ARG, "For input string: \"" + v + "\"");
        return mosaic_resolution(grid, (int)r, out);
    }
    if (grid == MOSAIC_GRID_BNG) {
        // BNGIndexSystem.resolutionMap (BNGIndexSystem.scala:43-57); an Int-typed value is checked
        // against `resolutions` first, a String only against the map.
        static const char* names[] = {"500km", "100km", "50km", "10km", "5km", "1km",
                                      "500m",  "100m",  "50m",  "10m",  "5m",  "1m"};
        static const int vals[] = {-1, 1, -2, 2, -3, 3, -4, 4, -5, 5, -6, 6};
        for (int i = 0; i < 12; i++)
            if (v == names[i]) {
                *out = vals[i];
                return MOSAIC_OK;
            }
        return fail(MOSAIC_E_RES, "BNG resolution not supported; found " + v);
    }
    return fail(MOSAIC_E_ARG, "unknown grid");
}

// status (device, nullable): rows of a decoded geometry column, present iff status == 1
static int point_to_cell_impl(ThreadCtx* c, int grid, int res, const double* x, const double* y,
                              const uint8_t* valid, const uint8_t* status, int64_t n, int64_t* out_cell,
                              uint8_t* out_valid) {
    int rc;
    const void *dx, *dy, *dv;
    if ((rc = to_device(c, c->stage_x, x, n * 8, &dx))) return rc;
    if ((rc = to_device(c, c->stage_y, y, n * 8, &dy))) return rc;
    if ((rc = to_device(c, c->stage_v, valid, n, &dv))) return rc;
    bool dev_out = is_device_ptr(out_cell);
    bool dev_vout = !out_valid || is_device_ptr(out_valid);
    if (!dev_out && (rc = c->stage_out.reserve(n * 8))) return rc;
    if (out_valid && !dev_vout && (rc = c->stage_out2.reserve(n))) return rc;
    long long* dout = dev_out ? (long long*)out_cell : (long long*)c->stage_out.p;
    uint8_t* dvout = out_valid ? (dev_vout ? out_valid : (uint8_t*)c->stage_out2.p) : nullptr;
    uint64_t cap = (uint64_t)std::min<int64_t>(n, std::max<int64_t>(n / 8, 1 << 20));
    if ((rc = c->amb_queue.reserve(cap * 8))) return rc;
    HIP_TRY(hipMemsetAsync(c->scalars.p, 0, kScalars * 8, c->stream));
    unsigned long long* sc = (unsigned long long*)c->scalars.p;
    CellArgs a;
    a.x = (const double*)dx;
    a.y = (const double*)dy;
    a.valid = (const uint8_t*)dv;
    a.status = status;
    a.n = n;
    a.res = res;
    a.jdk = c->jdk;
    a.out = dout;
    a.out_valid = dvout;
    a.amb_queue = (unsigned long long*)c->amb_queue.p;
    a.amb_count = sc + 0;
    a.amb_cap = cap;
    a.flags = (unsigned int*)(sc + 3);
    a.vec = (((uintptr_t)dx | (uintptr_t)dy | (uintptr_t)dout) & 15) == 0;  // (every group of rows starts 16-byte aligned: kCellRows even)
    int g = grid_size(c, n);
    if (grid == MOSAIC_GRID_H3) {
        // k_cell_h3's grid: 256 blocks per CU by default -- at the common 8 (occupancy 7 at 66 VGPRs) it
        // ran 11.1 ms per 1e9 points, 9.3 ms at 128-1024, 9.6 ms with one lane per row pair
        // (gpurun_out/r06s, r06s2; profiles/r06_cell_grid_sweep.txt)
        const int64_t groups = (n + kCellRows - 1) / kCellRows, want = (groups + c->block - 1) / c->block;
        const int64_t gc = c->cell_blocks_per_cu ? std::min<int64_t>(want, (int64_t)c->n_cu * c->cell_blocks_per_cu) : want;
        hipLaunchKernelGGL(k_cell_h3, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(gc, 0x7fffffff))), dim3(c->block),
                           0, c->stream, a);
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_cell_h3_exact, dim3(grid_size(c, (int64_t)cap)), dim3(c->block), 0, c->stream, a, 0);
        HIP_TRY(hipGetLastError());
    } else {
        hipLaunchKernelGGL(k_cell_bng, dim3(g), dim3(c->block), 0, c->stream, a);
        HIP_TRY(hipGetLastError());
    }
    bool host_side = !dev_out || (out_valid && !dev_vout);
    if (c->async && !host_side) return MOSAIC_OK;
    HIP_TRY(hipStreamSynchronize(c->stream));
    unsigned long long s[kScalars];
    HIP_TRY(hipMemcpy(s, c->scalars.p, sizeof s, hipMemcpyDeviceToHost));
    if (grid == MOSAIC_GRID_H3 && s[0] > cap) {  // queue overflow: recompute every row exactly
        hipLaunchKernelGGL(k_cell_h3_exact, dim3(grid_size(c, n)), dim3(c->block), 0, c->stream, a, 1);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    c->stats[0] = (int64_t)s[0];
    c->stats[1] = 0;
    c->stats[2] = 0;
    if (s[3] & 1u) return fail(MOSAIC_E_NAN, "NaN coordinates are not supported.");
    if (!dev_out) HIP_TRY(hipMemcpy(out_cell, dout, n * 8, hipMemcpyDeviceToHost));
    if (out_valid && !dev_vout) HIP_TRY(hipMemcpy(out_valid, dvout, n, hipMemcpyDeviceToHost));
    return MOSAIC_OK;
}

int mosaic_point_to_cell(mosaic_ctx* ctx, int grid, int res, const double* x, const double* y, const uint8_t* valid,
                         int64_t n, int64_t* out_cell, uint8_t* out_valid) {
    ENTER(ctx);
    if (!c || (n > 0 && (!x || !y || !out_cell))) return fail(MOSAIC_E_ARG, "null argument");
    if (n < 0) return fail(MOSAIC_E_ARG, "negative n");
    if (grid != MOSAIC_GRID_H3 && grid != MOSAIC_GRID_BNG) return fail(MOSAIC_E_ARG, "unknown grid");
    if (!valid_res(grid, res)) return res_error(grid, res);
    if (n == 0) return MOSAIC_OK;
    HIP_TRY(hipSetDevice(c->device));
    return point_to_cell_impl(c, grid, res, x, y, valid, nullptr, n, out_cell, out_valid);
}

int mosaic_point_to_cell_exact(mosaic_ctx* ctx, int res, const double* x, const double* y, int64_t n,
                               int64_t* out_cell) {
    ENTER(ctx);
    if (!c || (n > 0 && (!x || !y || !out_cell))) return fail(MOSAIC_E_ARG, "null argument");
    if (n < 0) return fail(MOSAIC_E_ARG, "negative n");
    if (!valid_res(MOSAIC_GRID_H3, res)) return res_error(MOSAIC_GRID_H3, res);
    if (n == 0) return MOSAIC_OK;
    HIP_TRY(hipSetDevice(c->device));
    int rc;
    const void *dx, *dy;
    if ((rc = to_device(c, c->stage_x, x, n * 8, &dx))) return rc;
    if ((rc = to_device(c, c->stage_y, y, n * 8, &dy))) return rc;
    bool dev_out = is_device_ptr(out_cell);
    if (!dev_out && (rc = c->stage_out.reserve(n * 8))) return rc;
    CellArgs a{};
    a.x = (const double*)dx;
    a.y = (const double*)dy;
    a.n = n;
    a.res = res;
    a.jdk = c->jdk;
    a.out = dev_out ? (long long*)out_cell : (long long*)c->stage_out.p;
    hipLaunchKernelGGL(k_cell_h3_exact, dim3(grid_size(c, n)), dim3(c->block), 0, c->stream, a, 1);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (!dev_out) HIP_TRY(hipMemcpy(out_cell, a.out, n * 8, hipMemcpyDeviceToHost));
    return MOSAIC_OK;
}

int mosaic_diag_libm(mosaic_ctx* ctx, int fn, const double* a, const double* b, int64_t n, double* out) {
    ENTER(ctx);
    if (!c || fn < 0 || fn > 4 || (n > 0 && (!a || !out || (fn == 4 && !b)))) return fail(MOSAIC_E_ARG, "bad argument");
    if (n <= 0) return MOSAIC_OK;
    HIP_TRY(hipSetDevice(c->device));
    int rc;
    const void *da, *db = nullptr;
    if ((rc = to_device(c, c->stage_x, a, n * 8, &da))) return rc;
    if (fn == 4 && (rc = to_device(c, c->stage_y, b, n * 8, &db))) return rc;
    bool dev_out = is_device_ptr(out);
    if (!dev_out && (rc = c->stage_out.reserve(n * 8))) return rc;
    double* dout = dev_out ? out : (double*)c->stage_out.p;
    hipLaunchKernelGGL(k_diag_libm, dim3(grid_size(c, n)), dim3(c->block), 0, c->stream, fn, (const double*)da,
                       (const double*)db, n, dout);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (!dev_out) HIP_TRY(hipMemcpy(out, dout, n * 8, hipMemcpyDeviceToHost));
    return MOSAIC_OK;
}

// Decode a point geometry column into c->dec_x / dec_y / dec_status (device); *n_rowpath = rows
// left to the reference row path.  Synchronous.
static int decode_points(ThreadCtx* c, int format, const void* offsets, const uint8_t* data, const uint8_t* valid,
                         int64_t n, int64_t* n_rowpath) {
    const int fmt = format & 0xff;
    const bool off64 = !(format & MOSAIC_GEOM_OFFSETS32);
    if (fmt != MOSAIC_GEOM_WKB && fmt != MOSAIC_GEOM_WKT && fmt != MOSAIC_GEOM_HEX)
        return fail(MOSAIC_E_ARG, "unknown geometry format");
    if ((format & ~0x1ff) != 0) return fail(MOSAIC_E_ARG, "unknown geometry format flags");
    const size_t ob = off64 ? 8 : 4;
    int rc;
    const void *doff, *ddata = nullptr, *dv;
    // the value buffer spans [0, offsets[n]) (Arrow: offsets are relative to the buffer start)
    int64_t end = 0;
    if (is_device_ptr(offsets)) {
        int64_t e64 = 0;
        int32_t e32 = 0;
        HIP_TRY(hipMemcpy(off64 ? (void*)&e64 : (void*)&e32, (const char*)offsets + n * ob, ob, hipMemcpyDeviceToHost));
        end = off64 ? e64 : e32;
    } else {
        end = off64 ? ((const int64_t*)offsets)[n] : ((const int32_t*)offsets)[n];
    }
    if (end < 0) return fail(MOSAIC_E_ARG, "negative offsets");
    if (end > 0 && !data) return fail(MOSAIC_E_ARG, "null argument");
    if ((rc = to_device(c, c->geo_off, offsets, (size_t)(n + 1) * ob, &doff))) return rc;
    if (end > 0 && (rc = to_device(c, c->geo_data, data, (size_t)end, &ddata))) return rc;
    if ((rc = to_device(c, c->stage_v, valid, n, &dv))) return rc;
    if ((rc = c->dec_x.reserve(n * 8)) || (rc = c->dec_y.reserve(n * 8)) || (rc = c->dec_status.reserve(n))) return rc;
    HIP_TRY(hipMemsetAsync(c->scalars.p, 0, kScalars * 8, c->stream));
    DecodeArgs a;
    a.offsets = doff;
    a.off64 = off64 ? 1 : 0;
    a.data = (const uint8_t*)ddata;
    a.valid = (const uint8_t*)dv;
    a.n = n;
    a.format = fmt;
    a.x = (double*)c->dec_x.p;
    a.y = (double*)c->dec_y.p;
    a.status = (uint8_t*)c->dec_status.p;
    a.n_rowpath = (unsigned long long*)c->scalars.p + 4;
    hipLaunchKernelGGL(k_decode_points, dim3(std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, (int64_t)c->n_cu * 8))), dim3(256), 0, c->stream, a);
    HIP_TRY(hipGetLastError());
    unsigned long long r = 0;
    HIP_TRY(hipMemcpyAsync(&r, a.n_rowpath, 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (n_rowpath) *n_rowpath = (int64_t)r;
    return MOSAIC_OK;
}

static int copy_out(ThreadCtx* c, void* dst, const void* src, size_t bytes) {
    if (!dst || !bytes) return MOSAIC_OK;
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, is_device_ptr(dst) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MOSAIC_OK;
}

int mosaic_point_geom_decode(mosaic_ctx* ctx, int format, const void* offsets, const uint8_t* data, const uint8_t* valid,
                             int64_t n, double* x, double* y, uint8_t* row_status, int64_t* n_rowpath) {
    ENTER(ctx);
    if (!c || !offsets || (n > 0 && (!x || !y || !row_status))) return fail(MOSAIC_E_ARG, "null argument");
    if (n < 0) return fail(MOSAIC_E_ARG, "negative n");
    if (n_rowpath) *n_rowpath = 0;
    if (n == 0) return MOSAIC_OK;
    HIP_TRY(hipSetDevice(c->device));
    int rc;
    if ((rc = decode_points(c, format, offsets, data, valid, n, n_rowpath))) return rc;
    if ((rc = copy_out(c, x, c->dec_x.p, n * 8)) || (rc = copy_out(c, y, c->dec_y.p, n * 8)) ||
        (rc = copy_out(c, row_status, c->dec_status.p, n)))
        return rc;
    return MOSAIC_OK;
}

int mosaic_point_geom_to_cell(mosaic_ctx* ctx, int grid, int res, int format, const void* offsets, const uint8_t* data,
                              const uint8_t* valid, int64_t n, int64_t* out_cell, uint8_t* row_status,
                              int64_t* n_rowpath) {
    ENTER(ctx);
    if (!c || !offsets || (n > 0 && (!out_cell || !row_status))) return fail(MOSAIC_E_ARG, "null argument");
    if (n < 0) return fail(MOSAIC_E_ARG, "negative n");
    if (grid != MOSAIC_GRID_H3 && grid != MOSAIC_GRID_BNG) return fail(MOSAIC_E_ARG, "unknown grid");
    if (!valid_res(grid, res)) return res_error(grid, res);
    if (n_rowpath) *n_rowpath = 0;
    if (n == 0) return MOSAIC_OK;
    HIP_TRY(hipSetDevice(c->device));
    int rc;
    if ((rc = decode_points(c, format, offsets, data, valid, n, n_rowpath))) return rc;
    const int async = c->async;
    c->async = 0;
    rc = point_to_cell_impl(c, grid, res, (const double*)c->dec_x.p, (const double*)c->dec_y.p, nullptr,
                            (const uint8_t*)c->dec_status.p, n, out_cell, nullptr);
    c->async = async;
    if (rc) return rc;
    return copy_out(c, row_status, c->dec_status.p, n);
}

// element idx of an int32 array in host or device memory
static int read_i32(ThreadCtx* c, const int32_t* p, int64_t idx, int32_t* out) {
    if (is_device_ptr(p)) {
        HIP_TRY(hipMemcpy(out, p + idx, 4, hipMemcpyDeviceToHost));
    } else {
        *out = p[idx];
    }
    (void)c;
    return MOSAIC_OK;
}

// Decode a COORDS point column into c->dec_x / dec_y / dec_status (device).  Synchronous.
static int decode_coords(ThreadCtx* c, const int32_t* type_id, const int32_t* bnd, const int32_t* ring,
                         const int32_t* crd, const double* values, const uint8_t* valid, int64_t n, int64_t* n_rowpath) {
    if (!type_id || !bnd || !ring || !crd) return fail(MOSAIC_E_ARG, "null argument");
    int rc;
    int32_t nb = 0, nr = 0, nv = 0;
    if ((rc = read_i32(c, bnd, n, &nb))) return rc;
    if (nb < 0) return fail(MOSAIC_E_ARG, "negative offsets");
    if ((rc = read_i32(c, ring, nb, &nr))) return rc;
    if (nr < 0) return fail(MOSAIC_E_ARG, "negative offsets");
    if ((rc = read_i32(c, crd, nr, &nv))) return rc;
    if (nv < 0 || (nv > 0 && !values)) return fail(MOSAIC_E_ARG, "bad coordinate values");
    const void *dt, *db, *dr, *dc, *dvals = nullptr, *dv;
    if ((rc = to_device(c, c->stage_idx, type_id, (size_t)n * 4, &dt)) ||
        (rc = to_device(c, c->geo_off, bnd, (size_t)(n + 1) * 4, &db)) ||
        (rc = to_device(c, c->stage_out, ring, (size_t)(nb + 1) * 4, &dr)) ||
        (rc = to_device(c, c->stage_out2, crd, (size_t)(nr + 1) * 4, &dc)) ||
        (nv > 0 && (rc = to_device(c, c->geo_data, values, (size_t)nv * 8, &dvals))) ||
        (rc = to_device(c, c->stage_v, valid, (size_t)n, &dv)))
        return rc;
    if ((rc = c->dec_x.reserve(n * 8)) || (rc = c->dec_y.reserve(n * 8)) || (rc = c->dec_status.reserve(n))) return rc;
    HIP_TRY(hipMemsetAsync(c->scalars.p, 0, kScalars * 8, c->stream));
    CoordsArgs a;
    a.type_id = (const int32_t*)dt;
    a.bnd = (const int32_t*)db;
    a.ring = (const int32_t*)dr;
    a.crd = (const int32_t*)dc;
    a.values = (const double*)dvals;
    a.valid = (const uint8_t*)dv;
    a.n = n;
    a.n_bnd = (int64_t)nb + 1;
    a.n_ring = (int64_t)nr + 1;
    a.n_values = nv;
    a.x = (double*)c->dec_x.p;
    a.y = (double*)c->dec_y.p;
    a.status = (uint8_t*)c->dec_status.p;
    a.n_rowpath = (unsigned long long*)c->scalars.p + 4;
    hipLaunchKernelGGL(k_decode_coords, dim3(grid_size(c, n)), dim3(256), 0, c->stream, a);
    HIP_TRY(hipGetLastError());
    unsigned long long r = 0;
    HIP_TRY(hipMemcpyAsync(&r, a.n_rowpath, 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (n_rowpath) *n_rowpath = (int64_t)r;
    return MOSAIC_OK;
}

int mosaic_point_coords_decode(mosaic_ctx* ctx, const int32_t* type_id, const int32_t* boundary_offsets,
                               const int32_t* coord_offsets, const int32_t* value_offsets, const double* values,
                               const uint8_t* valid, int64_t n, double* x, double* y, uint8_t* row_status,
                               int64_t* n_rowpath) {
    ENTER(ctx);
    if (n < 0) return fail(MOSAIC_E_ARG, "negative n");
    if (n > 0 && (!x || !y || !row_status)) return fail(MOSAIC_E_ARG, "null argument");
    if (n_rowpath) *n_rowpath = 0;
    if (n == 0) return MOSAIC_OK;
    HIP_TRY(hipSetDevice(c->device));
    int rc;
    if ((rc = decode_coords(c, type_id, boundary_offsets, coord_offsets, value_offsets, values, valid, n, n_rowpath)))
        return rc;
    if ((rc = copy_out(c, x, c->dec_x.p, n * 8)) || (rc = copy_out(c, y, c->dec_y.p, n * 8)) ||
        (rc = copy_out(c, row_status, c->dec_status.p, n)))
        return rc;
    return MOSAIC_OK;
}

int mosaic_point_coords_to_cell(mosaic_ctx* ctx, int grid, int res, const int32_t* type_id,
                                const int32_t* boundary_offsets, const int32_t* coord_offsets,
                                const int32_t* value_offsets, const double* values, const uint8_t* valid, int64_t n,
                                int64_t* out_cell, uint8_t* row_status, int64_t* n_rowpath) {
    ENTER(ctx);
    if (n < 0) return fail(MOSAIC_E_ARG, "negative n");
    if (n > 0 && (!out_cell || !row_status)) return fail(MOSAIC_E_ARG, "null argument");
    if (grid != MOSAIC_GRID_H3 && grid != MOSAIC_GRID_BNG) return fail(MOSAIC_E_ARG, "unknown grid");
    if (!valid_res(grid, res)) return res_error(grid, res);
    if (n_rowpath) *n_rowpath = 0;
    if (n == 0) return MOSAIC_OK;
    HIP_TRY(hipSetDevice(c->device));
    int rc;
    if ((rc = decode_coords(c, type_id, boundary_offsets, coord_offsets, value_offsets, values, valid, n, n_rowpath)))
        return rc;
    c->async = 0;
    rc = point_to_cell_impl(c, grid, res, (const double*)c->dec_x.p, (const double*)c->dec_y.p, nullptr,
                            (const uint8_t*)c->dec_status.p, n, out_cell, nullptr);
    if (rc) return rc;
    return copy_out(c, row_status, c->dec_status.p, n);
}

int mosaic_bng_parse_column(mosaic_ctx* ctx, int offsets32, const void* offsets, const uint8_t* chars,
                            const uint8_t* valid, int64_t n, int64_t* out_ids) {
    ENTER(ctx);
    if (n < 0 || (n > 0 && (!offsets || !out_ids))) return fail(MOSAIC_E_ARG, "invalid argument");
    if (n == 0) return MOSAIC_OK;
    HIP_TRY(hipSetDevice(c->device));
    const size_t ob = offsets32 ? 4 : 8;
    int64_t end = 0;
    if (is_device_ptr(offsets)) {
        int64_t e64 = 0;
        int32_t e32 = 0;
        HIP_TRY(hipMemcpy(offsets32 ? (void*)&e32 : (void*)&e64, (const char*)offsets + n * ob, ob, hipMemcpyDeviceToHost));
        end = offsets32 ? e32 : e64;
    } else {
        end = offsets32 ? ((const int32_t*)offsets)[n] : ((const int64_t*)offsets)[n];
    }
    if (end < 0 || (end > 0 && !chars)) return fail(MOSAIC_E_ARG, "bad string column");
    DevBuf s_off, s_chars, s_valid, s_ids, s_bad;
    auto done = [&](int rc) {
        for (DevBuf* b : {&s_off, &s_chars, &s_valid, &s_ids, &s_bad}) b->release();
        return rc;
    };
    int rc;
    const void *doff, *dchars = nullptr, *dv;
    if ((rc = to_device(c, s_off, offsets, (size_t)(n + 1) * ob, &doff)) ||
        (end > 0 && (rc = to_device(c, s_chars, chars, (size_t)end, &dchars))) ||
        (rc = to_device(c, s_valid, valid, (size_t)n, &dv)) || (rc = s_bad.reserve(8)))
        return done(rc);
    const bool dev_out = is_device_ptr(out_ids);
    if (!dev_out && (rc = s_ids.reserve((size_t)n * 8))) return done(rc);
    HIP_TRY(hipMemsetAsync(s_bad.p, 0xff, 8, c->stream));
    ParseArgs a;
    a.offsets = doff;
    a.off64 = offsets32 ? 0 : 1;
    a.chars = (const uint8_t*)dchars;
    a.valid = (const uint8_t*)dv;
    a.n = n;
    a.ids = dev_out ? out_ids : (int64_t*)s_ids.p;
    a.first_bad = (unsigned long long*)s_bad.p;
    hipLaunchKernelGGL(k_bng_parse, dim3(grid_size(c, n)), dim3(c->block), 0, c->stream, a);
    HIP_TRY(hipGetLastError());
    unsigned long long bad = 0;
    HIP_TRY(hipMemcpyAsync(&bad, s_bad.p, 8, hipMemcpyDeviceToHost, c->stream));
    if (!dev_out) HIP_TRY(hipMemcpyAsync(out_ids, s_ids.p, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (bad != ~0ULL) return done(fail(MOSAIC_E_ARG, "invalid BNG id at row " + std::to_string(bad)));
    return done(MOSAIC_OK);
}

// BNGIndexSystem.letterMap (BNGIndexSystem.scala:84-99) and quadrants (:36)
static const char* kLetterMap[13][7] = {
    {"SV", "SW", "SX", "SY", "SZ", "TV", "TW"}, {"SQ", "SR", "SS", "ST", "SU", "TQ", "TR"},
    {"SL", "SM", "SN", "SO", "SP", "TL", "TM"}, {"SF", "SG", "SH", "SJ", "SK", "TF", "TG"},
    {"SA", "SB", "SC", "SD", "SE", "TA", "TB"}, {"NV", "NW", "NX", "NY", "NZ", "OV", "OW"},
    {"NQ", "NR", "NS", "NT", "NU", "OQ", "OR"}, {"NL", "NM", "NN", "NO", "NP", "OL", "OM"},
    {"NF", "NG", "NH", "NJ", "NK", "OF", "OG"}, {"NA", "NB", "NC", "ND", "NE", "OA", "OB"},
    {"HV", "HW", "HX", "HY", "SZ", "JV", "JW"}, {"HQ", "HR", "HS", "HT", "HU", "JQ", "JR"},
    {"HL", "HM", "HN", "HO", "HP", "JL", "JM"}};
static const char* kQuadrants[5] = {"", "SW", "NW", "NE", "SE"};

int mosaic_bng_format(int64_t id, char* buf, size_t cap) {
    if (!buf) return fail(MOSAIC_E_ARG, "null buffer");
    if (id <= 0) return fail(MOSAIC_E_ARG, "invalid BNG id " + std::to_string(id));
    std::string d = std::to_string(id);
    auto num = [&](size_t a, size_t b) -> int {  // digits.slice(a, b).mkString.toInt
        if (a >= d.size()) return -1;
        return std::stoi(d.substr(a, std::min(b, d.size()) - a));
    };
    int row = num(3, 5), col = num(1, 3);
    if (row < 0 || col < 0 || row > 12 || col > 6) return fail(MOSAIC_E_ARG, "invalid BNG id " + d);
    std::string s;
    if (d.size() < 6) {
        s = std::string(1, kLetterMap[row][col][0]);
    } else {
        int q = d.back() - '0';
        if (q > 4) return fail(MOSAIC_E_ARG, "invalid BNG id " + d);
        size_t k = (d.size() - 6) / 2;
        s = std::string(kLetterMap[row][col]) + d.substr(5, k) + d.substr(5 + k, k) + kQuadrants[q];
    }
    if (s.size() + 1 > cap) return fail(MOSAIC_E_CAPACITY, "buffer too small");
    memcpy(buf, s.c_str(), s.size() + 1);
    return (int)s.size();
}


int mosaic_bng_parse(const char* cs, int64_t* out) {
    if (!cs || !out) return fail(MOSAIC_E_ARG, "null argument");
    const size_t len = strlen(cs);
    if (len > 64 || !bng::parse(cs, (int)len, out)) return fail(MOSAIC_E_ARG, std::string("invalid BNG id ") + cs);
    return MOSAIC_OK;
}

static const int kLdsCountsMax = 8192;
static const size_t kStreamLdsMax = 160 * 1024;  // LDS per CU (MI355X): one k_join_stream workgroup's budget

static int chip_table_create(ThreadCtx* c, int grid, int res, int64_t n_chips, const uint8_t* is_core,
                             const int64_t* index_id, const void* wkb_off, bool off32, const uint8_t* wkb,
                             const int32_t* polygon_key, int32_t n_polygons, mosaic_chips** out);

int mosaic_chip_table_create(mosaic_ctx* ctx, int grid, int res, int64_t n_chips, const uint8_t* is_core,
                             const int64_t* index_id, const int64_t* wkb_offsets, const uint8_t* wkb,
                             const int32_t* polygon_key, int32_t n_polygons, mosaic_chips** out) {
    ENTER(ctx);
    return chip_table_create(c, grid, res, n_chips, is_core, index_id, wkb_offsets, false, wkb, polygon_key, n_polygons,
                             out);
}

int mosaic_chip_table_create_arrow(mosaic_ctx* ctx, int grid, int res, int64_t n_chips, const uint8_t* is_core,
                                   const int64_t* index_id, const void* wkb_offsets, int wkb_offsets32,
                                   const uint8_t* wkb, const int32_t* polygon_key, int32_t n_polygons,
                                   mosaic_chips** out) {
    ENTER(ctx);
    return chip_table_create(c, grid, res, n_chips, is_core, index_id, wkb_offsets, wkb_offsets32 != 0, wkb,
                             polygon_key, n_polygons, out);
}

struct TmpBuf : DevBuf {  // scratch released on every return path
    ~TmpBuf() { release(); }
};

static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// Build-side phase trace (measurement only): MOSAIC_BUILD_TRACE=1 prints each phase's wall time of
// a chip-table build to stderr.
// With the driver's per-process statistics readable, each line also shows the time the queues of
// every KFD process visible here have spent evicted so far (sysfs proc/<pid>/stats_<gpu>/evicted_ms;
// the pids are the host's, so all are listed).
static std::string kfd_evicted_ms() {
    std::string out;
    const char* root = "/sys/class/kfd/kfd/proc";
    if (DIR* d = opendir(root)) {
        while (dirent* e = readdir(d)) {
            if (e->d_name[0] == '.') continue;
            std::string pdir = std::string(root) + "/" + e->d_name;
            if (DIR* d2 = opendir(pdir.c_str())) {
                while (dirent* s = readdir(d2)) {
                    if (strncmp(s->d_name, "stats_", 6) != 0) continue;
                    std::string f = pdir + "/" + s->d_name + "/evicted_ms";
                    if (FILE* fp = fopen(f.c_str(), "r")) {
                        long long v = 0;
                        if (fscanf(fp, "%lld", &v) == 1) out += std::string(" ") + e->d_name + ":" + (s->d_name + 6) + "=" + std::to_string(v);
                        fclose(fp);
                    }
                }
                closedir(d2);
            }
        }
        closedir(d);
    }
    return out;
}
struct BuildTrace {
    bool on = getenv("MOSAIC_BUILD_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(const char* what) {
        if (!on) return;
        fprintf(stderr, "[build] %-28s %8.3f ms  (evicted ms:%s)\n", what, ms_since(t), kfd_evicted_ms().c_str());
        t = std::chrono::steady_clock::now();
    }
};

// The pages of a large host buffer that a device-to-host copy is about to fill: transparent huge pages
// where the system allows them, first touched by several threads (a copy into pageable memory
// otherwise takes every page fault on the one thread that runs it: 7 -> 36 ms swings in the raster
// build's copies of 15-23 MB).
static void prefault(void* p, size_t bytes) {
    if (bytes < ((size_t)4 << 20)) return;
    const uintptr_t a0 = (uintptr_t)p & ~(uintptr_t)4095, a1 = (uintptr_t)p + bytes;
    // (huge pages only on request, MOSAIC_THP=1: collapsing or migrating pages of a range the GPU
    // driver tracks evicts the process's queues -- see HostStage)
    static const bool thp = getenv("MOSAIC_THP") && getenv("MOSAIC_THP")[0] == '1';
    if (thp) (void)madvise((void*)a0, a1 - a0, MADV_HUGEPAGE);
    const int nt = (int)std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency()));
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; t++)
        pool.emplace_back([=]() {
            const uintptr_t b = a0 + (a1 - a0) / nt * t, e = t + 1 == nt ? a1 : a0 + (a1 - a0) / nt * (t + 1);
            for (uintptr_t q = std::max<uintptr_t>(b, (uintptr_t)p); q < e; q += 4096) *(volatile uint8_t*)q = 0;
        });
    for (auto& th : pool) th.join();
}

// Phase 1 of tiles::Builder::build_raster on the GPU (k_raster_sub, k_raster_line, k_raster_cells)
// over the chip table already on the device; the host then assembles the raster from `rc` exactly
// as after classify_raster_host, so both builds give the same bytes (raster_digest).
static int raster_classify_gpu(ThreadCtx* c, const mosaic_chips* ch, const tiles::Builder& tb,
                               tiles::Builder::RasterClass& rc) {
    BuildTrace trace;
    const size_t n_recs = tb.recs.size(), SS = (size_t)tb.S * tb.S, CC = (size_t)tb.C * tb.C;
    const int64_t n_sub = (int64_t)(n_recs * SS);
    if (tb.tile_of_rec.size() != n_recs || tb.rec_curv.size() != n_recs || !ch->tile_rec.p || !ch->tile_ent.p)
        return fail(MOSAIC_E_ARG, "raster build: tile directory not on the device");
    // (device scratch held by the thread state and reused: a build allocates and frees nothing here)
    DevBuf &d_tor = c->rbuild[0], &d_dev = c->rbuild[1], &d_code = c->rbuild[2], &d_list = c->rbuild[3],
           &d_kind = c->rbuild[4], &d_line = c->rbuild[5], &d_cells = c->rbuild[6];
    int e;
    if ((e = d_tor.reserve(std::max<size_t>(n_recs * 4, 16))) || (e = d_dev.reserve(std::max<size_t>(n_recs * sizeof(tiles::TileCurv), 16))) ||
        (e = d_code.reserve(std::max<size_t>((size_t)n_sub * 2, 16))))
        return e;
    if ((e = h2d(c, d_tor.p, tb.tile_of_rec.data(), n_recs * 4)) ||
        (e = h2d(c, d_dev.p, tb.rec_curv.data(), n_recs * sizeof(tiles::TileCurv))))
        return e;
    RBuildArgs a{};
    a.recs = (const tiles::TileRec*)ch->tile_rec.p;
    a.tile_of_rec = (const int32_t*)d_tor.p;
    a.rec_curv = (const tiles::TileCurv*)d_dev.p;
    a.entries = (const uint32_t*)ch->tile_ent.p;
    a.n_recs = (int32_t)n_recs;
    a.tnx = tb.grid.nx;
    a.gx0 = tb.grid.x0;
    a.gy0 = tb.grid.y0;
    a.tw = 1.0 / tb.grid.sx;
    a.th = 1.0 / tb.grid.sy;
    a.S = tb.S;
    a.C = tb.C;
    a.N = tb.S * tb.C;
    a.res = tb.res_;
    a.lines = tb.lines ? 1 : 0;
    a.table = (const HashEntry*)ch->table.p;
    a.meta = (const uint32_t*)ch->meta.p;
    a.store = ch->store.view();
    a.ht = tiles::Builder::hex_table_values();
    a.code = (uint16_t*)d_code.p;
    auto grid_of = [](int64_t n) { return dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 1 << 22))); };
    rc.code.resize((size_t)n_sub);
    prefault(rc.code.data(), rc.code.size() * 2);
    if (n_sub) {
        hipLaunchKernelGGL(k_raster_sub, grid_of(n_sub), dim3(256), 0, c->stream, a);
        HIP_TRY(hipGetLastError());
        if ((e = d2h(c, rc.code.data(), d_code.p, (size_t)n_sub * 2))) return e;
    }
    trace.mark("  k_raster_sub + copy");
    // mixed sub-blocks in record, then scan order (the order assemble_raster consumes them)
    std::vector<uint32_t> list;
    for (int64_t g = 0; g < n_sub; g++)
        if (rc.code[(size_t)g] == tiles::kMixed) list.push_back((uint32_t)g);
    const int64_t n_mixed = (int64_t)list.size();
    rc.kind.assign((size_t)n_mixed, 0);
    rc.line.assign((size_t)n_mixed, tiles::LineRec{0, 0, 0, 0, 0});
    rc.cell_at.assign((size_t)n_mixed, 0);
    rc.cells.clear();
    if (!n_mixed) return MOSAIC_OK;
    if ((e = d_list.reserve(list.size() * 4)) || (e = d_kind.reserve(list.size())) ||
        (e = d_line.reserve(list.size() * sizeof(tiles::LineRec))))
        return e;
    if ((e = h2d(c, d_list.p, list.data(), list.size() * 4))) return e;
    a.mixed = (const uint32_t*)d_list.p;
    a.n_mixed = n_mixed;
    a.kind = (uint8_t*)d_kind.p;
    a.line = (tiles::LineRec*)d_line.p;
    if (c->raster_build == 2)  // one lane per sub-block (the first GPU form, kept for comparison)
        hipLaunchKernelGGL(k_raster_line, grid_of(n_mixed), dim3(256), 0, c->stream, a);
    else  // one wave per sub-block
        hipLaunchKernelGGL(k_raster_line_wave, dim3((unsigned)((n_mixed + 3) / 4)), dim3(256), 0, c->stream, a);
    HIP_TRY(hipGetLastError());
    if ((e = d2h(c, rc.kind.data(), d_kind.p, list.size())) ||
        (e = d2h(c, rc.line.data(), d_line.p, list.size() * sizeof(tiles::LineRec))))
        return e;
    trace.mark("  mixed list + line kernel");
    // the other mixed sub-blocks: C x C leaf cells each
    std::vector<uint32_t> cell_sb;
    for (int64_t m = 0; m < n_mixed; m++)
        if (!rc.kind[(size_t)m]) {
            rc.cell_at[(size_t)m] = (uint32_t)cell_sb.size();
            cell_sb.push_back(list[(size_t)m]);
        }
    if (cell_sb.empty()) return MOSAIC_OK;
    const int64_t n_cells = (int64_t)(cell_sb.size() * CC);
    if ((e = d_cells.reserve((size_t)n_cells * 2))) return e;
    if ((e = h2d(c, d_list.p, cell_sb.data(), cell_sb.size() * 4))) return e;
    a.cell_sb = (const uint32_t*)d_list.p;
    a.n_cell_sb = (int64_t)cell_sb.size();
    a.cells = (uint16_t*)d_cells.p;
    // (one lane per leaf cell; a workgroup-per-sub-block form with the candidate hexagons and corner
    // images in LDS measured slower: 7.4 -> 9.6 ms for NYC res 9, profiles/r03_build_trace_v4.txt)
    hipLaunchKernelGGL(k_raster_cells, grid_of(n_cells), dim3(256), 0, c->stream, a);
    HIP_TRY(hipGetLastError());
    rc.cells.resize((size_t)n_cells);
    prefault(rc.cells.data(), rc.cells.size() * 2);
    if ((e = d2h(c, rc.cells.data(), d_cells.p, (size_t)n_cells * 2))) return e;
    trace.mark("  k_raster_cells + copy");
    rc.cline_at.clear();
    rc.cline.clear();
    if (!tb.leaf_lines) return MOSAIC_OK;
    // leaf lines: the kMixed cells in index order (hipcub select), one line fit per cell
    DevBuf &d_ml = c->rbuild[7], &d_nml = c->rbuild[8], &d_tmp = c->rbuild[9], &d_ok = c->rbuild[10],
           &d_lrec = c->rbuild[11];
    if ((e = d_ml.reserve((size_t)n_cells * 4)) || (e = d_nml.reserve(8))) return e;
    hipcub::CountingInputIterator<uint32_t> idx(0u);
    size_t tmp_bytes = 0;
    HIP_TRY(hipcub::DeviceSelect::If(nullptr, tmp_bytes, idx, (uint32_t*)d_ml.p, (int64_t*)d_nml.p, n_cells,
                                     RasterMixedCell{(const uint16_t*)d_cells.p}, c->stream));
    if ((e = d_tmp.reserve(std::max<size_t>(tmp_bytes, 16)))) return e;
    HIP_TRY(hipcub::DeviceSelect::If(d_tmp.p, tmp_bytes, idx, (uint32_t*)d_ml.p, (int64_t*)d_nml.p, n_cells,
                                     RasterMixedCell{(const uint16_t*)d_cells.p}, c->stream));
    int64_t n_ml = 0;
    if ((e = d2h(c, &n_ml, d_nml.p, 8))) return e;
    if (n_ml <= 0) return MOSAIC_OK;
    DevBuf &d_cands = c->rbuild[12], &d_ncand = c->rbuild[13];
    if ((e = d_ok.reserve((size_t)n_ml)) || (e = d_lrec.reserve((size_t)n_ml * sizeof(tiles::LineRec))) ||
        (e = d_cands.reserve(cell_sb.size() * 64 * 4)) || (e = d_ncand.reserve(cell_sb.size() * 4)))
        return e;
    hipLaunchKernelGGL(k_sub_cands, dim3((unsigned)((cell_sb.size() + 3) / 4)), dim3(256), 0, c->stream, a,
                       (int32_t*)d_cands.p, (int32_t*)d_ncand.p);
    hipLaunchKernelGGL(k_raster_cell_lines, dim3((unsigned)((n_ml + 3) / 4)), dim3(256), 0, c->stream, a,
                       (const uint32_t*)d_ml.p, n_ml, (const int32_t*)d_cands.p, (const int32_t*)d_ncand.p,
                       (uint8_t*)d_ok.p, (tiles::LineRec*)d_lrec.p);
    HIP_TRY(hipGetLastError());
    std::vector<uint32_t> ml((size_t)n_ml);
    std::vector<uint8_t> okv((size_t)n_ml);
    std::vector<tiles::LineRec> lrec((size_t)n_ml);
    if ((e = d2h(c, okv.data(), d_ok.p, (size_t)n_ml)) || (e = d2h(c, ml.data(), d_ml.p, (size_t)n_ml * 4)) ||
        (e = d2h(c, lrec.data(), d_lrec.p, (size_t)n_ml * sizeof(tiles::LineRec))))
        return e;
    for (int64_t m = 0; m < n_ml; m++)
        if (okv[(size_t)m]) {
            rc.cline_at.push_back(ml[(size_t)m]);
            rc.cline.push_back(lrec[(size_t)m]);
        }
    trace.mark("  leaf lines");
    return MOSAIC_OK;
}

// FNV-1a over 8-byte words (then the tail bytes): a fingerprint of the raster arrays
static uint64_t fnv1a(uint64_t h, const void* p, size_t n) {
    const uint8_t* b = (const uint8_t*)p;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, b + i, 8);
        h = (h ^ w) * 1099511628211ull;
    }
    for (; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

static int chip_table_create(ThreadCtx* c, int grid, int res, int64_t n_chips, const uint8_t* is_core,
                             const int64_t* index_id, const void* wkb_off, bool off32, const uint8_t* wkb,
                             const int32_t* polygon_key, int32_t n_polygons, mosaic_chips** out) {
    const auto t_begin = std::chrono::steady_clock::now();
    BuildTrace trace;
    // Arrow binary (int32 offsets) or large_binary (int64)
    auto wkb_offsets = [&](int64_t i) -> int64_t {
        return off32 ? (int64_t)((const int32_t*)wkb_off)[i] : ((const int64_t*)wkb_off)[i];
    };
    if (!c || !out || n_chips < 0 || n_polygons < 0) return fail(MOSAIC_E_ARG, "invalid argument");
    if (n_chips > 0 && (!is_core || !index_id || !wkb_off || !polygon_key))
        return fail(MOSAIC_E_ARG, "null chip column");
    if (grid != MOSAIC_GRID_H3 && grid != MOSAIC_GRID_BNG) return fail(MOSAIC_E_ARG, "unknown grid");
    if (!valid_res(grid, res)) return res_error(grid, res);
    if (n_chips >= (int64_t)1 << 31) return fail(MOSAIC_E_ARG, "too many chips");
    HIP_TRY(hipSetDevice(c->device));
    // chips grouped by cell, original order kept within a cell: (cell, position) pairs sorted on
    // host threads (sorted runs, then pairwise merges), which is the stable order by cell
    const int n_thr = (int)std::max<int64_t>(
        1, std::min<int64_t>(std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency())), n_chips / 65536));
    std::vector<uint32_t> order(n_chips);
    {
        std::vector<std::pair<int64_t, uint32_t>> kv((size_t)n_chips), tmp;
        auto range = [&](int k, int parts) { return (int64_t)((__int128)n_chips * k / parts); };
        parallel_for(n_thr, [&](int k) {
            for (int64_t t = range(k, n_thr); t < range(k + 1, n_thr); t++) kv[(size_t)t] = {index_id[t], (uint32_t)t};
            std::sort(kv.begin() + range(k, n_thr), kv.begin() + range(k + 1, n_thr));
        });
        if (n_thr > 1) tmp.resize(kv.size());
        for (int w = 1; w < n_thr; w *= 2) {  // merge runs [k w, (k + 1) w) pairwise
            const int groups = (n_thr + 2 * w - 1) / (2 * w);
            parallel_for(groups, [&](int g) {
                const int64_t a0 = range(2 * g * w, n_thr), a1 = range(std::min(2 * g * w + w, n_thr), n_thr),
                              b1 = range(std::min(2 * g * w + 2 * w, n_thr), n_thr);
                std::merge(kv.begin() + a0, kv.begin() + a1, kv.begin() + a1, kv.begin() + b1, tmp.begin() + a0);
            });
            kv.swap(tmp);
        }
        parallel_for(n_thr, [&](int k) {
            for (int64_t t = range(k, n_thr); t < range(k + 1, n_thr); t++) order[(size_t)t] = kv[(size_t)t].second;
        });
    }
    trace.mark("sort by cell");
    // WKB parse on host threads, contiguous ranges of the sorted order, then concatenated: the same
    // arrays (and the same first error) as one sequential pass
    GeomBuilder gb;
    std::vector<uint32_t> meta(std::max<int64_t>(n_chips, 1));
    int64_t n_border = 0;
    {
        struct Part {
            GeomBuilder gb;
            int64_t n_border = 0, bad_t = -1;
            int bad_code = 0;
            std::string bad_msg;
        };
        std::vector<Part> parts((size_t)n_thr);
        auto range = [&](int k) { return (int64_t)((__int128)n_chips * k / n_thr); };
        parallel_for(n_thr, [&](int k) {
            Part& pt = parts[(size_t)k];
            for (int64_t t = range(k); t < range(k + 1); t++) {
                uint32_t i = order[t];
                auto bad = [&](int code, const std::string& msg) {
                    pt.bad_t = t;
                    pt.bad_code = code;
                    pt.bad_msg = msg;
                };
                if (polygon_key[i] < 0 || polygon_key[i] >= n_polygons) {
                    bad(MOSAIC_E_ARG, "polygon_key out of range at chip " + std::to_string(i));
                    return;
                }
                if (index_id[i] == kEmptyKey) {
                    bad(MOSAIC_E_ARG, "reserved index_id at chip " + std::to_string(i));
                    return;
                }
                bool core = is_core[i] != 0;
                meta[t] = ((uint32_t)polygon_key[i] << 1) | (core ? 1u : 0u);
                int64_t a = wkb_offsets(i), b = wkb_offsets(i + 1);
                if (b < a || (b > a && !wkb)) {
                    bad(MOSAIC_E_ARG, "bad wkb offsets at chip " + std::to_string(i));
                    return;
                }
                // core chips are accepted without a test: their geometry is never read
                if (!pt.gb.add(core ? nullptr : wkb + a, core ? 0 : (size_t)(b - a))) {
                    bad(MOSAIC_E_WKB, "chip " + std::to_string(i) + ": " + pt.gb.error);
                    return;
                }
                pt.n_border += !core;
            }
        });
        for (const Part& pt : parts)  // the first failing chip in the sorted order, as a sequential pass
            if (pt.bad_t >= 0) return fail(pt.bad_code, pt.bad_msg);
        size_t nv = 0, nr = 0, np = 0, ng = 0;
        std::vector<size_t> v0(parts.size()), r0(parts.size()), p0(parts.size()), g0(parts.size());
        for (size_t k = 0; k < parts.size(); k++) {
            v0[k] = nv;
            r0[k] = nr;
            p0[k] = np;
            g0[k] = ng;
            nv += parts[k].gb.verts.size();
            nr += parts[k].gb.ring_bbox.size();
            np += parts[k].gb.part_ring.size() - 1;
            ng += parts[k].gb.geom_bbox.size();
            n_border += parts[k].n_border;
        }
        if (nv > std::numeric_limits<uint32_t>::max()) return fail(MOSAIC_E_WKB, "too many vertices");
        gb.verts.resize(nv);
        gb.ring_bbox.resize(nr);
        gb.ring_start.resize(nr + 1);
        gb.part_ring.resize(np + 1);
        gb.geom_part.resize(ng + 1);
        gb.geom_bbox.resize(ng);
        parallel_for((int)parts.size(), [&](int k) {
            const GeomBuilder& q = parts[(size_t)k].gb;
            std::copy(q.verts.begin(), q.verts.end(), gb.verts.begin() + v0[k]);
            std::copy(q.ring_bbox.begin(), q.ring_bbox.end(), gb.ring_bbox.begin() + r0[k]);
            std::copy(q.geom_bbox.begin(), q.geom_bbox.end(), gb.geom_bbox.begin() + g0[k]);
            for (size_t j = 1; j < q.ring_start.size(); j++) gb.ring_start[r0[k] + j] = q.ring_start[j] + (uint32_t)v0[k];
            for (size_t j = 1; j < q.part_ring.size(); j++) gb.part_ring[p0[k] + j] = q.part_ring[j] + (uint32_t)r0[k];
            for (size_t j = 1; j < q.geom_part.size(); j++) gb.geom_part[g0[k] + j] = q.geom_part[j] + (uint32_t)p0[k];
        });
    }
    trace.mark("wkb parse");
    // distinct cells -> [first, count)
    std::vector<std::pair<int64_t, uint32_t>> cells;  // (cell, first)
    std::vector<uint32_t> counts;
    for (int64_t t = 0; t < n_chips; t++) {
        int64_t id = index_id[order[t]];
        if (cells.empty() || cells.back().first != id) {
            cells.push_back({id, (uint32_t)t});
            counts.push_back(0);
        }
        counts.back()++;
    }
    uint64_t capacity = 16;
    while (capacity < 2 * cells.size() + 1) capacity <<= 1;
    std::vector<HashEntry> table(capacity, HashEntry{kEmptyKey, 0, 0});
    for (size_t k = 0; k < cells.size(); k++) {
        uint64_t slot = mix64((uint64_t)cells[k].first) & (capacity - 1);
        while (table[slot].key != kEmptyKey) slot = (slot + 1) & (capacity - 1);
        table[slot] = HashEntry{cells[k].first, cells[k].second, counts[k]};
    }
    mosaic_chips* ch = new mosaic_chips();
    ch->grid = grid;
    ch->res = res;
    ch->device = c->device;
    ch->n_chips = n_chips;
    ch->n_cells = (int64_t)cells.size();
    ch->n_border = n_border;
    ch->n_vertices = (int64_t)gb.verts.size();
    ch->n_rings = (int64_t)gb.ring_bbox.size();
    ch->n_polygons = n_polygons;
    ch->capacity = capacity;
    // ring descriptors: the common chip (one Polygon, one shell ring) is tested without walking
    // the part / ring offset arrays
    std::vector<uint2> ring_desc(meta.size(), make_uint2(0, 0));
    for (int64_t t = 0; t < n_chips; t++) {
        uint32_t p0 = gb.geom_part[t], p1 = gb.geom_part[t + 1];
        if (p1 - p0 != 1) continue;
        uint32_t r0 = gb.part_ring[p0], r1 = gb.part_ring[p0 + 1];
        if (r1 - r0 != 1) continue;
        uint32_t v0 = gb.ring_start[r0], v1 = gb.ring_start[r0 + 1];
        if (v1 > v0) ring_desc[t] = make_uint2(v0, v1 - v0);
    }
    // ray-parity rasters for one-ring border chips (raster.h); other chips take the general path
    // (contiguous chip ranges on host threads, concatenated in chip order: the same arrays as one
    // sequential pass).  Built on a background thread while the tile directory is built and the
    // point raster is classified on the GPU (neither reads them); joined before their upload.
    raster::Builder rb;
    rb.hdr.resize(meta.size());
    bool rb_overflow = false;
    // too many polygons for point-raster codes (H3): the join sorts points by tile and tests chips
    // from LDS tile images or the chip table (join_binned.hip), not through chip rasters, so small
    // rings (buildings) get none -- their direct ring walk is as short as a raster lookup
    const int64_t min_segments = (grid == MOSAIC_GRID_H3 && n_polygons > (int32_t)tiles::kMaxRasterKeys)
                                     ? std::max<int64_t>(c->raster_min_segments, 16)
                                     : c->raster_min_segments;
    auto chip_rasters = [&]() {
        const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(
            std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency())), n_chips / 256));
        std::vector<raster::Builder> part((size_t)nt);
        auto work = [&](int k) {
            raster::Builder& pb = part[(size_t)k];
            for (int64_t t = n_chips * k / nt; t < n_chips * (k + 1) / nt; t++) {
                raster::ChipHdr& h = rb.hdr[t];
                memset(&h, 0, sizeof h);
                h.box = gb.geom_bbox[t];
                h.cell_base = raster::kNoRaster;
                uint2 d = ring_desc[t];
                if (!(meta[t] & 1u) && d.y >= 2 && (int64_t)d.y - 1 >= min_segments) {
                    // option raster_adaptive: small rings get small rasters (2 ceil(sqrt(segments))
                    // cells a side, at most "raster"), so tables of millions of small chips stay compact
                    int dims = c->raster;
                    if (c->raster_adaptive) dims = std::min(dims, std::max(2, 2 * (int)ceil(sqrt((double)(d.y - 1)))));
                    pb.add_ring(h, gb.verts.data() + d.x, d.y, dims);
                }
            }
        };
        std::vector<std::thread> pool;
        for (int k = 1; k < nt; k++) pool.emplace_back(work, k);
        work(0);
        for (auto& th : pool) th.join();
        for (int k = 0; k < nt; k++) {
            const size_t c0 = rb.cells.size(), e0 = rb.edges.size();
            for (int64_t t = n_chips * k / nt; t < n_chips * (k + 1) / nt; t++)
                if (rb.hdr[t].cell_base != raster::kNoRaster) rb.hdr[t].cell_base += (uint32_t)c0;
            for (raster::CellRec cr : part[(size_t)k].cells) {
                if (cr.m) cr.word += (uint32_t)(e0 << 1);
                rb.cells.push_back(cr);
            }
            rb.edges.insert(rb.edges.end(), part[(size_t)k].edges.begin(), part[(size_t)k].edges.end());
            rb.pure_cells += part[(size_t)k].pure_cells;
            if (rb.edges.size() >= (1ull << 31) || rb.cells.size() >= (size_t)raster::kNoRaster) {
                rb_overflow = true;
                return;
            }
        }
        if (meta.size() > (size_t)n_chips) {
            memset(&rb.hdr.back(), 0, sizeof(raster::ChipHdr));
            rb.hdr.back().cell_base = raster::kNoRaster;
        }
        if (rb.cells.empty()) rb.cells.push_back(raster::CellRec{0, 0});
        if (rb.edges.empty()) rb.edges.push_back(pip::Edge{0, 0, 0, 0});
    };
    struct JoinOnExit {  // every return path waits for the background build first
        std::thread t;
        ~JoinOnExit() {
            if (t.joinable()) t.join();
        }
    } rb_job;
    rb_job.t = std::thread(chip_rasters);
    ch->raster = c->raster;
    size_t total = 0;
    int rc;
    if ((rc = ch->table.reserve(capacity * sizeof(HashEntry))) || (rc = ch->meta.reserve(meta.size() * 4)) ||
        (rc = ch->store.upload(gb, c, &total))) {
        ch->release_all();
        delete ch;
        return rc;
    }
    if ((rc = h2d(c, ch->table.p, table.data(), capacity * sizeof(HashEntry))) ||
        (rc = h2d(c, ch->meta.p, meta.data(), meta.size() * 4)))
        return rc;
    // the chip rasters: joined here when the build has no point raster to classify, else after it
    bool rb_uploaded = false;
    auto upload_chip_rasters = [&]() -> int {
        if (rb_uploaded) return MOSAIC_OK;
        rb_uploaded = true;
        if (rb_job.t.joinable()) rb_job.t.join();
        trace.mark("chip rasters (joined)");
        if (rb_overflow) return fail(MOSAIC_E_ARG, "chip table too large for the raster record index");
        ch->raster_cells = (int64_t)rb.cells.size();
        ch->raster_pure = rb.pure_cells;
        ch->raster_records = (int64_t)rb.edges.size();
        int e;
        if ((e = ch->hdr.reserve(rb.hdr.size() * sizeof(raster::ChipHdr))) ||
            (e = ch->cells.reserve(rb.cells.size() * sizeof(raster::CellRec))) ||
            (e = ch->rast_edges.reserve(rb.edges.size() * sizeof(pip::Edge))))
            return e;
        if ((e = h2d(c, ch->hdr.p, rb.hdr.data(), rb.hdr.size() * sizeof(raster::ChipHdr))) ||
            (e = h2d(c, ch->cells.p, rb.cells.data(), rb.cells.size() * sizeof(raster::CellRec))) ||
            (e = h2d(c, ch->rast_edges.p, rb.edges.data(), rb.edges.size() * sizeof(pip::Edge))))
            return e;
        return MOSAIC_OK;
    };
    trace.mark("core uploads");
    if (grid == MOSAIC_GRID_BNG && res >= 1 && c->tiles && !cells.empty()) {
        // BNG dense cell table (see k_join_stream_bng): decode every chip cell id to its cell
        // coordinates and check the decoding by re-encoding the cell's lower-left corner
        const int32_t div = (int32_t)bng::pow10i(6 - res), per = 100000 / div;
        const int64_t p10n = (int64_t)bng::pow10i(res), p10n1 = (int64_t)bng::pow10i(res - 1);
        std::vector<std::pair<int32_t, int32_t>> cc(cells.size());
        bool ok = true;
        int32_t e0 = INT32_MAX, n0 = INT32_MAX, e1 = -1, n1 = -1;
        for (size_t k = 0; k < cells.size() && ok; k++) {
            const int64_t id = cells[k].first;
            if (id < 0) {
                ok = false;
                break;
            }
            const int64_t nBin = (id / 10) % p10n1, eBin = (id / p10n) % p10n1;
            // id = 10^(2n+3) + eL 10^(2n+1) + nL 10^(2n-1) + eBin 10^n + nBin 10 + quadrant (n = res)
            const int64_t sh_nL = (int64_t)bng::pow10i(2 * res - 1), sh_eL = (int64_t)bng::pow10i(2 * res + 1);
            const int64_t nLet = (id / sh_nL) % 100, eLet = (id / sh_eL) % 100;
            const int64_t ce = eLet * per + eBin, cn = nLet * per + nBin;
            int64_t re = 0;
            if (ce < 0 || cn < 0 || (ce + 1) * div > 10000000 || (cn + 1) * div > 10000000 ||
                !bng::point_to_index((double)(ce * div), (double)(cn * div), res, &re) || re != id) {
                ok = false;
                break;
            }
            cc[k] = {(int32_t)ce, (int32_t)cn};
            e0 = std::min(e0, (int32_t)ce);
            e1 = std::max(e1, (int32_t)ce);
            n0 = std::min(n0, (int32_t)cn);
            n1 = std::max(n1, (int32_t)cn);
        }
        const int64_t ne = (int64_t)e1 - e0 + 1, nn = (int64_t)n1 - n0 + 1;
        if (ok && ne > 0 && nn > 0 && ne * nn <= ((int64_t)1 << 26)) {
            std::vector<uint32_t> tab((size_t)(ne * nn), 0u);
            std::vector<tiles::BngBorderCell> border;
            std::vector<size_t> border_at;
            for (size_t k = 0; k < cells.size(); k++) {
                uint64_t slot = mix64((uint64_t)cells[k].first) & (capacity - 1);
                while (table[slot].key != cells[k].first) slot = (slot + 1) & (capacity - 1);
                const HashEntry& he = table[slot];
                uint32_t ent = (uint32_t)slot + 1;
                const size_t at = (size_t)((cc[k].second - n0) * ne + (cc[k].first - e0));
                if (he.count == 1 && (meta[he.first] & 1u) && (meta[he.first] >> 1) + 1 < (uint32_t)tiles::kMixed) {
                    ent = kBngPure | ((meta[he.first] >> 1) + 1);
                } else if (n_polygons < tiles::kMaxRasterKeys && c->point_raster) {
                    border.push_back(tiles::BngBorderCell{(double)cc[k].first * div, (double)cc[k].second * div,
                                                          (uint32_t)slot});
                    border_at.push_back(at);
                }
                tab[at] = ent;
            }
            // leaf blocks of the border cells (C x C sub-cell entries, C = option bng_cell: 3.1 m
            // sub-cells at 100 m resolution with the default 32; line records with option raster_lines)
            std::vector<uint16_t> leaf;
            std::vector<uint32_t> lbase_kept;  // border cell b's leaf block at leaf[lbase_kept[b]]
            std::vector<uint16_t> bng_glines;  // group-level line codes (tiles.h bng_leaf_blocks glines)
            const int C = c->bng_cell;
            if (!border.empty()) {
                std::vector<uint32_t> sfirst(capacity, 0), scount(capacity, 0);
                for (uint64_t q = 0; q < capacity; q++)
                    if (table[q].key != kEmptyKey) {
                        sfirst[q] = table[q].first;
                        scount[q] = table[q].count;
                    }
                tiles::Builder::ChipSource src;
                src.slot_first = sfirst.data();
                src.slot_count = scount.data();
                src.meta = meta.data();
                src.store = pip::GeomStore{gb.verts.data(), gb.ring_start.data(), gb.ring_bbox.data(),
                                           gb.part_ring.data(), gb.geom_part.data(), gb.geom_bbox.data()};
                src.n_polygons = n_polygons;
                int threads = (int)std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency()));
                // (leaf offsets are 32-bit buffer offsets in k_join_stream_bng)
                std::vector<uint32_t>& lbase = lbase_kept;
                // (leaf element offsets < 2^30, byte offsets below kNoLoad)
                if (tiles::bng_leaf_blocks(src, border, (double)div, C, c->raster_lines != 0, threads, leaf, lbase,
                                           c->bng_group_lines ? &bng_glines : nullptr, c->bng_wedges != 0) &&
                    leaf.size() * 2 < (size_t)kNoLoad) {
                    for (size_t b = 0; b < border.size(); b++) {
                        tab[border_at[b]] = kBngLeaf | lbase[b];
                        for (int q = 0; q < C * C; q++) {
                            const uint16_t v = leaf[lbase[b] + q];
                            ch->bng_sub_stats[0] += v == tiles::kMixed;
                            ch->bng_sub_stats[1] += v != tiles::kMixed && (v & 0xC000u) == 0xC000u;
                        }
                    }
                    ch->bng_C = C;
                    ch->bng_wedges = c->bng_wedges && c->raster_lines ? 1 : 0;
                } else {
                    leaf.clear();
                }
            }
            if (leaf.empty()) leaf.assign((size_t)C * C, tiles::kMixed);
            // sub-block levels, dense over the table's cells (only border cells' lines are ever read:
            // k_join_stream_bng_cpt gathers them beside the cell entry); tables too large for a
            // 512 MB level array take k_join_stream_bng
            std::vector<uint16_t> lvl;
            const int LV = tiles::bng_level_stride(C), CB = tiles::bng_level_side(C);
            if (ch->bng_C && (size_t)tab.size() * LV * 2 <= ((size_t)512 << 20)) {
                lvl.assign(tab.size() * (size_t)LV, tiles::kMixed);
                for (size_t b = 0; b < border.size(); b++)
                    for (int bj = 0; bj < CB; bj++)
                        for (int bi = 0; bi < CB; bi++)
                        {
                            uint16_t v = tiles::bng_level_code(&leaf[lbase_kept[b]], C, bi, bj);
                            // a group certified for one line record: that line code (tiles.h glines)
                            if (v == tiles::kSubBlock && !bng_glines.empty()) v = bng_glines[b * (size_t)CB * CB + (size_t)bj * CB + bi];
                            lvl[border_at[b] * LV + (size_t)bj * CB + bi] = v;
                        }
            }
            // LDS cell level (BngStreamArgs::lcell): the finest block size 2^lsh whose byte table fits
            // the stream kernel's LDS beside its counts and 16 per-wave stages
            std::vector<uint8_t> lcell;
            int lsh = 0;
            int64_t lnx = 0;
            if (c->bng_lds) {
                const size_t other = (n_polygons <= kLdsCountsMax ? ((size_t)n_polygons + 64) * 4 : 0) + 16 * kStageWords * 4;
                const size_t budget = kStreamLdsMax > other ? (kStreamLdsMax - other) & ~(size_t)3 : 0;
                int64_t lny = 0;
                for (; lsh <= 16; lsh++) {
                    lnx = (ne + (1 << lsh) - 1) >> lsh;
                    lny = (nn + (1 << lsh) - 1) >> lsh;
                    if ((size_t)((lnx * lny + 3) & ~3) <= budget) break;
                }
                if (lsh <= 16) {
                    auto byte_of = [](uint32_t t) -> uint8_t {
                        if (t == 0) return 0;
                        if ((t & kBngPure) && (t & ~kBngPure) < kBngLdsGather) return (uint8_t)(t & ~kBngPure);
                        return (uint8_t)kBngLdsGather;
                    };
                    lcell.assign((size_t)((lnx * lny + 3) & ~3), 0);
                    std::vector<uint8_t> seen(lcell.size(), 0);
                    for (int64_t j = 0; j < nn; j++)
                        for (int64_t i = 0; i < ne; i++) {
                            const size_t b = (size_t)((j >> lsh) * lnx + (i >> lsh));
                            const uint8_t v = byte_of(tab[(size_t)(j * ne + i)]);
                            if (!seen[b]) lcell[b] = v, seen[b] = 1;
                            else if (lcell[b] != v) lcell[b] = (uint8_t)kBngLdsGather;
                        }
                }
            }
            size_t bb = tab.size() * 4, lb = leaf.size() * 2;
            if ((rc = ch->bng_cells.reserve(bb)) || (rc = ch->bng_leaf.reserve(lb)) ||
                (!lvl.empty() && (rc = ch->bng_lvl.reserve(lvl.size() * 2))) ||
                (!lcell.empty() && (rc = ch->bng_lcell.reserve(lcell.size())))) {
                ch->release_all();
                delete ch;
                return rc;
            }
            if ((rc = h2d(c, ch->bng_cells.p, tab.data(), bb))) return rc;
            if ((rc = h2d(c, ch->bng_leaf.p, leaf.data(), lb))) return rc;
            if (!lvl.empty()) {
                if ((rc = h2d(c, ch->bng_lvl.p, lvl.data(), lvl.size() * 2))) return rc;
                ch->bng_lvl_bytes = lvl.size() * 2;
                total += lvl.size() * 2;
            }
            ch->bng_cpt_ok = !lvl.empty() || !ch->bng_C;
            if (!lcell.empty()) {
                if ((rc = h2d(c, ch->bng_lcell.p, lcell.data(), lcell.size()))) return rc;
                ch->bng_lwords = (int32_t)(lcell.size() / 4);
                ch->bng_lsh = lsh;
                ch->bng_lnx = (int32_t)lnx;
                total += lcell.size();
            }
            ch->bng_leaf_bytes = lb;
            total += lb;
            if (!ch->bng_C) ch->bng_C = C;
            ch->bng_ok = true;
            ch->bng_e0 = e0;
            ch->bng_n0 = n0;
            ch->bng_ne = (int32_t)ne;
            ch->bng_nn = (int32_t)nn;
            ch->bng_div = div;
            total += bb;
        }
    }
    if (grid == MOSAIC_GRID_H3 && c->tiles && !cells.empty()) {
        std::vector<int64_t> cell_ids(cells.size());
        for (size_t k = 0; k < cells.size(); k++) cell_ids[k] = cells[k].first;
        const uint64_t cmask = capacity - 1;
        auto slot_of = [&](int64_t h) -> int64_t {
            uint64_t slot = mix64((uint64_t)h) & cmask;
            while (table[slot].key != kEmptyKey) {
                if (table[slot].key == h) return (int64_t)slot;
                slot = (slot + 1) & cmask;
            }
            return -1;
        };
        tiles::Builder tb;
        ch->build_ms[0] = ms_since(t_begin);
        auto t_dir = std::chrono::steady_clock::now();
        trace.mark("(core)");
        const bool dir_ok = tb.build(res, cell_ids, slot_of);
        ch->build_ms[1] = ms_since(t_dir);
        trace.mark("tile directory");
        if (dir_ok) {
            size_t b0 = tb.tile_idx.size() * 4, b1 = tb.recs.size() * sizeof(tiles::TileRec), b2 = tb.entries.size() * 4;
            if ((rc = ch->tile_idx.reserve(b0)) || (rc = ch->tile_rec.reserve(b1)) || (rc = ch->tile_ent.reserve(b2))) {
                ch->release_all();
                delete ch;
                return rc;
            }
            if ((rc = h2d(c, ch->tile_idx.p, tb.tile_idx.data(), b0))) return rc;
            if ((rc = h2d(c, ch->tile_rec.p, tb.recs.data(), b1))) return rc;
            if ((rc = h2d(c, ch->tile_ent.p, tb.entries.data(), b2))) return rc;
            ch->tiles_ok = true;
            ch->tgrid = tb.grid;
            ch->tile_stats[0] = tb.grid.nx;
            ch->tile_stats[1] = tb.grid.ny;
            ch->tile_stats[2] = (int64_t)tb.recs.size();
            ch->tile_stats[3] = (int64_t)tb.entries.size();
            ch->tile_stats[4] = tb.n_full;
            ch->tile_stats[5] = tb.rings;
            total += b0 + b1 + b2;
            if (c->point_raster) {
                std::vector<uint32_t> sfirst(capacity, 0), scount(capacity, 0);
                for (uint64_t q = 0; q < capacity; q++)
                    if (table[q].key != kEmptyKey) {
                        sfirst[q] = table[q].first;
                        scount[q] = table[q].count;
                    }
                tiles::Builder::ChipSource src;
                src.slot_first = sfirst.data();
                src.slot_count = scount.data();
                src.meta = meta.data();
                src.store = pip::GeomStore{gb.verts.data(), gb.ring_start.data(), gb.ring_bbox.data(),
                                           gb.part_ring.data(), gb.geom_part.data(), gb.geom_bbox.data()};
                src.n_polygons = n_polygons;
                int threads = (int)std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency()));
                // LDS quad level: by default as many entries as one k_join_stream workgroup's LDS holds
                // beside its counts, its per-wave stages (1024 threads) and, when small, tile_base
                size_t avail = kStreamLdsMax - 16 * kStageWords * 4 - 1024 -
                               (n_polygons <= kLdsCountsMax ? ((size_t)n_polygons + 64) * 4 : 0);
                // (option raster_tb_lds 2 / 0: the tile bases of a large tile grid out of LDS, a finer
                // quad level in their place, k_join_stream_cpt gathering the tile base beside the
                // sub-block entry -- at C3 quad shift 6 -> 5, pending rows 28 % -> 18 %, but the extra
                // gathers cost more than the saved ones: stream 3.80 -> 3.87 ms)
                const size_t tbytes = tb.tile_idx.size() * 4;
                ch->tb_lds_budget = c->raster_tb_lds == 1 ? tbytes <= avail / 3 : (c->raster_tb_lds == 2 && tbytes <= avail / 16);
                if (ch->tb_lds_budget) avail -= tbytes;
                // quad level in at most half of it, quad records in the rest (option raster_quad_records)
                if (c->raster_quad_records && c->raster_quad == 1) {
                    tb.quad_max = (int)std::min<size_t>(tiles::kQuadLimit, avail / 4);
                    tb.quad_lds_bytes = avail;
                } else {
                    tb.quad_max = c->raster_quad > 1 ? c->raster_quad : (int)std::min<size_t>(tiles::kQuadLimit, avail / 2);
                    tb.quad_lds_bytes = 0;
                }
                tb.lines = c->raster_lines != 0;
                tb.leaf_lines = c->raster_leaf_lines != 0;
                bool raster_built = false;
                auto t_cls = std::chrono::steady_clock::now();
                if (tb.raster_setup(src, c->raster_sub, c->raster_cell)) {
                    tiles::Builder::RasterClass cls;
                    if (c->raster_build) {
                        if ((rc = raster_classify_gpu(c, ch, tb, cls))) {
                            ch->release_all();
                            delete ch;
                            return rc;
                        }
                    } else {
                        tb.classify_raster_host(src, threads, cls);
                    }
                    ch->build_ms[2] = ms_since(t_cls);
                    trace.mark("raster setup + classify");
                    if ((rc = upload_chip_rasters())) {
                        ch->release_all();
                        delete ch;
                        return rc;
                    }
                    auto t_asm = std::chrono::steady_clock::now();
                    raster_built = tb.assemble_raster(cls, threads);
                    ch->build_ms[3] = ms_since(t_asm);
                    defer_free(std::move(cls));
                    trace.mark("raster assemble");
                }
                if (raster_built) {
                    ch->raster_parts[0] = tb.sub.size() * 2;
                    ch->raster_parts[1] = tb.blocks.size() * 2;
                    ch->raster_parts[2] = tb.tile_base.size() * 4;
                    ch->raster_parts[3] = tb.quad.size() * 2;
                    ch->raster_parts[4] = tb.qrec_mask.size() * 4;
                    ch->raster_parts[5] = tb.qrec_code.size() * 2;
                    ch->raster_parts[6] = tb.llines.empty() ? 0 : tb.tile_lbase.size() * 4;
                    ch->raster_parts[7] = tb.llines.size() * sizeof(tiles::LineRec);
                    size_t r0 = tb.sub.size() * 2, r1 = tb.blocks.size() * 2, rm = tb.tile_base.size() * 4;
                    if ((rc = ch->rsub.reserve(r0)) || (rc = ch->rblocks.reserve(r1)) || (rc = ch->rmid.reserve(rm))) {
                        ch->release_all();
                        delete ch;
                        return rc;
                    }
                    trace.mark("  raster reserve");
                    if ((rc = h2d(c, ch->rsub.p, tb.sub.data(), r0))) return rc;
                    if ((rc = h2d(c, ch->rmid.p, tb.tile_base.data(), rm))) return rc;
                    if ((rc = h2d(c, ch->rblocks.p, tb.blocks.data(), r1))) return rc;
                    if (!tb.llines.empty()) {
                        if ((rc = ch->rlbase.reserve(ch->raster_parts[6])) || (rc = ch->rllines.reserve(ch->raster_parts[7])) ||
                            (rc = h2d(c, ch->rlbase.p, tb.tile_lbase.data(), ch->raster_parts[6])) ||
                            (rc = h2d(c, ch->rllines.p, tb.llines.data(), ch->raster_parts[7]))) {
                            ch->release_all();
                            delete ch;
                            return rc;
                        }
                        total += ch->raster_parts[6] + ch->raster_parts[7];
                    }
                    trace.mark("  raster copies (sub, blocks)");
                    total += rm;
                    ch->raster_ok = true;
                    ch->praster.sub = (const uint16_t*)ch->rsub.p;
                    ch->praster.tile_base = (const uint32_t*)ch->rmid.p;
                    ch->praster.sshift = tb.sshift;
                    ch->praster.tnx = tb.grid.nx;
                    ch->praster.blocks = (const uint16_t*)ch->rblocks.p;
                    ch->praster.tile_lbase = tb.llines.empty() ? nullptr : (const uint32_t*)ch->rlbase.p;
                    ch->praster.llines = tb.llines.empty() ? nullptr : (const tiles::LineRec*)ch->rllines.p;
                    ch->praster.sx = tb.grid.sx * tb.S;
                    ch->praster.sy = tb.grid.sy * tb.S;
                    ch->praster.nx = tb.grid.nx * tb.S;
                    ch->praster.ny = tb.grid.ny * tb.S;
                    ch->praster.C = tb.C;
                    ch->praster.cshift = tb.cshift;
                    ch->praster.quad = nullptr;
                    if (!tb.quad.empty() && c->raster_quad) {
                        size_t r2 = (tb.quad.size() + 1) / 2 * 4;  // read as uint32 words by k_join_stream
                        if ((rc = ch->rquad.reserve(r2))) {
                            ch->release_all();
                            delete ch;
                            return rc;
                        }
                        if ((rc = h2d(c, ch->rquad.p, tb.quad.data(), tb.quad.size() * 2))) return rc;
                        ch->praster.quad = (const uint16_t*)ch->rquad.p;
                        ch->praster.qnx = tb.qnx;
                        ch->praster.qny = tb.qny;
                        ch->praster.qshift = tb.qshift;
                        total += r2;
                    }
                    // k_join_stream's view of the raster (tiles::raster_code, lane-parallel)
                    const size_t nsub = (size_t)ch->praster.nx * ch->praster.ny;
                    const size_t csub_bytes = (tb.sub.size() - nsub) * 2, blocks_bytes = tb.blocks.size() * 2;
                    if (ch->praster.quad && tb.edge_ok && csub_bytes < kNoLoad && blocks_bytes < kNoLoad &&
                        rm < kNoLoad && (int64_t)ch->praster.nx * tb.C < (1 << 30) && (int64_t)ch->praster.ny * tb.C < (1 << 30)) {
                        StreamArgs& sa = ch->stream;
                        sa.x0 = tb.grid.x0;
                        sa.y0 = tb.grid.y0;
                        sa.sxC = ch->praster.sx * tb.C;
                        sa.syC = ch->praster.sy * tb.C;
                        sa.gxmax = (double)ch->praster.nx * tb.C - 1.0;
                        sa.gymax = (double)ch->praster.ny * tb.C - 1.0;
                        // fixed-point coordinates of k_join_stream_pipe (tiles::raster_code_fixed):
                        // power-of-two scalings of the same products
                        const double fs = (double)(1 << tiles::kFixBits);
                        sa.sxF = sa.sxC * fs;
                        sa.syF = sa.syC * fs;
                        sa.gx0F = (-sa.x0 * sa.sxC) * fs;
                        sa.gy0F = (-sa.y0 * sa.syC) * fs;
                        sa.fix_ok = ((int64_t)ch->praster.nx * tb.C << tiles::kFixBits) < ((int64_t)1 << 31) &&
                                    ((int64_t)ch->praster.ny * tb.C << tiles::kFixBits) < ((int64_t)1 << 31);
                        sa.gxmaxF = sa.fix_ok ? (int32_t)(((int64_t)ch->praster.nx * tb.C - 1) << tiles::kFixBits) : 0;
                        sa.gymaxF = sa.fix_ok ? (int32_t)(((int64_t)ch->praster.ny * tb.C - 1) << tiles::kFixBits) : 0;
                        sa.cs = tb.cshift;
                        sa.qs = tb.qshift;
                        sa.qsh = tb.cshift + tb.qshift;
                        sa.tsh = tb.cshift + tb.sshift;
                        sa.qnx = tb.qnx;
                        sa.tnx = tb.grid.nx;
                        sa.n_quad_words = (int32_t)((tb.quad.size() + 1) / 2);
                        sa.n_tiles = (int32_t)tb.tile_base.size();
                        sa.tb_lds = 0;
                        sa.stage_words = kStageWords;
                        sa.quad = (const uint32_t*)ch->rquad.p;
                        sa.tile_base = (const uint32_t*)ch->rmid.p;
                        sa.csub = (const uint16_t*)ch->rsub.p + nsub;
                        sa.blocks = (const uint16_t*)ch->rblocks.p;
                        sa.tile_lbase = ch->praster.tile_lbase;
                        sa.llines = ch->praster.llines;
                        sa.csub_bytes = (uint32_t)csub_bytes;
                        sa.blocks_bytes = (uint32_t)blocks_bytes;
                        sa.tile_base_bytes = (uint32_t)rm;
                        // quad records: mask words, then the codes (>= 2 words, so index 0 is readable)
                        std::vector<uint32_t> qw(tb.qrec_mask);
                        const size_t nrec = tb.qrec_code.size();
                        qw.resize(2 * nrec + (nrec + 1) / 2, 0u);
                        if (nrec) memcpy(qw.data() + 2 * nrec, tb.qrec_code.data(), nrec * 2);
                        if (qw.size() < 2) qw.resize(2, 0u);
                        if ((rc = ch->rqrec.reserve(qw.size() * 4))) {
                            ch->release_all();
                            delete ch;
                            return rc;
                        }
                        if ((rc = h2d(c, ch->rqrec.p, qw.data(), qw.size() * 4))) return rc;
                        sa.qrec = (const uint32_t*)ch->rqrec.p;
                        sa.n_qrec = (int32_t)nrec;
                        sa.n_qrec_words = (int32_t)qw.size();
                        sa.qrl = tb.qrec_shift;
                        ch->praster.qrec_mask = nrec ? (const uint32_t*)ch->rqrec.p : nullptr;
                        ch->praster.qrec_code = nrec ? (const uint16_t*)((const uint32_t*)ch->rqrec.p + 2 * nrec) : nullptr;

                        ch->praster.n_qrec = (int32_t)nrec;
                        ch->praster.qrec_shift = tb.qrec_shift;
                        ch->stream_ok = true;
                    }
                    ch->raster_stats[0] = tb.S;
                    ch->raster_stats[1] = tb.C;
                    ch->raster_stats[2] = tb.n_sub_pure;
                    ch->raster_stats[3] = tb.n_sub_mixed;
                    ch->raster_stats[4] = tb.n_cell_mixed;
                    ch->raster_stats[5] = tb.n_sub_line;
                    ch->raster_stats[6] = tb.n_cell_line;
                    total += r0 + r1;
                }
            }
        }
        // per-tile chip images for the binned join's LDS tiles (join_binned.h): tables without a
        // point raster to stream (option tile_images 1), or always (2)
        if (ch->tiles_ok && (c->tile_images == 2 || (c->tile_images == 1 && !ch->raster_ok))) {
            binned::ImageSource is;
            is.recs = tb.recs.data();
            is.n_recs = tb.recs.size();
            is.grid = tb.grid;
            is.tile_idx = tb.tile_idx.data();
            is.entries = tb.entries.data();
            std::vector<uint32_t> sfirst(capacity, 0), scount(capacity, 0);
            for (uint64_t q = 0; q < capacity; q++)
                if (table[q].key != kEmptyKey) {
                    sfirst[q] = table[q].first;
                    scount[q] = table[q].count;
                }
            is.slot_first = sfirst.data();
            is.slot_count = scount.data();
            is.meta = meta.data();
            is.store = pip::GeomStore{gb.verts.data(), gb.ring_start.data(), gb.ring_bbox.data(), gb.part_ring.data(),
                                      gb.geom_part.data(), gb.geom_bbox.data()};
            is.threads = (int)std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency()));
            binned::ImageSet iset;
            if (binned::build_tile_images(is, iset) && !iset.words.empty()) {
                const std::vector<uint32_t>* src[4] = {&iset.words, &iset.off, &iset.rec, &iset.bin_map};
                DevBuf* dst[4] = {&ch->img_words, &ch->img_off, &ch->img_rec, &ch->img_binmap};
                for (int k = 0; k < 4; k++) {
                    if ((rc = dst[k]->reserve(src[k]->size() * 4))) {
                        ch->release_all();
                        delete ch;
                        return rc;
                    }
                    if ((rc = h2d(c, dst[k]->p, src[k]->data(), src[k]->size() * 4))) return rc;
                    total += src[k]->size() * 4;
                }
                ch->img_max_words = iset.max_words;
                ch->img_count = (int64_t)iset.off.size();
                ch->img_records = (int64_t)std::count_if(iset.off.begin(), iset.off.end(),
                                                         [](uint32_t o) { return o != binned::kNoImage; });
            }
            trace.mark("tile images");
        }
        defer_free(std::move(tb));
        trace.mark("(tile builder handed off)");
    }
    trace.mark("raster uploads + stream args");
    if ((rc = upload_chip_rasters())) {
        ch->release_all();
        delete ch;
        return rc;
    }
    // the staged uploads are ordered on this thread's stream: complete before any stream joins the table
    HIP_TRY(hipStreamSynchronize(c->stream));
    trace.mark("chip rasters uploaded");
    ch->device_bytes = total + capacity * sizeof(HashEntry) + meta.size() * 4 + rb.hdr.size() * sizeof(raster::ChipHdr) +
                       rb.cells.size() * sizeof(raster::CellRec) + rb.edges.size() * sizeof(pip::Edge);
    // the host-side build arrays (chip rasters, geometry store) are released off the return path
    defer_free(std::move(rb));
    defer_free(std::move(gb));
    *out = ch;
    return MOSAIC_OK;
}

int mosaic_chip_table_destroy(mosaic_chips* ch) {
    if (!ch) return MOSAIC_OK;
    (void)hipSetDevice(ch->device);
    ch->release_all();
    delete ch;
    return MOSAIC_OK;
}

int mosaic_chip_table_info(const mosaic_chips* ch, int64_t* o) {
    if (!ch || !o) return fail(MOSAIC_E_ARG, "null argument");
    o[0] = ch->n_chips;
    o[1] = ch->n_cells;
    o[2] = ch->n_border;
    o[3] = ch->n_vertices;
    o[4] = ch->n_rings;
    o[5] = (int64_t)ch->device_bytes;
    o[6] = (int64_t)ch->capacity;
    o[7] = ch->n_polygons;
    return MOSAIC_OK;
}

int mosaic_chip_table_tiles(const mosaic_chips* ch, int64_t* o) {
    if (!ch || !o) return fail(MOSAIC_E_ARG, "null argument");
    o[0] = ch->tiles_ok ? 1 : 0;
    for (int k = 0; k < 6; k++) o[k + 1] = ch->tile_stats[k];
    if (ch->grid == MOSAIC_GRID_BNG) {  // BNG dense cell table: built, cells along e, cells along n
        o[0] = ch->bng_ok ? 1 : 0;
        o[1] = ch->bng_ne;
        o[2] = ch->bng_nn;
        o[3] = (int64_t)ch->bng_lwords * 4;  // LDS cell level: bytes, block shift
        o[4] = ch->bng_lsh;
        o[5] = ch->bng_sub_stats[0];  // mixed sub-cells, line sub-cells
        o[6] = ch->bng_sub_stats[1];
    }
    o[7] = ch->raster_ok ? 1 : 0;
    for (int k = 0; k < 5; k++) o[k + 8] = ch->raster_stats[k];
    return MOSAIC_OK;
}

int mosaic_chip_table_raster(const mosaic_chips* ch, int64_t* o) {
    if (!ch || !o) return fail(MOSAIC_E_ARG, "null argument");
    o[0] = ch->raster_stats[5];
    o[1] = ch->praster.quad ? (int64_t)ch->praster.qnx * ch->praster.qny : 0;
    o[2] = ch->praster.quad ? ch->praster.qshift : 0;
    o[3] = ch->raster_ok ? (int64_t)(ch->rsub.bytes + ch->rmid.bytes + ch->rblocks.bytes + ch->rquad.bytes + ch->rqrec.bytes +
                                     ch->rlbase.bytes + ch->rllines.bytes) : 0;
    o[4] = ch->stream_ok ? 1 : 0;
    o[5] = ch->img_records;  // binned join: LDS chip images (record parts), their bytes, the largest image
    o[6] = (int64_t)(ch->img_words.bytes + ch->img_off.bytes);
    o[7] = (int64_t)ch->img_max_words * 4;
    o[8] = ch->raster_stats[6];  // leaf lines
    return MOSAIC_OK;
}

int mosaic_chip_table_build_info(const mosaic_chips* ch, double* ms4, uint64_t* digest) {
    if (!ch || !ms4 || !digest) return fail(MOSAIC_E_ARG, "null argument");
    for (int k = 0; k < 4; k++) ms4[k] = ch->build_ms[k];
    *digest = 0;
    if (!ch->raster_ok) return MOSAIC_OK;
    if (!ch->raster_digest) {
        // FNV-1a over the raster arrays as uploaded (sub-block table, blocks, tile bases, quad level,
        // quad-record masks and codes): read back from the device on request, off the build's path
        HIP_TRY(hipSetDevice(ch->device));
        const void* src[8] = {ch->rsub.p, ch->rblocks.p, ch->rmid.p, ch->rquad.p, ch->rqrec.p,
                              ch->rqrec.p ? (const void*)((const uint8_t*)ch->rqrec.p + ch->raster_parts[4]) : nullptr,
                              ch->rlbase.p, ch->rllines.p};
        uint64_t h = 1469598103934665603ull;
        std::vector<uint8_t> buf;
        for (int k = 0; k < 8; k++) {
            buf.resize(src[k] ? ch->raster_parts[k] : 0);  // (parts not uploaded: quad level or records off)
            if (!buf.empty()) HIP_TRY(hipMemcpy(buf.data(), src[k], buf.size(), hipMemcpyDeviceToHost));
            h = fnv1a(h, buf.data(), buf.size());
        }
        const_cast<mosaic_chips*>(ch)->raster_digest = h;
    }
    *digest = ch->raster_digest;
    return MOSAIC_OK;
}

int mosaic_chip_table_tile_grid(const mosaic_chips* ch, double* o) {
    if (!ch || !o) return fail(MOSAIC_E_ARG, "null argument");
    o[0] = ch->tgrid.x0;
    o[1] = ch->tgrid.y0;
    o[2] = ch->tgrid.sx;
    o[3] = ch->tgrid.sy;
    return MOSAIC_OK;
}


static int run_join(ThreadCtx* c, const mosaic_chips* ch, const double* x, const double* y, int64_t n,
                    int64_t* counts, int64_t* out_row, int32_t* out_key, int64_t cap, int64_t* n_out) {
    bool pairs = out_row != nullptr;
    if (!c || !ch) return fail(MOSAIC_E_ARG, "null context or chip table");
    if (n < 0) return fail(MOSAIC_E_ARG, "negative n");
    if (n > 0 && (!x || !y)) return fail(MOSAIC_E_ARG, "null coordinates");
    if (!pairs && !counts && ch->n_polygons > 0) return fail(MOSAIC_E_ARG, "null counts");
    if (ch->device != c->device) return fail(MOSAIC_E_ARG, "chip table belongs to another device");
    HIP_TRY(hipSetDevice(c->device));
    int rc;
    const void *dx, *dy;
    if ((rc = to_device(c, c->stage_x, x, n * 8, &dx))) return rc;
    if ((rc = to_device(c, c->stage_y, y, n * 8, &dy))) return rc;
    bool dev_counts = counts && is_device_ptr(counts);
    size_t cbytes = (size_t)std::max<int32_t>(ch->n_polygons, 1) * 8;
    if (!dev_counts && (rc = c->stage_out.reserve(cbytes))) return rc;
    unsigned long long* dcounts = dev_counts ? (unsigned long long*)counts : (unsigned long long*)c->stage_out.p;
    {
        const int64_t nz = (int64_t)(cbytes / 8) + kScalars;
        hipLaunchKernelGGL(k_zero_join, dim3((unsigned)std::min<int64_t>((nz + 255) / 256, 1024)), dim3(256), 0, c->stream,
                           (unsigned long long*)dcounts, (int64_t)(cbytes / 8), (unsigned long long*)c->scalars.p);
        HIP_TRY(hipGetLastError());
    }
    uint64_t qcap = (uint64_t)std::max<int64_t>(std::min<int64_t>(n, std::max<int64_t>(n / 8, 1 << 20)), 1);
    if (c->exact_cap > 0) qcap = (uint64_t)c->exact_cap;
    c->last_qcap = qcap;
    if ((rc = c->amb_queue.reserve(qcap * 8))) return rc;
    bool dev_pairs = pairs && is_device_ptr(out_row) && is_device_ptr(out_key);
    if (pairs && !dev_pairs) {
        if ((rc = c->stage_idx.reserve((size_t)std::max<int64_t>(cap, 1) * 8))) return rc;
        if ((rc = c->stage_out2.reserve((size_t)std::max<int64_t>(cap, 1) * 4))) return rc;
    }
    unsigned long long* sc = (unsigned long long*)c->scalars.p;
    c->binned_rows = 0;
    JoinArgs a;
    a.x = (const double*)dx;
    a.y = (const double*)dy;
    a.valid = nullptr;
    a.n = n;
    a.res = ch->res;
    a.jdk = c->jdk;
    a.table = (const HashEntry*)ch->table.p;
    a.mask = ch->capacity - 1;
    a.chip_meta = (const uint32_t*)ch->meta.p;
    a.hdr = (const raster::ChipHdr*)ch->hdr.p;
    a.cells = (const raster::CellRec*)ch->cells.p;
    a.rast_edges = (const pip::Edge*)ch->rast_edges.p;
    a.lane_edges = (uint32_t)c->lane_edges;
    a.store = ch->store.view();
    a.tgrid = ch->tgrid;
    a.tile_idx = (const uint32_t*)ch->tile_idx.p;
    a.tile_rec = (const tiles::TileRec*)ch->tile_rec.p;
    a.tile_ent = (const uint32_t*)ch->tile_ent.p;
    a.praster = ch->praster;
    a.row_lo = 0;
    a.bng_cells = nullptr;
    a.bng_leaf = nullptr;
    a.bng_e0 = a.bng_n0 = a.bng_ne = a.bng_nn = 0;
    a.bng_div = 1;
    a.bng_C = 1;
    a.mixq = nullptr;
    a.mixq_count = sc + 4;
    a.counts = dcounts;
    a.n_polygons = ch->n_polygons;
    a.amb_queue = (unsigned long long*)c->amb_queue.p;
    a.amb_count = sc + 0;
    a.amb_cap = qcap;
    a.pair_row = pairs ? (long long*)(dev_pairs ? (void*)out_row : c->stage_idx.p) : nullptr;
    a.pair_key = pairs ? (int*)(dev_pairs ? (void*)out_key : c->stage_out2.p) : nullptr;
    a.pair_count = sc + 1;
    a.pair_cap = cap;
    a.tests = sc + 2;
    a.flags = (unsigned int*)(sc + 3);
    a.cstride = 1;
    a.rowmap = nullptr;
    bool lds = ch->n_polygons <= kLdsCountsMax;
    size_t shm = lds ? (size_t)ch->n_polygons * 4 : 0;
    int g = grid_size(c, n);
    bool binned_used = false, exact_inline = false;
    if (n > 0) {
        hipEvent_t tstop;
        if ((rc = timing_begin(c, &tstop))) return rc;
        const bool h3g = ch->grid == MOSAIC_GRID_H3;
#define MOSAIC_LAUNCH(KERNEL, SHM) hipLaunchKernelGGL(KERNEL, dim3(g), dim3(c->block), SHM, c->stream, a)
        const bool tiled = h3g && c->tiles && ch->tiles_ok;
        const bool praster = tiled && c->point_raster && ch->raster_ok;
        const bool bngdense = !h3g && c->tiles && ch->bng_ok;
        // k_join_stream's LDS: [counts + 64 spill words] [per-wave stages] [tile_base if it fits] [quad]
        StreamArgs sa = ch->stream;
        const int blk = c->stream_block;
        size_t shm_s = (lds && !pairs ? ((size_t)ch->n_polygons + 64) * 4 : 0) + (size_t)(blk / 64) * sa.stage_words * 4 +
                       (size_t)sa.n_quad_words * 4 + (size_t)sa.n_qrec_words * 4;
        sa.tb_lds = ch->tb_lds_budget && shm_s + (size_t)sa.n_tiles * 4 <= kStreamLdsMax ? 1 : 0;
        if (sa.tb_lds) shm_s += (size_t)sa.n_tiles * 4;
        const bool stream = praster && ch->stream_ok && shm_s <= kStreamLdsMax;
        // border-chip-heavy tables (no point raster to stream): points binned by tile first
        binned_used = tiled && !stream && c->bin_points && n >= c->bin_min_rows;
        if (bngdense) {
            a.bng_cells = (const uint32_t*)ch->bng_cells.p;
            a.bng_e0 = ch->bng_e0;
            a.bng_n0 = ch->bng_n0;
            a.bng_ne = ch->bng_ne;
            a.bng_nn = ch->bng_nn;
            a.bng_div = ch->bng_div;
            a.bng_leaf = (const uint16_t*)ch->bng_leaf.p;
            a.bng_C = ch->bng_C;
            a.bng_wedge = ch->bng_C > 0 && ch->bng_wedges ? 1 : 0;
            BngStreamArgs bs;
            bs.e0 = ch->bng_e0;
            bs.n0 = ch->bng_n0;
            bs.ne = ch->bng_ne;
            bs.nn = ch->bng_nn;
            bs.C = ch->bng_C;
            bs.div = (double)ch->bng_div;
            bs.inv_div = 1.0 / (double)ch->bng_div;
            bs.f = (double)ch->bng_C / (double)ch->bng_div;
            bs.idiv = ch->bng_div;
            bs.ff = (float)bs.f;
            bs.cells = (const uint32_t*)ch->bng_cells.p;
            bs.leaf = (const uint16_t*)ch->bng_leaf.p;
            bs.cells_bytes = (uint32_t)((size_t)ch->bng_ne * ch->bng_nn * 4);
            bs.leaf_bytes = (uint32_t)std::min<size_t>(ch->bng_leaf_bytes, kNoLoad);
            bs.lvl = (const uint16_t*)ch->bng_lvl.p;
            bs.lvl_bytes = (uint32_t)ch->bng_lvl_bytes;
            bs.lvl_stride = tiles::bng_level_stride(ch->bng_C);
            bs.lvl_cb = tiles::bng_level_side(ch->bng_C);
            const int64_t chunk = ((int64_t)1 << 32) - 256;
            const int64_t rows = std::min<int64_t>(n, chunk);
            if ((rc = c->mix_queue.reserve((size_t)rows * 4 + 16))) return rc;
            a.mixq = (uint32_t*)c->mix_queue.p;
            const bool aligned = (((uintptr_t)dx | (uintptr_t)dy) & 15) == 0;
            const int blkb = c->stream_block;
            size_t shm_b = (lds && !pairs ? ((size_t)ch->n_polygons + 64) * 4 : 0) + (size_t)(blkb / 64) * kStageWords * 4;
            // the LDS cell level when it fits this launch's LDS
            bs.lcell = (const uint32_t*)ch->bng_lcell.p;
            bs.lsh = ch->bng_lsh;
            bs.lnx = ch->bng_lnx;
            bs.lcell_words = shm_b + (size_t)ch->bng_lwords * 4 <= kStreamLdsMax ? ch->bng_lwords : 0;
            shm_b += (size_t)bs.lcell_words * 4;
            // k_join_stream_bng_cpt (option bng_cpt): with the LDS cell level, a 24-bit cell index and
            // room for its per-wave compaction buffers
            const size_t cpt_bytes = (size_t)(blkb / 64) * kCptBufWords * 4;
            const bool bcpt = c->bng_cpt && aligned && bs.lcell_words > 0 && ch->bng_cpt_ok &&
                              (int64_t)ch->bng_ne * ch->bng_nn < ((int64_t)1 << 24) && shm_b + cpt_bytes <= kStreamLdsMax;
            if (bcpt) shm_b += cpt_bytes;
            auto kernel_for = [&](bool vec) -> const void* {
                return stream_kernel_bng(lds, pairs, vec, bcpt);
            };
            c->last_kernel = bcpt ? "k_join_stream_bng_cpt" : "k_join_stream_bng";
            int per_cu = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel_for(true), blkb, shm_b) != hipSuccess || per_cu < 1)
                per_cu = 1;
            for (int64_t lo = 0; lo < n; lo += chunk) {
                JoinArgs ac = a;
                ac.row_lo = lo;
                ac.n = std::min<int64_t>(n, lo + chunk);
                if (lo > 0) HIP_TRY(hipMemsetAsync(ac.mixq_count, 0, 8, c->stream));
                const void* kfn = kernel_for(aligned && ac.n - lo >= 256);
                const int gs = (int)std::max<int64_t>(1, std::min<int64_t>((ac.n - lo + 4 * blkb - 1) / (4 * blkb),
                                                                           (int64_t)c->n_cu * per_cu));
                void* kargs[] = {&ac, &bs};
                HIP_TRY(hipLaunchKernel(kfn, dim3(gs), dim3(blkb), kargs, shm_b, c->stream));
                if (tstop && lo == 0) HIP_TRY(hipEventRecord(tstop, c->stream));
                const int gm = (int)std::max<int64_t>(1, std::min<int64_t>((ac.n - lo + 4 * c->block - 1) / (4 * c->block),
                                                                           (int64_t)c->n_cu * c->mixed_blocks_per_cu));
#define MOSAIC_MIXED_BNG(R_)                                                                                     \
    do {                                                                                                         \
        if (pairs) hipLaunchKernelGGL((k_join_mixed_bng<false, true, R_>), dim3(gm), dim3(c->block), 0, c->stream, ac); \
        else if (lds) hipLaunchKernelGGL((k_join_mixed_bng<true, false, R_>), dim3(gm), dim3(c->block), shm, c->stream, ac); \
        else hipLaunchKernelGGL((k_join_mixed_bng<false, false, R_>), dim3(gm), dim3(c->block), 0, c->stream, ac); \
    } while (0)
                hipEvent_t mstop = nullptr;  // option timing = 2: the mixed kernel is timed too
                if (c->timing == 2 && lo == 0 && (rc = timing_begin(c, &mstop))) return rc;
                if (c->mixed_rows == 4) MOSAIC_MIXED_BNG(4);
                else if (c->mixed_rows == 2) MOSAIC_MIXED_BNG(2);
                else MOSAIC_MIXED_BNG(1);
#undef MOSAIC_MIXED_BNG
                if (mstop) HIP_TRY(hipEventRecord(mstop, c->stream));
                HIP_TRY(hipGetLastError());
            }
            tstop = nullptr;
        } else if (stream) {
            // k_join_stream + k_join_mixed over rows in chunks of < 2^32 (uint32 queue entries)
            const int64_t chunk = ((int64_t)1 << 32) - 256;  // multiple of 256: chunk starts stay aligned
            const int64_t rows = std::min<int64_t>(n, chunk);
            if ((rc = c->mix_queue.reserve((size_t)rows * 4 + 16))) return rc;
            a.mixq = (uint32_t*)c->mix_queue.p;
            a.mixq_count = sc + 4;
            // k_join_leaf between the stream and mixed kernels: tables with leaf lines, fixed-point
            // coordinates (tiles::raster_code_fixed's chain)
            const bool leafq = c->leaf_join && sa.llines && sa.fix_ok;
            if (leafq && (rc = c->mix_queue2.reserve((size_t)rows * 4 + 16))) return rc;
            // the mixed kernel answers its uncertified rows itself: no exact pass after it (option
            // exact_defer: it queues them for k_join_h3_exact instead)
            a.exact_inline = c->exact_defer ? 0 : 1;
            exact_inline = !c->exact_defer;
            const bool aligned = (((uintptr_t)dx | (uintptr_t)dy) & 15) == 0;
            auto mode_for = [&](bool vec) -> int {
                // the pipelined forms where they apply (the compacted one, k_join_stream_cpt, carries
                // cs + kFixBits + qs <= 24 low bits of the fine-cell coordinates and a 16-bit tile index
                // per pending row, and per wave a kCptBufWords compaction buffer in LDS)
                // (k_join_stream_pipe reads tile bases from LDS; k_join_stream_cpt from LDS or memory)
                int mode = vec && sa.fix_ok ? c->stream_pipe : 0;
                if (mode >= 2 && !(sa.cs + tiles::kFixBits + sa.qs <= 24 && sa.tsh + tiles::kFixBits <= 24 && sa.n_tiles <= 65536 &&
                                   shm_s + (size_t)(blk / 64) * kCptBufWords * 4 <= kStreamLdsMax))
                    mode = 1;
                if (mode == 1 && !sa.tb_lds) mode = 0;
                return mode;
            };
            auto kernel_for = [&](bool vec) -> const void* { return stream_kernel_h3(mode_for(vec), lds, pairs, vec); };
            auto shm_for = [&](bool vec) -> size_t {
                return shm_s + (mode_for(vec) >= 2 ? (size_t)(blk / 64) * kCptBufWords * 4 : 0);
            };
            int per_cu = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel_for(true), blk, shm_for(true)) != hipSuccess ||
                per_cu < 1)
                per_cu = 1;
            for (int64_t lo = 0; lo < n; lo += chunk) {
                JoinArgs ac = a;
                ac.row_lo = lo;
                ac.n = std::min<int64_t>(n, lo + chunk);
                // 16-byte loads need aligned columns and >= 256 rows (the prefetch past the end
                // re-reads the chunk's first 256)
                const void* kfn = kernel_for(aligned && ac.n - lo >= 256);
                const int mode = mode_for(aligned && ac.n - lo >= 256);
                if (lo == 0) {
                    static const char* const names[3] = {"k_join_stream", "k_join_stream_pipe", "k_join_stream_cpt"};
                    c->last_kernel = names[mode];
                }
                if (lo > 0) HIP_TRY(hipMemsetAsync(ac.mixq_count, 0, 8, c->stream));
                // persistent grid: the workgroups resident at once (each fills its LDS once)
                const int gs = (int)std::max<int64_t>(1, std::min<int64_t>((ac.n - lo + 4 * blk - 1) / (4 * blk),
                                                                           (int64_t)c->n_cu * per_cu));
                void* kargs[] = {&ac, &sa};
                HIP_TRY(hipLaunchKernel(kfn, dim3(gs), dim3(blk), kargs, shm_for(aligned && ac.n - lo >= 256), c->stream));
                if (tstop && lo == 0) HIP_TRY(hipEventRecord(tstop, c->stream));
                // (the queue holds at most the chunk's rows)
                const int gm = (int)std::max<int64_t>(1, std::min<int64_t>((ac.n - lo + 4 * c->block - 1) / (4 * c->block),
                                                                           (int64_t)c->n_cu * c->mixed_blocks_per_cu));
#define MOSAIC_MIXED(KERNEL, SHM) \
    hipLaunchKernelGGL(KERNEL, dim3(gm), dim3(c->block), SHM, c->stream, ac)
                hipEvent_t mstop = nullptr;  // option timing = 2: the mixed kernel is timed too
                if (c->timing == 2 && lo == 0 && (rc = timing_begin(c, &mstop))) return rc;
                const int lb = leafq ? std::max(1, c->n_cu * c->leaf_blocks_per_cu) : 0;
                if (leafq) {
                    uint32_t* q2 = (uint32_t*)c->mix_queue2.p;
                    unsigned long long* q2c = sc + 7;
                    // (k_zero_join cleared it for the first chunk: no fill dispatch between the stream and
                    // leaf kernels)
                    if (lo > 0) HIP_TRY(hipMemsetAsync(q2c, 0, 8, c->stream));
                    void* largs[] = {&ac, &sa, &q2, &q2c};
                    HIP_TRY(hipLaunchKernel(leaf_kernel(lds, pairs), dim3((unsigned)lb), dim3(256), largs,
                                            (lds && !pairs ? shm : 0) + 4 * kStageWords * 4, c->stream));
                    ac.mixq = q2;
                    ac.mixq_count = q2c;
                }
                if (c->mixed_rows == 4) {
                    if (pairs) MOSAIC_MIXED((k_join_mixed<false, true, 4>), 0);
                    else if (lds) MOSAIC_MIXED((k_join_mixed<true, false, 4>), shm);
                    else MOSAIC_MIXED((k_join_mixed<false, false, 4>), 0);
                } else if (c->mixed_rows == 2) {
                    if (pairs) MOSAIC_MIXED((k_join_mixed<false, true, 2>), 0);
                    else if (lds) MOSAIC_MIXED((k_join_mixed<true, false, 2>), shm);
                    else MOSAIC_MIXED((k_join_mixed<false, false, 2>), 0);
                } else {
                    if (pairs) MOSAIC_MIXED((k_join_mixed<false, true, 1>), 0);
                    else if (lds) MOSAIC_MIXED((k_join_mixed<true, false, 1>), shm);
                    else MOSAIC_MIXED((k_join_mixed<false, false, 1>), 0);
                }
#undef MOSAIC_MIXED
                HIP_TRY(hipGetLastError());
                if (mstop) HIP_TRY(hipEventRecord(mstop, c->stream));
            }
            tstop = nullptr;  // recorded after the first stream launch
        } else if (binned_used) {
            // (k_join_tiles packs a chip index and a lane into 32 bits)
            const bool use_img = c->tile_images && ch->img_words.p && ch->n_chips < ((int64_t)1 << 26);
            c->last_kernel = use_img ? "k_join_tiles" : "k_join_binned";
            const uint32_t max_code = (uint32_t)ch->tile_stats[2] + 1u;
            for (int64_t lo = 0; lo < n; lo += c->bin_chunk) {
                const int64_t hi = std::min<int64_t>(n, lo + c->bin_chunk);
                binned::Images img;
                if (use_img) {
                    img.words = (const uint32_t*)ch->img_words.p;
                    img.off = (const uint32_t*)ch->img_off.p;
                    img.rec = (const uint32_t*)ch->img_rec.p;
                    img.bin_map = (const uint32_t*)ch->img_binmap.p;
                    img.max_words = ch->img_max_words;
                    img.n_images = (uint32_t)ch->img_count;
                }
                c->bins.spin_cap = c->bin_spin_cap;
                hipError_t e = binned::join(a, lo, hi, max_code, lds && !pairs, c->n_cu, img, c->bins, c->stream);
                if (e == hipErrorOutOfMemory) return fail(MOSAIC_E_NOMEM, "binned join: device allocation failed");
                if (e != hipSuccess) return fail(MOSAIC_E_HIP, std::string("binned join: ") + hipGetErrorString(e));
                c->binned_rows += c->bins.sorted_rows;
                // this chunk's exact-H3 rows, before the next chunk reuses the sorted buffers
                const int ge = std::min(grid_size(c, (int64_t)qcap), std::max(1, c->n_cu * 2));
                if (pairs)
                    hipLaunchKernelGGL((k_join_h3_exact<true>), dim3(ge), dim3(c->block), 0, c->stream, c->bins.exact_args, 0);
                else
                    hipLaunchKernelGGL((k_join_h3_exact<false>), dim3(ge), dim3(c->block), 0, c->stream, c->bins.exact_args, 0);
                hipLaunchKernelGGL(k_amb_roll, dim3(1), dim3(1), 0, c->stream, sc, (unsigned long long)qcap);
                HIP_TRY(hipGetLastError());
            }
            hipLaunchKernelGGL(k_amb_final, dim3(1), dim3(1), 0, c->stream, sc, (unsigned long long)qcap);
            HIP_TRY(hipGetLastError());
        } else if (tiled) {
            c->last_kernel = "k_join_tiled";
            if (pairs) MOSAIC_LAUNCH((k_join_tiled<false, true>), 0);
            else if (lds) MOSAIC_LAUNCH((k_join_tiled<true, false>), shm);
            else MOSAIC_LAUNCH((k_join_tiled<false, false>), 0);
        } else if (h3g) {
            c->last_kernel = "k_join_raster";
            if (pairs) MOSAIC_LAUNCH((k_join_raster<MOSAIC_GRID_H3, false, true>), 0);
            else if (lds) MOSAIC_LAUNCH((k_join_raster<MOSAIC_GRID_H3, true, false>), shm);
            else MOSAIC_LAUNCH((k_join_raster<MOSAIC_GRID_H3, false, false>), 0);
        } else {
            c->last_kernel = "k_join_raster";
            if (pairs) MOSAIC_LAUNCH((k_join_raster<MOSAIC_GRID_BNG, false, true>), 0);
            else if (lds) MOSAIC_LAUNCH((k_join_raster<MOSAIC_GRID_BNG, true, false>), shm);
            else MOSAIC_LAUNCH((k_join_raster<MOSAIC_GRID_BNG, false, false>), 0);
        }
#undef MOSAIC_LAUNCH
        HIP_TRY(hipGetLastError());
        if (tstop) HIP_TRY(hipEventRecord(tstop, c->stream));
        if (h3g && !binned_used && !exact_inline) {
            // the margin queue is nearly always a handful of rows: a grid of 2 workgroups per CU keeps
            // the launch short (a 2048-workgroup grid cost ~40 us of dispatch for ~1 row)
            int ge = std::min(grid_size(c, (int64_t)qcap), std::max(1, c->n_cu * 2));
            if (pairs)
                hipLaunchKernelGGL((k_join_h3_exact<true>), dim3(ge), dim3(c->block), 0, c->stream, a, 0);
            else
                hipLaunchKernelGGL((k_join_h3_exact<false>), dim3(ge), dim3(c->block), 0, c->stream, a, 0);
            HIP_TRY(hipGetLastError());
        }
    }
    if (c->async && !pairs && dev_counts) return MOSAIC_OK;
    HIP_TRY(hipStreamSynchronize(c->stream));
    unsigned long long s[kScalars];
    HIP_TRY(hipMemcpy(s, c->scalars.p, sizeof s, hipMemcpyDeviceToHost));
    if (ch->grid == MOSAIC_GRID_H3 && s[0] > qcap && !exact_inline) {
        // queue overflow (adversarial input): recompute the whole batch on the exact path
        HIP_TRY(hipMemsetAsync(dcounts, 0, cbytes, c->stream));
        HIP_TRY(hipMemsetAsync(sc + 1, 0, 2 * 8, c->stream));
        if (pairs)
            hipLaunchKernelGGL((k_join_h3_exact<true>), dim3(g), dim3(c->block), 0, c->stream, a, 1);
        else
            hipLaunchKernelGGL((k_join_h3_exact<false>), dim3(g), dim3(c->block), 0, c->stream, a, 1);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipStreamSynchronize(c->stream));
        HIP_TRY(hipMemcpy(s + 1, sc + 1, 2 * 8, hipMemcpyDeviceToHost));
    }
    c->stats[0] = (int64_t)s[0];
    c->stats[1] = (int64_t)s[2];
    c->stats[2] = (int64_t)s[1];
    if (s[3] & 1u) return fail(MOSAIC_E_NAN, "NaN coordinates are not supported.");
    if (counts && !dev_counts) HIP_TRY(hipMemcpy(counts, dcounts, (size_t)ch->n_polygons * 8, hipMemcpyDeviceToHost));
    if (pairs) {
        *n_out = (int64_t)s[1];
        if ((int64_t)s[1] > cap) return fail(MOSAIC_E_CAPACITY, "pair buffer too small");
        if (!dev_pairs && s[1] > 0) {
            HIP_TRY(hipMemcpy(out_row, c->stage_idx.p, s[1] * 8, hipMemcpyDeviceToHost));
            HIP_TRY(hipMemcpy(out_key, c->stage_out2.p, s[1] * 4, hipMemcpyDeviceToHost));
        }
    }
    return MOSAIC_OK;
}

// Host-resident coordinates: the batch is joined in chunks of host_chunk rows.  Chunk i's join
// runs (asynchronously, counts on the device) while chunk i + 1 is copied on copy_stream into the
// other pair of device buffers; then chunk i is finished exactly as a synchronous call would be
// (NaN -> MOSAIC_E_NAN; an exact-path queue overflow reruns the chunk synchronously) and its counts
// are added on the host.  The PCIe copy and the join overlap instead of adding.
static int join_count_host_chunked(ThreadCtx* c, const mosaic_chips* ch, const double* x, const double* y, int64_t n,
                                   int64_t* counts) {
    HIP_TRY(hipSetDevice(c->device));
    const int64_t CH = c->host_chunk;
    int rc;
    for (int b = 0; b < 2; b++)
        if ((rc = c->hx[b].reserve((size_t)CH * 8)) || (rc = c->hy[b].reserve((size_t)CH * 8))) return rc;
    const int32_t np = std::max<int32_t>(ch->n_polygons, 1);
    if ((rc = c->hcounts.reserve((size_t)np * 8))) return rc;
    if (!c->copy_stream) HIP_TRY(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    std::vector<int64_t> total((size_t)np, 0), part((size_t)np, 0);
    int64_t st0 = 0, st1 = 0;
    const int64_t nch = (n + CH - 1) / CH;
    auto copy = [&](int64_t i) -> int {
        const int64_t lo = i * CH, m = std::min(CH, n - lo);
        HIP_TRY(hipMemcpyAsync(c->hx[i & 1].p, x + lo, (size_t)m * 8, hipMemcpyHostToDevice, c->copy_stream));
        HIP_TRY(hipMemcpyAsync(c->hy[i & 1].p, y + lo, (size_t)m * 8, hipMemcpyHostToDevice, c->copy_stream));
        return MOSAIC_OK;
    };
    if ((rc = copy(0))) return rc;
    HIP_TRY(hipStreamSynchronize(c->copy_stream));
    const int saved_async = c->async;
    for (int64_t i = 0; i < nch; i++) {
        const int64_t m = std::min(CH, n - i * CH);
        const double* dx = (const double*)c->hx[i & 1].p;
        const double* dy = (const double*)c->hy[i & 1].p;
        c->async = 1;
        rc = run_join(c, ch, dx, dy, m, (int64_t*)c->hcounts.p, nullptr, nullptr, 0, nullptr);
        c->async = saved_async;
        if (rc) return rc;
        if (i + 1 < nch && (rc = copy(i + 1))) return rc;
        rc = sync_impl(c);
        if (rc == MOSAIC_E_CAPACITY) {
            c->async = 0;
            rc = run_join(c, ch, dx, dy, m, (int64_t*)c->hcounts.p, nullptr, nullptr, 0, nullptr);
            c->async = saved_async;
            if (rc) return rc;
        } else if (rc) {
            HIP_TRY(hipStreamSynchronize(c->copy_stream));
            return rc;
        } else {
            unsigned long long s[kScalars];
            HIP_TRY(hipMemcpy(s, c->scalars.p, sizeof s, hipMemcpyDeviceToHost));
            c->stats[0] = (int64_t)s[0];
            c->stats[1] = (int64_t)s[2];
        }
        st0 += c->stats[0];
        st1 += c->stats[1];
        HIP_TRY(hipMemcpy(part.data(), c->hcounts.p, (size_t)np * 8, hipMemcpyDeviceToHost));
        for (int32_t k = 0; k < np; k++) total[(size_t)k] += part[(size_t)k];
        HIP_TRY(hipStreamSynchronize(c->copy_stream));
    }
    c->stats[0] = st0;
    c->stats[1] = st1;
    c->stats[2] = 0;
    if (ch->n_polygons > 0) memcpy(counts, total.data(), (size_t)ch->n_polygons * 8);
    return MOSAIC_OK;
}

int mosaic_pip_join_count(mosaic_ctx* ctx, const mosaic_chips* ch, const double* x, const double* y, int64_t n,
                          int64_t* counts) {
    ENTER(ctx);
    if (c && ch && x && y && counts && c->host_chunk > 0 && n > c->host_chunk && ch->device == c->device &&
        !is_device_ptr(x) && !is_device_ptr(y) && !is_device_ptr(counts))
        return join_count_host_chunked(c, ch, x, y, n, counts);
    return run_join(c, ch, x, y, n, counts, nullptr, nullptr, 0, nullptr);
}

int mosaic_pip_join_pairs(mosaic_ctx* ctx, const mosaic_chips* ch, const double* x, const double* y, int64_t n,
                          int64_t* out_row, int32_t* out_key, int64_t cap, int64_t* n_out) {
    ENTER(ctx);
    if (!out_row || !out_key || !n_out || cap < 0) return fail(MOSAIC_E_ARG, "null pair output");
    return run_join(c, ch, x, y, n, nullptr, out_row, out_key, cap, n_out);
}

int mosaic_st_contains(mosaic_ctx* ctx, int64_t n_geoms, const int64_t* wkb_offsets, const uint8_t* wkb,
                       const int32_t* geom_index, const double* px, const double* py, int64_t n, uint8_t* out) {
    ENTER(ctx);
    if (!c || n < 0 || n_geoms < 0 || (n_geoms > 0 && !wkb_offsets) || (n > 0 && (!geom_index || !px || !py || !out)))
        return fail(MOSAIC_E_ARG, "invalid argument");
    HIP_TRY(hipSetDevice(c->device));
    GeomBuilder gb;
    for (int64_t g = 0; g < n_geoms; g++) {
        int64_t a = wkb_offsets[g], b = wkb_offsets[g + 1];
        if (b < a || (b > a && !wkb)) return fail(MOSAIC_E_ARG, "bad wkb offsets");
        if (!gb.add(wkb + a, (size_t)(b - a))) return fail(MOSAIC_E_WKB, "geometry " + std::to_string(g) + ": " + gb.error);
    }
    if (n == 0) return MOSAIC_OK;
    GeomStoreDev st;
    size_t total = 0;
    int rc = st.upload(gb, c, &total);
    if (rc) {
        st.release();
        return rc;
    }
    const void *dpx, *dpy, *dgi;
    if ((rc = to_device(c, c->stage_x, px, n * 8, &dpx)) || (rc = to_device(c, c->stage_y, py, n * 8, &dpy)) ||
        (rc = to_device(c, c->stage_idx, geom_index, n * 4, &dgi))) {
        st.release();
        return rc;
    }
    bool dev_out = is_device_ptr(out);
    if (!dev_out && (rc = c->stage_out.reserve(n))) {
        st.release();
        return rc;
    }
    ContainsArgs a;
    a.store = st.view();
    a.n_geoms = n_geoms;
    a.geom_index = (const int*)dgi;
    a.px = (const double*)dpx;
    a.py = (const double*)dpy;
    a.n = n;
    a.out = dev_out ? out : (uint8_t*)c->stage_out.p;
    hipLaunchKernelGGL(k_st_contains, dim3(grid_size(c, n)), dim3(c->block), 0, c->stream, a);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess && !dev_out) e = hipMemcpy(out, a.out, n, hipMemcpyDeviceToHost);
    st.release();
    if (e != hipSuccess) return fail(MOSAIC_E_HIP, std::string("st_contains: ") + hipGetErrorString(e));
    return MOSAIC_OK;
}


int mosaic_intersects_aggregate(mosaic_ctx* ctx, const mosaic_chips* left, const mosaic_chips* right,
                                int32_t* out_left_key, int32_t* out_right_key, uint8_t* out_flag, int64_t cap,
                                int64_t* n_out) {
    ENTER(ctx);
    if (!c || !left || !right || !n_out || cap < 0 || (cap > 0 && (!out_left_key || !out_right_key || !out_flag)))
        return fail(MOSAIC_E_ARG, "invalid argument");
    if (left->grid != right->grid || left->res != right->res)
        return fail(MOSAIC_E_ARG, "st_intersects_aggregate: both chip tables must use the same grid and resolution");
    *n_out = 0;
    HIP_TRY(hipSetDevice(c->device));
    if (left->n_chips == 0 || right->n_chips == 0) return MOSAIC_OK;
    IsectArgs a;
    a.ta = (const HashEntry*)left->table.p;
    a.capa = left->capacity;
    a.meta_a = (const uint32_t*)left->meta.p;
    a.sa = left->store.view();
    a.tb = (const HashEntry*)right->table.p;
    a.maskb = right->capacity - 1;
    a.meta_b = (const uint32_t*)right->meta.p;
    a.sb = right->store.view();
    // pass 0: chip pairs (an upper bound on the groups) size the group hash
    DevBuf cnt, gkey, gflag, ovf;
    auto done = [&](int rc) {
        for (DevBuf* b : {&cnt, &gkey, &gflag, &ovf}) b->release();
        return rc;
    };
    int rc;
    if ((rc = cnt.reserve(8)) || (rc = ovf.reserve(4))) return done(rc);
    HIP_TRY(hipMemsetAsync(cnt.p, 0, 8, c->stream));
    HIP_TRY(hipMemsetAsync(ovf.p, 0, 4, c->stream));
    a.pass = 0;
    a.pair_count = (unsigned long long*)cnt.p;
    a.gkey = nullptr;
    a.gflag = nullptr;
    a.gmask = 0;
    a.overflow = (int*)ovf.p;
    const int64_t waves = (int64_t)left->capacity;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((waves * 64 + 255) / 256, (int64_t)c->n_cu * 16));
    hipLaunchKernelGGL(k_isect_agg, dim3(grid), dim3(256), 0, c->stream, a);
    HIP_TRY(hipGetLastError());
    unsigned long long pairs = 0;
    HIP_TRY(hipMemcpyAsync(&pairs, cnt.p, 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (pairs == 0) return done(MOSAIC_OK);
    uint64_t gcap = 1024;
    while (gcap < 2 * pairs) gcap <<= 1;
    if ((rc = gkey.reserve(gcap * 8)) || (rc = gflag.reserve(gcap * 4))) return done(rc);
    HIP_TRY(hipMemsetAsync(gkey.p, 0xff, gcap * 8, c->stream));
    HIP_TRY(hipMemsetAsync(gflag.p, 0, gcap * 4, c->stream));
    a.pass = 1;
    a.gkey = (unsigned long long*)gkey.p;
    a.gflag = (uint32_t*)gflag.p;
    a.gmask = gcap - 1;
    hipLaunchKernelGGL(k_isect_agg, dim3(grid), dim3(256), 0, c->stream, a);
    HIP_TRY(hipGetLastError());
    std::vector<unsigned long long> hk(gcap);
    std::vector<uint32_t> hf(gcap);
    int hov = 0;
    HIP_TRY(hipMemcpyAsync(hk.data(), gkey.p, gcap * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(hf.data(), gflag.p, gcap * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(&hov, ovf.p, 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (hov) return done(fail(MOSAIC_E_CAPACITY, "st_intersects_aggregate: group table overflow"));
    std::vector<std::pair<unsigned long long, uint8_t>> groups;
    for (uint64_t s = 0; s < gcap; s++)
        if (hk[s] != kEmptyGroup) groups.push_back({hk[s], (uint8_t)(hf[s] ? 1 : 0)});
    std::sort(groups.begin(), groups.end());
    *n_out = (int64_t)groups.size();
    if ((int64_t)groups.size() > cap)
        return done(fail(MOSAIC_E_CAPACITY, "st_intersects_aggregate: " + std::to_string(groups.size()) + " groups"));
    for (size_t i = 0; i < groups.size(); i++) {
        out_left_key[i] = (int32_t)(groups[i].first >> 32);
        out_right_key[i] = (int32_t)(groups[i].first & 0xffffffffULL);
        out_flag[i] = groups[i].second;
    }
    return done(MOSAIC_OK);
}

// The units of a chip join (k_isect_units over a's group table) run through
// k_isect_overlay in batches of <= 2 GB of scratch.  Per unit (sorted by group slot, then left cell
// slot): its record, edge count (-1: a capacity was exceeded), area, and edges (4 doubles each) at
// edge_off[u] .. edge_off[u] + count.
struct OverlayResult {
    std::vector<IsectUnit> units;
    std::vector<int32_t> count;
    std::vector<double> area;
    std::vector<int64_t> edge_off;
    std::vector<double> edges;
};

static int run_unit_overlay(ThreadCtx* c, const IsectArgs& a, int grid_sys, uint64_t unit_cap, OverlayResult& r) {
    DevBuf du, dn;
    DevBufGuard guard{{&du, &dn}};
    int rc;
    if ((rc = du.reserve(std::max<uint64_t>(unit_cap, 1) * sizeof(IsectUnit))) || (rc = dn.reserve(8))) return rc;
    HIP_TRY(hipMemsetAsync(dn.p, 0, 8, c->stream));
    const int64_t waves = (int64_t)a.capa;
    const int g = (int)std::max<int64_t>(1, std::min<int64_t>((waves * 64 + 255) / 256, (int64_t)c->n_cu * 16));
    hipLaunchKernelGGL(k_isect_units, dim3(g), dim3(256), 0, c->stream, a, (IsectUnit*)du.p, (unsigned long long*)dn.p,
                       (unsigned long long)unit_cap);
    HIP_TRY(hipGetLastError());
    unsigned long long nu = 0;
    HIP_TRY(hipMemcpyAsync(&nu, dn.p, 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (nu > unit_cap) return fail(MOSAIC_E_CAPACITY, "st_intersection_aggregate: unit list overflow");
    r.units.resize(nu);
    if (nu) HIP_TRY(hipMemcpy(r.units.data(), du.p, nu * sizeof(IsectUnit), hipMemcpyDeviceToHost));
    std::sort(r.units.begin(), r.units.end(), [](const IsectUnit& p, const IsectUnit& q) {
        return p.gs < q.gs || (p.gs == q.gs && p.slot < q.slot);
    });
    r.count.assign(nu, 0);
    r.area.assign(nu, 0.0);
    r.edge_off.assign(nu + 1, 0);
    std::vector<int64_t> sbytes(nu);
    for (size_t u = 0; u < nu; u++) {
        const IsectUnit& x = r.units[u];
        const bool cc = x.flags & 1u, skip = !cc && x.n_edges > kMaxUnitEdges;  // (skip: not answered)
        r.edge_off[u + 1] = r.edge_off[u] + (cc || skip ? 16 : 5 * (int64_t)x.n_edges + 64);
        sbytes[u] = cc || skip ? 0 : ((((int64_t)x.n_parts * (int64_t)sizeof(overlay::PartRef) + 63) & ~(int64_t)63) +
                                      ((overlay::scratch_bytes(x.n_edges) + 63) & ~(int64_t)63));
    }
    r.edges.assign((size_t)r.edge_off[nu] * 4, 0.0);
    const int64_t kBatch = (int64_t)2 << 30;
    // (the calling thread's scratch, kept between calls: fresh multi-GB allocations cost more than
    // the overlay itself)
    DevBuf &bu = c->ov[0], &bso = c->ov[1], &bsc = c->ov[2], &boo = c->ov[3], &bout = c->ov[4], &bcnt = c->ov[5],
           &bar = c->ov[6], &bord = c->ov[7];
    for (size_t u0 = 0; u0 < nu;) {
        size_t u1 = u0;
        int64_t sb = 0;
        while (u1 < nu && (u1 == u0 || sb + sbytes[u1] <= kBatch) && u1 - u0 < ((size_t)1 << 20)) sb += sbytes[u1++];
        const size_t m = u1 - u0;
        std::vector<int64_t> so(m), oo(m + 1);
        int64_t acc = 0;
        for (size_t i = 0; i < m; i++) so[i] = acc, acc += sbytes[u0 + i];
        for (size_t i = 0; i <= m; i++) oo[i] = r.edge_off[u0 + i] - r.edge_off[u0];
        std::vector<uint32_t> ord(m);
        for (size_t i = 0; i < m; i++) ord[i] = (uint32_t)i;
        std::stable_sort(ord.begin(), ord.end(), [&](uint32_t p, uint32_t q) {
            return r.units[u0 + p].n_edges > r.units[u0 + q].n_edges;
        });
        if ((rc = bu.reserve(m * sizeof(IsectUnit))) || (rc = bso.reserve(m * 8)) || (rc = bsc.reserve((size_t)std::max<int64_t>(acc, 64))) ||
            (rc = boo.reserve((m + 1) * 8)) || (rc = bout.reserve((size_t)std::max<int64_t>(oo[m], 1) * 32)) ||
            (rc = bcnt.reserve(m * 4)) || (rc = bar.reserve(m * 8)) || (rc = bord.reserve(m * 4)))
            return rc;
        HIP_TRY(hipMemcpyAsync(bord.p, ord.data(), m * 4, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(bu.p, r.units.data() + u0, m * sizeof(IsectUnit), hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(bso.p, so.data(), m * 8, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(boo.p, oo.data(), (m + 1) * 8, hipMemcpyHostToDevice, c->stream));
        OverlayArgs x;
        x.base = a;
        x.units = (const IsectUnit*)bu.p;
        x.order = (const uint32_t*)bord.p;
        x.n_units = m;
        x.scratch_off = (const int64_t*)bso.p;
        x.scratch = (char*)bsc.p;
        x.out_off = (const int64_t*)boo.p;
        x.out = (double*)bout.p;
        x.out_count = (int32_t*)bcnt.p;
        x.out_area = (double*)bar.p;
        x.grid = grid_sys;
        x.jdk = c->jdk;
        const int go = (int)std::max<size_t>(1, std::min<size_t>(m, (size_t)c->n_cu * 32));
        hipLaunchKernelGGL(k_isect_overlay, dim3(go), dim3(64), 0, c->stream, x);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(r.count.data() + u0, bcnt.p, m * 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(r.area.data() + u0, bar.p, m * 8, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(r.edges.data() + 4 * r.edge_off[u0], bout.p, (size_t)oo[m] * 32, hipMemcpyDeviceToHost,
                               c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        u0 = u1;
    }
    return MOSAIC_OK;
}

// Node tolerance of the stitch: chips are the reference's planar clips (llclip.h), so the same cell
// side crossing computed in two adjacent cells is the same double (the cells share their
// h3ToGeoBoundary vertices bit for bit and JTS's crossing arithmetic is symmetric in its segments);
// what is left are the overlay's own node positions (tol 2^-40 of the coordinates, overlay.h).  A
// fixed tolerance of that scale -- 180 x 2^-40 degrees (1.6e-10, ~16 um), 1e6 x 2^-40 metres for BNG
// -- never merges distinct chip vertices at any resolution (until round 5 it was 0.05 e^2 for the
// gnomonic-plane chips, kilometres at res 3).
static double stitch_snap(int grid, int res) {
    (void)res;
    return (grid == MOSAIC_GRID_BNG ? 1e6 : 180.0) * 9.094947017729282e-13;
}
// cell edge in output units (stitch check scale): H3 edge length in degrees, BNG the square's edge
static double agg_cell_edge(int grid, int res) {
    if (grid == MOSAIC_GRID_BNG) {
        static const double e_by_res[] = {0, 100000, 10000, 1000, 100, 10, 1};
        const int ar = res < 0 ? -res : res;
        return res == -1 ? 500000 : (res > 0 ? e_by_res[ar > 6 ? 6 : ar] : e_by_res[ar > 6 ? 6 : ar - 1] / 2.0);
    }
    static const double kEdgeKm[16] = {1107.712591, 418.6760055, 158.2446558, 59.81085794, 22.6063794, 8.544408276,
                                       3.229482772, 1.220629759, 0.461354684, 0.174375668, 0.065907807, 0.024910561,
                                       0.009415526, 0.003559893, 0.001348575, 0.000509713};
    return kEdgeKm[res < 0 ? 0 : (res > 15 ? 15 : res)] / 111.32;
}

struct mosaic_isect_geoms {
    std::vector<int32_t> lk, rk;
    std::vector<double> area;
    std::vector<uint8_t> status;
    std::vector<int64_t> off;
    std::vector<uint8_t> wkb;
};

// The units of the chip join of two tables through the cell overlay; groups are runs of units with
// one group slot (gstart), keyed by gkey[slot] = left key << 32 | right key.
struct AggUnits {
    OverlayResult r;
    std::vector<unsigned long long> gkey;
    std::vector<size_t> gstart;  // group g = units [gstart[g], gstart[g + 1])
};

static int aggregate_units(ThreadCtx* c, const mosaic_chips* left, const mosaic_chips* right, AggUnits& out) {
    out.gstart.assign(1, 0);
    if (left->n_chips == 0 || right->n_chips == 0) return MOSAIC_OK;
    IsectArgs a;
    a.ta = (const HashEntry*)left->table.p;
    a.capa = left->capacity;
    a.meta_a = (const uint32_t*)left->meta.p;
    a.sa = left->store.view();
    a.tb = (const HashEntry*)right->table.p;
    a.maskb = right->capacity - 1;
    a.meta_b = (const uint32_t*)right->meta.p;
    a.sb = right->store.view();
    DevBuf cnt, gkey, ovf;
    DevBufGuard guard{{&cnt, &gkey, &ovf}};
    int rc;
    if ((rc = cnt.reserve(8)) || (rc = ovf.reserve(4))) return rc;
    HIP_TRY(hipMemsetAsync(cnt.p, 0, 8, c->stream));
    HIP_TRY(hipMemsetAsync(ovf.p, 0, 4, c->stream));
    a.pass = 0;
    a.pair_count = (unsigned long long*)cnt.p;
    a.gkey = nullptr;
    a.gflag = nullptr;
    a.gmask = 0;
    a.overflow = (int*)ovf.p;
    const int64_t waves = (int64_t)left->capacity;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((waves * 64 + 255) / 256, (int64_t)c->n_cu * 16));
    hipLaunchKernelGGL(k_isect_agg, dim3(grid), dim3(256), 0, c->stream, a);  // pass 0: chip pairs
    HIP_TRY(hipGetLastError());
    unsigned long long pairs = 0;
    HIP_TRY(hipMemcpyAsync(&pairs, cnt.p, 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (pairs == 0) return MOSAIC_OK;
    uint64_t gcap = 1024;
    while (gcap < 2 * pairs) gcap <<= 1;
    if (gcap > ((uint64_t)1 << 32)) return fail(MOSAIC_E_CAPACITY, "st_intersection_aggregate: too many chip pairs");
    if ((rc = gkey.reserve(gcap * 8))) return rc;
    HIP_TRY(hipMemsetAsync(gkey.p, 0xff, gcap * 8, c->stream));
    a.gkey = (unsigned long long*)gkey.p;
    a.gmask = gcap - 1;
    if ((rc = run_unit_overlay(c, a, left->grid, pairs, out.r))) return rc;
    int hov = 0;
    out.gkey.resize(gcap);
    HIP_TRY(hipMemcpy(&hov, ovf.p, 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(out.gkey.data(), gkey.p, gcap * 8, hipMemcpyDeviceToHost));
    if (hov) return fail(MOSAIC_E_CAPACITY, "st_intersection_aggregate: group table overflow");
    out.gstart.clear();
    for (size_t u = 0; u < out.r.units.size(); u++)
        if (u == 0 || out.r.units[u].gs != out.r.units[u - 1].gs) out.gstart.push_back(u);
    out.gstart.push_back(out.r.units.size());
    return MOSAIC_OK;
}

// per group: the area (its units' areas summed in cell-slot order: the same bits on every call) or
// NaN when a unit exceeded a capacity / had no area; the order of groups by key pair
static void aggregate_areas(const AggUnits& g, std::vector<double>& area, std::vector<size_t>& order) {
    const size_t ng = g.gstart.size() - 1;
    area.assign(ng, 0.0);
    for (size_t k = 0; k < ng; k++)
        for (size_t u = g.gstart[k]; u < g.gstart[k + 1]; u++)
            area[k] = (g.r.count[u] < 0 || g.r.area[u] != g.r.area[u]) ? NAN : area[k] + g.r.area[u];
    order.resize(ng);
    for (size_t k = 0; k < ng; k++) order[k] = k;
    std::sort(order.begin(), order.end(), [&](size_t p, size_t q) {
        return g.gkey[g.r.units[g.gstart[p]].gs] < g.gkey[g.r.units[g.gstart[q]].gs];
    });
}

int mosaic_intersection_aggregate_geometry(mosaic_ctx* ctx, const mosaic_chips* left, const mosaic_chips* right,
                                           mosaic_isect_geoms** out) {
    ENTER(ctx);
    if (!c || !left || !right || !out) return fail(MOSAIC_E_ARG, "invalid argument");
    if (left->grid != right->grid || left->res != right->res)
        return fail(MOSAIC_E_ARG, "st_intersection_aggregate: both chip tables must use the same grid and resolution");
    *out = nullptr;
    HIP_TRY(hipSetDevice(c->device));
    AggUnits g;
    int rc;
    if ((rc = aggregate_units(c, left, right, g))) return rc;
    const OverlayResult& r = g.r;
    const size_t ng = g.gstart.size() - 1;
    std::vector<double> garea;
    std::vector<size_t> ord;
    aggregate_areas(g, garea, ord);
    // each group's cell boundaries stitched into its polygons, on host threads
    std::vector<std::vector<uint8_t>> wkbs(ng);
    std::vector<uint8_t> gst(ng, 0);
    const double snap = stitch_snap(left->grid, left->res), edge = agg_cell_edge(left->grid, left->res);
    std::atomic<size_t> next{0};
    auto work = [&]() {
        std::vector<double> e;
        for (size_t k; (k = next.fetch_add(1)) < ng;) {
            e.clear();
            if (garea[k] != garea[k]) {
                gst[k] = 1;
                continue;
            }
            for (size_t u = g.gstart[k]; u < g.gstart[k + 1]; u++)
                e.insert(e.end(), r.edges.begin() + 4 * r.edge_off[u], r.edges.begin() + 4 * (r.edge_off[u] + r.count[u]));
            double stitched = 0;
            // the dissolved polygons must keep the units' area: a stitch that merged or lost pieces
            // is flagged (status 1), not returned distorted
            const double bound = 1e-9 * std::max(fabs(garea[k]), edge * edge);
            if (!isect_geom::stitch_wkb(e.data(), e.size() / 4, snap, wkbs[k], &stitched) ||
                !(fabs(stitched - garea[k]) <= bound)) {
                gst[k] = 1;
                wkbs[k].clear();
            }
        }
    };
    {
        const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        std::vector<std::thread> th;
        for (unsigned t = 1; t < nt && t < ng; t++) th.emplace_back(work);
        work();
        for (auto& t : th) t.join();
    }
    auto* res = new mosaic_isect_geoms();
    res->off.push_back(0);
    for (size_t k : ord) {
        const unsigned long long key = g.gkey[r.units[g.gstart[k]].gs];
        res->lk.push_back((int32_t)(key >> 32));
        res->rk.push_back((int32_t)(key & 0xffffffffULL));
        res->area.push_back(gst[k] ? NAN : garea[k]);
        res->status.push_back(gst[k]);
        res->wkb.insert(res->wkb.end(), wkbs[k].begin(), wkbs[k].end());
        res->off.push_back((int64_t)res->wkb.size());
    }
    *out = res;
    return MOSAIC_OK;
}

int mosaic_isect_geoms_info(const mosaic_isect_geoms* g, int64_t* n_groups, int64_t* wkb_bytes) {
    if (!g || !n_groups || !wkb_bytes) return fail(MOSAIC_E_ARG, "null argument");
    *n_groups = (int64_t)g->lk.size();
    *wkb_bytes = (int64_t)g->wkb.size();
    return MOSAIC_OK;
}

int mosaic_isect_geoms_export(const mosaic_isect_geoms* g, int32_t* left_key, int32_t* right_key, double* area,
                              uint8_t* status, int64_t* wkb_offsets, uint8_t* wkb) {
    if (!g) return fail(MOSAIC_E_ARG, "null argument");
    const size_t n = g->lk.size();
    if (left_key) std::copy(g->lk.begin(), g->lk.end(), left_key);
    if (right_key) std::copy(g->rk.begin(), g->rk.end(), right_key);
    if (area) std::copy(g->area.begin(), g->area.end(), area);
    if (status) std::copy(g->status.begin(), g->status.end(), status);
    if (wkb_offsets) std::copy(g->off.begin(), g->off.begin() + (long)(n + 1), wkb_offsets);
    if (wkb && !g->wkb.empty()) memcpy(wkb, g->wkb.data(), g->wkb.size());
    return MOSAIC_OK;
}

int mosaic_isect_geoms_destroy(mosaic_isect_geoms* g) {
    delete g;
    return MOSAIC_OK;
}

int mosaic_intersection_aggregate(mosaic_ctx* ctx, const mosaic_chips* left, const mosaic_chips* right,
                                  int32_t* out_left_key, int32_t* out_right_key, double* out_area, uint8_t* out_status,
                                  int64_t cap, int64_t* n_out) {
    ENTER(ctx);
    if (!c || !left || !right || !n_out || cap < 0 ||
        (cap > 0 && (!out_left_key || !out_right_key || !out_area || !out_status)))
        return fail(MOSAIC_E_ARG, "invalid argument");
    if (left->grid != right->grid || left->res != right->res)
        return fail(MOSAIC_E_ARG, "st_intersection_aggregate: both chip tables must use the same grid and resolution");
    *n_out = 0;
    HIP_TRY(hipSetDevice(c->device));
    AggUnits g;
    int rc;
    if ((rc = aggregate_units(c, left, right, g))) return rc;
    std::vector<double> garea;
    std::vector<size_t> ord;
    aggregate_areas(g, garea, ord);
    *n_out = (int64_t)ord.size();
    if ((int64_t)ord.size() > cap)
        return fail(MOSAIC_E_CAPACITY, "st_intersection_aggregate: " + std::to_string(ord.size()) + " groups");
    for (size_t i = 0; i < ord.size(); i++) {
        const size_t k = ord[i];
        const unsigned long long key = g.gkey[g.r.units[g.gstart[k]].gs];
        out_left_key[i] = (int32_t)(key >> 32);
        out_right_key[i] = (int32_t)(key & 0xffffffffULL);
        out_area[i] = garea[k];
        out_status[i] = (uint8_t)(garea[k] != garea[k] ? 1 : 0);
    }
    return MOSAIC_OK;
}

int mosaic_cell_kring(mosaic_ctx* ctx, int grid, const int64_t* cells, const uint8_t* valid, int64_t n, int k, int loop,
                      int64_t* out, int32_t* out_count) {
    ENTER(ctx);
    if (!c || n < 0 || (n > 0 && (!cells || !out || !out_count))) return fail(MOSAIC_E_ARG, "invalid argument");
    if (grid != MOSAIC_GRID_BNG && grid != MOSAIC_GRID_H3) return fail(MOSAIC_E_ARG, "unknown grid");
    if (k < 0 || k > 1000) return fail(MOSAIC_E_ARG, "k must be in [0, 1000]");
    if (n == 0) return MOSAIC_OK;
    HIP_TRY(hipSetDevice(c->device));
    const bool h3g = grid == MOSAIC_GRID_H3;
    const int64_t stride = h3g ? (loop ? std::max<int64_t>(6 * (int64_t)k, 1) : 1 + 3 * (int64_t)k * (k + 1))
                               : (loop ? 8 * (int64_t)k : 1 + 4 * (int64_t)k * (k + 1));
    const int64_t slots = stride * n;  // 0 for a k = 0 loop: nothing to copy back
    DevBuf s_cells, s_valid, s_out, s_cnt, s_flags;
    auto done = [&](int rc) {
        for (DevBuf* b : {&s_cells, &s_valid, &s_out, &s_cnt, &s_flags}) b->release();
        return rc;
    };
    int rc;
    const void *dc, *dv;
    if ((rc = to_device(c, s_cells, cells, (size_t)n * 8, &dc)) || (rc = to_device(c, s_valid, valid, (size_t)n, &dv)))
        return done(rc);
    const bool dev_out = is_device_ptr(out), dev_cnt = is_device_ptr(out_count);
    if ((!dev_out && (rc = s_out.reserve(std::max<size_t>((size_t)slots * 8, 16)))) || (!dev_cnt && (rc = s_cnt.reserve((size_t)n * 4))) ||
        (rc = s_flags.reserve(4)))
        return done(rc);
    HIP_TRY(hipMemsetAsync(s_flags.p, 0, 4, c->stream));
    KringArgs a;
    a.cells = (const int64_t*)dc;
    a.valid = (const uint8_t*)dv;
    a.n = n;
    a.k = k;
    a.loop = loop ? 1 : 0;
    a.stride = stride;
    a.out = dev_out ? out : (int64_t*)s_out.p;
    a.count = dev_cnt ? out_count : (int32_t*)s_cnt.p;
    a.flags = (unsigned int*)s_flags.p;
    if (h3g) hipLaunchKernelGGL(k_h3_kring, dim3(grid_size(c, n)), dim3(c->block), 0, c->stream, a);
    else hipLaunchKernelGGL(k_bng_kring, dim3(grid_size(c, n)), dim3(c->block), 0, c->stream, a);
    HIP_TRY(hipGetLastError());
    if (h3g) {
        // rows where H3 meets a pentagon (count -3): H3's fallback search, with scratch per row
        std::vector<int32_t> cnt((size_t)n);
        HIP_TRY(hipMemcpyAsync(cnt.data(), a.count, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        std::vector<int64_t> rows;
        for (int64_t i = 0; i < n; i++)
            if (cnt[(size_t)i] == -3) rows.push_back(i);
        if (!rows.empty() && k > h3nb::kSlowMaxK) {
            // beyond kSlowMaxK H3's search (~5 k^3 dependent visits per row: seconds for one lane at
            // k ~ 200, the device form would hold a wave that long) runs on host threads -- the same
            // h3nb::kring_slow (h3_neighbors.h) compiled by g++ (kring_host.cpp), so the rows equal
            // h3-java's _kRingInternal tables as the device rows do
            const int64_t m = h3nb::max_kring_size(k), m1 = h3nb::max_kring_size(k - 1);
            std::vector<int64_t> origin(rows.size());
            if (is_device_ptr(cells)) {
                std::vector<int64_t> all((size_t)n);
                HIP_TRY(hipMemcpy(all.data(), cells, (size_t)n * 8, hipMemcpyDeviceToHost));
                for (size_t j = 0; j < rows.size(); j++) origin[j] = all[(size_t)rows[j]];
            } else {
                for (size_t j = 0; j < rows.size(); j++) origin[j] = cells[(size_t)rows[j]];
            }
            std::vector<int64_t> res((size_t)rows.size() * (size_t)stride, 0);
            std::atomic<size_t> next{0};
            auto work = [&]() {
                std::vector<int64_t> tab((size_t)(m + m1));
                std::vector<int32_t> dist((size_t)m);
                std::vector<uint64_t> stack((size_t)k + 1);
                for (size_t j; (j = next.fetch_add(1)) < rows.size();)
                    cnt[(size_t)rows[j]] = mosaic::kring_slow_host((uint64_t)origin[j], k, loop, res.data() + j * (size_t)stride,
                                                                    tab.data(), dist.data(), stack.data());
            };
            {
                // (tables of ~3 k^2 cells per thread: at most 16 threads, fewer for huge k)
                const size_t per = (size_t)(m + m1) * 8 + (size_t)m * 4;
                const unsigned cap = (unsigned)std::max<size_t>(1, ((size_t)4 << 30) / std::max<size_t>(per, 1));
                const unsigned nt = std::max(1u, std::min({16u, std::thread::hardware_concurrency(), cap, (unsigned)rows.size()}));
                std::vector<std::thread> th;
                for (unsigned t = 1; t < nt; t++) th.emplace_back(work);
                work();
                for (auto& t : th) t.join();
            }
            for (size_t j = 0; j < rows.size(); j++)
                HIP_TRY(hipMemcpyAsync(a.out + rows[j] * stride, res.data() + j * (size_t)stride, (size_t)stride * 8,
                                       hipMemcpyHostToDevice, c->stream));
            HIP_TRY(hipMemcpyAsync(a.count, cnt.data(), (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
            HIP_TRY(hipStreamSynchronize(c->stream));
            rows.clear();
        }
        if (!rows.empty()) {
            const int64_t m = h3nb::max_kring_size(k), m1 = k ? h3nb::max_kring_size(k - 1) : 1;
            const int64_t per = std::max<int64_t>(1, ((int64_t)1 << 30) / ((m + m1) * 8 + m * 4 + (k + 1) * 8));
            const int lanes = k >= 16 ? 1 : 64;
            DevBuf s_rows, s_tab, s_dist, s_stack;
            auto done2 = [&](int r2) {
                for (DevBuf* b : {&s_rows, &s_tab, &s_dist, &s_stack}) b->release();
                return done(r2);
            };
            for (size_t r0 = 0; r0 < rows.size(); r0 += (size_t)per) {
                const int64_t nr = std::min<int64_t>(per, (int64_t)(rows.size() - r0));
                if ((rc = s_rows.reserve((size_t)nr * 8)) || (rc = s_tab.reserve((size_t)(nr * (m + m1)) * 8)) ||
                    (rc = s_dist.reserve((size_t)(nr * m) * 4)) || (rc = s_stack.reserve((size_t)(nr * (k + 1)) * 8)))
                    return done2(rc);
                HIP_TRY(hipMemcpyAsync(s_rows.p, rows.data() + r0, (size_t)nr * 8, hipMemcpyHostToDevice, c->stream));
                hipLaunchKernelGGL(k_h3_kring_slow, dim3((unsigned)((nr + lanes - 1) / lanes)), dim3(64), 0, c->stream, a,
                                   (const int64_t*)s_rows.p, nr, lanes, (int64_t*)s_tab.p, m + m1, (int32_t*)s_dist.p, m,
                                   (uint64_t*)s_stack.p);
                HIP_TRY(hipGetLastError());
                HIP_TRY(hipStreamSynchronize(c->stream));
            }
            for (DevBuf* b : {&s_rows, &s_tab, &s_dist, &s_stack}) b->release();
        }
    }
    unsigned int flags = 0;
    HIP_TRY(hipMemcpyAsync(&flags, s_flags.p, 4, hipMemcpyDeviceToHost, c->stream));
    if (!dev_out && slots > 0)
        HIP_TRY(hipMemcpyAsync(out, s_out.p, (size_t)slots * 8, hipMemcpyDeviceToHost, c->stream));
    if (!dev_cnt) HIP_TRY(hipMemcpyAsync(out_count, s_cnt.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (flags & 1u) return done(fail(MOSAIC_E_ARG, "invalid BNG cell id"));
    return done(MOSAIC_OK);
}


int mosaic_bng_format_column(mosaic_ctx* ctx, const int64_t* ids, const uint8_t* valid, int64_t n, int64_t* offsets,
                             char* chars, int64_t chars_cap, int64_t* chars_needed) {
    ENTER(ctx);
    if (!c || n < 0 || !offsets || !chars_needed || (n > 0 && !ids) || chars_cap < 0 || (chars_cap > 0 && !chars))
        return fail(MOSAIC_E_ARG, "invalid argument");
    HIP_TRY(hipSetDevice(c->device));
    DevBuf s_ids, s_valid, s_off, s_chars, s_flags, s_tmp;
    auto done = [&](int rc) {
        for (DevBuf* b : {&s_ids, &s_valid, &s_off, &s_chars, &s_flags, &s_tmp}) b->release();
        return rc;
    };
    int rc;
    const void *di, *dv;
    if ((rc = to_device(c, s_ids, ids, (size_t)n * 8, &di)) || (rc = to_device(c, s_valid, valid, (size_t)n, &dv)))
        return done(rc);
    const bool dev_off = is_device_ptr(offsets);
    if ((!dev_off && (rc = s_off.reserve((size_t)(n + 1) * 8))) || (rc = s_flags.reserve(4))) return done(rc);
    int64_t* doff = dev_off ? offsets : (int64_t*)s_off.p;
    HIP_TRY(hipMemsetAsync(doff, 0, 8, c->stream));
    HIP_TRY(hipMemsetAsync(s_flags.p, 0, 4, c->stream));
    FormatArgs a;
    a.ids = (const int64_t*)di;
    a.valid = (const uint8_t*)dv;
    a.n = n;
    a.offsets = doff;
    a.chars = nullptr;
    a.flags = (unsigned int*)s_flags.p;
    if (n > 0) {
        hipLaunchKernelGGL(k_bng_format_len, dim3(grid_size(c, n)), dim3(c->block), 0, c->stream, a);
        HIP_TRY(hipGetLastError());
        size_t tmp_bytes = 0;
        // n may exceed INT_MAX: scan in pieces of 2^30 rows, carrying the running total
        const int64_t piece = (int64_t)1 << 30;
        HIP_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, tmp_bytes, doff + 1, doff + 1, (int)std::min(n, piece),
                                                 c->stream));
        if ((rc = s_tmp.reserve(std::max<size_t>(tmp_bytes, 16)))) return done(rc);
        for (int64_t lo = 0; lo < n; lo += piece) {
            const int m = (int)std::min(piece, n - lo);
            if (lo > 0) {
                // add the previous pieces' total to this piece's first length
                hipLaunchKernelGGL(k_add_prev, dim3(1), dim3(1), 0, c->stream, doff + 1 + lo, doff + lo);
                HIP_TRY(hipGetLastError());
            }
            size_t tb = s_tmp.bytes;
            HIP_TRY(hipcub::DeviceScan::InclusiveSum(s_tmp.p, tb, doff + 1 + lo, doff + 1 + lo, m, c->stream));
        }
    }
    int64_t total = 0;
    unsigned int flags = 0;
    HIP_TRY(hipMemcpyAsync(&total, doff + n, 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(&flags, s_flags.p, 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (flags & 1u) return done(fail(MOSAIC_E_ARG, "invalid BNG id in the column"));
    *chars_needed = total;
    if (!dev_off) HIP_TRY(hipMemcpy(offsets, doff, (size_t)(n + 1) * 8, hipMemcpyDeviceToHost));
    if (total > chars_cap) return done(fail(MOSAIC_E_CAPACITY, "chars buffer too small"));
    if (total == 0) return done(MOSAIC_OK);
    const bool dev_chars = is_device_ptr(chars);
    if (!dev_chars && (rc = s_chars.reserve((size_t)total))) return done(rc);
    a.chars = dev_chars ? chars : (char*)s_chars.p;
    hipLaunchKernelGGL(k_bng_format_write, dim3(grid_size(c, n)), dim3(c->block), 0, c->stream, a);
    HIP_TRY(hipGetLastError());
    if (!dev_chars) HIP_TRY(hipMemcpyAsync(chars, s_chars.p, (size_t)total, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return done(MOSAIC_OK);
}


int mosaic_h3_cell_geometry(mosaic_ctx* ctx, int mode, const int64_t* ids, const uint8_t* valid, int64_t n,
                            void* out, int32_t* out_count) {
    ENTER(ctx);
    if (!c || n < 0 || mode < 0 || mode > 2 || (n > 0 && (!ids || !out || !out_count)))
        return fail(MOSAIC_E_ARG, "invalid argument");
    if (n == 0) return MOSAIC_OK;
    HIP_TRY(hipSetDevice(c->device));
    DevBuf s_ids, s_valid, s_out, s_cnt, s_flags;
    DevBufGuard guard{{&s_ids, &s_valid, &s_out, &s_cnt, &s_flags}};
    int rc;
    const void *di, *dv;
    if ((rc = to_device(c, s_ids, ids, (size_t)n * 8, &di)) || (rc = to_device(c, s_valid, valid, (size_t)n, &dv)))
        return rc;
    const size_t bytes = (size_t)n * (mode == 0 ? 16 : (mode == 1 ? 160 : (size_t)kH3WkbStride));
    const bool dev_out = is_device_ptr(out), dev_cnt = is_device_ptr(out_count);
    if ((!dev_out && (rc = s_out.reserve(bytes))) || (!dev_cnt && (rc = s_cnt.reserve((size_t)n * 4))) ||
        (rc = s_flags.reserve(4)))
        return rc;
    void* dout = dev_out ? out : s_out.p;
    int32_t* dcnt = dev_cnt ? out_count : (int32_t*)s_cnt.p;
    HIP_TRY(hipMemsetAsync(dout, 0, bytes, c->stream));
    HIP_TRY(hipMemsetAsync(s_flags.p, 0, 4, c->stream));
    hipLaunchKernelGGL(k_h3_geom, dim3(grid_size(c, n)), dim3(c->block), 0, c->stream, (const int64_t*)di,
                       (const uint8_t*)dv, n, mode, c->jdk, dout, dcnt, (unsigned int*)s_flags.p);
    HIP_TRY(hipGetLastError());
    unsigned int flags = 0;
    HIP_TRY(hipMemcpyAsync(&flags, s_flags.p, 4, hipMemcpyDeviceToHost, c->stream));
    if (!dev_out) HIP_TRY(hipMemcpyAsync(out, dout, bytes, hipMemcpyDeviceToHost, c->stream));
    if (!dev_cnt) HIP_TRY(hipMemcpyAsync(out_count, dcnt, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (flags & 1u) return fail(MOSAIC_E_ARG, "invalid H3 cell id");
    return MOSAIC_OK;
}

int mosaic_cell_boundary_wkb(mosaic_ctx* ctx, int grid, const int64_t* ids, const uint8_t* valid, int64_t n,
                             uint8_t* out) {
    ENTER(ctx);
    if (!c || n < 0 || (n > 0 && (!ids || !out))) return fail(MOSAIC_E_ARG, "invalid argument");
    if (grid != MOSAIC_GRID_BNG)
        return fail(MOSAIC_E_ARG, "grid_boundaryaswkb: only the BNG grid is implemented by this engine");
    if (n == 0) return MOSAIC_OK;
    HIP_TRY(hipSetDevice(c->device));
    DevBuf s_ids, s_valid, s_out, s_flags;
    auto done = [&](int rc) {
        for (DevBuf* b : {&s_ids, &s_valid, &s_out, &s_flags}) b->release();
        return rc;
    };
    int rc;
    const void *di, *dv;
    if ((rc = to_device(c, s_ids, ids, (size_t)n * 8, &di)) || (rc = to_device(c, s_valid, valid, (size_t)n, &dv)))
        return done(rc);
    const size_t bytes = (size_t)n * bng::kCellWkbBytes;
    const bool dev_out = is_device_ptr(out);
    if ((!dev_out && (rc = s_out.reserve(bytes))) || (rc = s_flags.reserve(4))) return done(rc);
    uint8_t* dout = dev_out ? out : (uint8_t*)s_out.p;
    if (!dev_out && valid) HIP_TRY(hipMemsetAsync(dout, 0, bytes, c->stream));
    HIP_TRY(hipMemsetAsync(s_flags.p, 0, 4, c->stream));
    hipLaunchKernelGGL(k_bng_cell_wkb, dim3(grid_size(c, n)), dim3(c->block), 0, c->stream, (const int64_t*)di,
                       (const uint8_t*)dv, n, dout, (unsigned int*)s_flags.p);
    HIP_TRY(hipGetLastError());
    unsigned int flags = 0;
    HIP_TRY(hipMemcpyAsync(&flags, s_flags.p, 4, hipMemcpyDeviceToHost, c->stream));
    if (!dev_out) HIP_TRY(hipMemcpyAsync(out, dout, bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (flags & 1u) return done(fail(MOSAIC_E_ARG, "invalid BNG cell id"));
    return done(MOSAIC_OK);
}

}  // extern "C"

// ---- grid_tessellateexplode (BNG): per-cell classification on the GPU ----
// Reference: IndexSystem.getCoreChips / getBorderChips (core/index/IndexSystem.scala:152-186) via
// Mosaic.mosaicFill (core/Mosaic.scala:60-87).  The producer's contract (tessellate.cpp emit_cell):
// a candidate cell is a BORDER cell if any polygon segment comes within eps of the cell square,
// else a CORE cell if its centre is inside a part (even-odd over the part's rings), else it is
// dropped.  That test is O(segments) per cell and dominates chip production; one wave per
// candidate cell runs it here, lanes strided over each ring's segments (HBM/L2-resident rings,
// read once per wave; the rings of one geometry stay in L2 across its candidates).  Arithmetic is
// the host test's, operation for operation (no contraction), so the classes are bit-identical.
namespace tessgpu {

__device__ inline bool seg_near_square(double px, double py, double qx, double qy, const double* sx,
                                       const double* sy, double eps) {
    // tessellate.cpp seg_near_convex with the 4-vertex ccw square (sx[k], sy[k])
    auto inside = [&](double rx, double ry) {
        for (int i = 0; i < 4; i++) {
            double ax = sx[i], ay = sy[i], bx = sx[(i + 1) & 3], by = sy[(i + 1) & 3];
            double ex = bx - ax, ey = by - ay, len = sqrt(ex * ex + ey * ey);
            if ((ex * (ry - ay) - ey * (rx - ax)) / len < -eps) return false;
        }
        return true;
    };
    if (inside(px, py) || inside(qx, qy)) return true;
    auto dist_seg = [](double rx, double ry, double ax, double ay, double bx, double by) {
        double ex = bx - ax, ey = by - ay;
        double t = ((rx - ax) * ex + (ry - ay) * ey) / (ex * ex + ey * ey);
        t = fmax(0.0, fmin(1.0, t));
        double dx = ax + t * ex - rx, dy = ay + t * ey - ry;
        return sqrt(dx * dx + dy * dy);
    };
    for (int i = 0; i < 4; i++) {
        double ax = sx[i], ay = sy[i], bx = sx[(i + 1) & 3], by = sy[(i + 1) & 3];
        double d1 = (bx - ax) * (py - ay) - (by - ay) * (px - ax);
        double d2 = (bx - ax) * (qy - ay) - (by - ay) * (qx - ax);
        double d3 = (qx - px) * (ay - py) - (qy - py) * (ax - px);
        double d4 = (qx - px) * (by - py) - (qy - py) * (bx - px);
        if (((d1 > 0) != (d2 > 0)) && ((d3 > 0) != (d4 > 0))) return true;
        if (dist_seg(ax, ay, px, py, qx, qy) < eps || dist_seg(px, py, ax, ay, bx, by) < eps ||
            dist_seg(qx, qy, ax, ay, bx, by) < eps)
            return true;
    }
    return false;
}

struct ClassifyArgs {
    const double* xy;             // interleaved vertices (x, y)
    const int64_t* ring_offsets;  // [n_rings + 1]
    const int64_t* part_rings;    // [n_parts + 1]
    const int64_t* geom_parts;    // [n_geoms + 1]
    const int32_t* cand_geom;     // [n_cand]
    const int64_t* cand_ij;       // [2 n_cand] lower-left cell corner / e
    int64_t n_cand;
    double e, eps;
    uint8_t* cls;  // 0 dropped, 1 core, 2 border
};

__global__ void __launch_bounds__(256) k_bng_tess_classify(ClassifyArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t n_waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t c = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; c < a.n_cand; c += n_waves) {
        const int g = a.cand_geom[c];
        const double cx0 = (double)a.cand_ij[2 * c] * a.e, cy0 = (double)a.cand_ij[2 * c + 1] * a.e;
        double sx[4] = {cx0, cx0 + a.e, cx0 + a.e, cx0};
        double sy[4] = {cy0, cy0, cy0 + a.e, cy0 + a.e};
        const int64_t p0 = a.geom_parts[g], p1 = a.geom_parts[g + 1];
        bool near = false;
        for (int64_t p = p0; p < p1 && !near; p++)
            for (int64_t r = a.part_rings[p]; r < a.part_rings[p + 1]; r++) {
                const int64_t b = a.ring_offsets[r], n = a.ring_offsets[r + 1] - b;
                bool hit = false;
                for (int64_t v = lane; v + 1 < n && !hit; v += 64) {
                    const double* s = a.xy + 2 * (b + v);
                    hit = seg_near_square(s[0], s[1], s[2], s[3], sx, sy, a.eps);
                }
                if (__ballot(hit)) {
                    near = true;
                    break;
                }
            }
        uint8_t out = 2;
        if (!near) {
            // centre = ((((0 + x0) + x1) + x2) + x3) / 4 as the host sums the clip square
            const double cx = (((0.0 + sx[0]) + sx[1]) + sx[2] + sx[3]) / 4.0;
            const double cy = (((0.0 + sy[0]) + sy[1]) + sy[2] + sy[3]) / 4.0;
            bool inside = false;
            for (int64_t p = p0; p < p1 && !inside; p++) {
                bool par = false;
                for (int64_t r = a.part_rings[p]; r < a.part_rings[p + 1]; r++) {
                    const int64_t b = a.ring_offsets[r], n = a.ring_offsets[r + 1] - b;
                    for (int64_t i = lane; i < n; i += 64) {
                        const int64_t j = i == 0 ? n - 1 : i - 1;
                        const double ix = a.xy[2 * (b + i)], iy = a.xy[2 * (b + i) + 1];
                        const double jx = a.xy[2 * (b + j)], jy = a.xy[2 * (b + j) + 1];
                        if (((iy > cy) != (jy > cy)) && (cx < (jx - ix) * (cy - iy) / (jy - iy) + ix)) par = !par;
                    }
                }
                inside = (__popcll(__ballot(par)) & 1) != 0;
            }
            out = inside ? 1 : 0;
        }
        if (lane == 0) a.cls[c] = out;
    }
}

}  // namespace tessgpu

extern "C" {

// Classification step of mosaic_tessellate_gpu (tessellate.cpp); not part of the public header.

int mosaic_tess_classify_bng(mosaic_ctx* ctx, int64_t n_geoms, const int64_t* geom_parts, const int64_t* part_rings,
                             const int64_t* ring_offsets, const double* xy, int64_t n_cand, const int32_t* cand_geom,
                             const int64_t* cand_ij, double e, double eps, uint8_t* cls) {
    ENTER(ctx);
    if (!c || n_geoms < 0 || n_cand < 0 || (n_cand > 0 && (!geom_parts || !part_rings || !ring_offsets || !xy ||
                                                            !cand_geom || !cand_ij || !cls)))
        return fail(MOSAIC_E_ARG, "invalid argument");
    if (n_cand == 0) {
        c->last_tess_classify_ms = 0;  // (no kernel ran)
        return MOSAIC_OK;
    }
    for (int64_t k = 0; k < n_cand; k++)  // the kernel indexes geom_parts[g + 1]
        if (cand_geom[k] < 0 || cand_geom[k] >= n_geoms) return fail(MOSAIC_E_ARG, "candidate geometry out of range");
    HIP_TRY(hipSetDevice(c->device));
    const int64_t n_parts = geom_parts[n_geoms], n_rings = part_rings[n_parts], n_verts = ring_offsets[n_rings];
    DevBuf s_gp, s_pr, s_ro, s_xy, s_cg, s_ij, s_cls;
    DevBufGuard guard{{&s_gp, &s_pr, &s_ro, &s_xy, &s_cg, &s_ij, &s_cls}};
    auto done = [&](int rc) { return rc; };  // (the guard releases the buffers)
    int rc;
    const void *dgp, *dpr, *dro, *dxy, *dcg, *dij;
    if ((rc = to_device(c, s_gp, geom_parts, (size_t)(n_geoms + 1) * 8, &dgp)) ||
        (rc = to_device(c, s_pr, part_rings, (size_t)(n_parts + 1) * 8, &dpr)) ||
        (rc = to_device(c, s_ro, ring_offsets, (size_t)(n_rings + 1) * 8, &dro)) ||
        (rc = to_device(c, s_xy, xy, (size_t)std::max<int64_t>(n_verts, 1) * 16, &dxy)) ||
        (rc = to_device(c, s_cg, cand_geom, (size_t)n_cand * 4, &dcg)) ||
        (rc = to_device(c, s_ij, cand_ij, (size_t)n_cand * 16, &dij)) || (rc = s_cls.reserve((size_t)n_cand)))
        return done(rc);
    tessgpu::ClassifyArgs a;
    a.xy = (const double*)dxy;
    a.ring_offsets = (const int64_t*)dro;
    a.part_rings = (const int64_t*)dpr;
    a.geom_parts = (const int64_t*)dgp;
    a.cand_geom = (const int32_t*)dcg;
    a.cand_ij = (const int64_t*)dij;
    a.n_cand = n_cand;
    a.e = e;
    a.eps = eps;
    a.cls = (uint8_t*)s_cls.p;
    const int64_t blocks = std::min<int64_t>((n_cand + 3) / 4, (int64_t)c->n_cu * 16);  // 4 waves per block
    EventGuard ev;
    HIP_TRY(hipEventCreate(&ev.e[0]));
    HIP_TRY(hipEventCreate(&ev.e[1]));
    hipEvent_t t0 = ev.e[0], t1 = ev.e[1];
    HIP_TRY(hipEventRecord(t0, c->stream));
    hipLaunchKernelGGL(tessgpu::k_bng_tess_classify, dim3((unsigned)blocks), dim3(256), 0, c->stream, a);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(t1, c->stream));
    HIP_TRY(hipMemcpyAsync(cls, s_cls.p, (size_t)n_cand, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, t0, t1);
    c->last_tess_classify_ms = ms;
    return done(MOSAIC_OK);
}

double mosaic_tess_last_classify_ms(const mosaic_ctx* ctx) {
    ThreadCtx* c = enter(const_cast<mosaic_ctx*>(ctx));
    return c ? c->last_tess_classify_ms : -1.0;
}

}  // extern "C"

// ---- grid_tessellateexplode (H3): the same classification against a per-cell convex clip polygon ----
// The host producer classifies an H3 cell in its icosahedron face's gnomonic hex2d plane against the
// (densified) hexagon (tessellate.cpp, mosaic_tessellate H3 branch).  The hexagon vertices are
// computed on the host (glibc cos/sin) and passed per candidate, so the device test reads exactly the
// host's operands; rings arrive already projected into the face plane.
namespace tessgpu {

__device__ inline bool seg_near_poly(double px, double py, double qx, double qy, const double* P, int nv, double eps) {
    // tessellate.cpp seg_near_convex over the open ccw vertex list P[0..nv)
    auto inside = [&](double rx, double ry) {
        for (int i = 0; i < nv; i++) {
            const int k = i + 1 == nv ? 0 : i + 1;
            double ax = P[2 * i], ay = P[2 * i + 1], bx = P[2 * k], by = P[2 * k + 1];
            double ex = bx - ax, ey = by - ay, len = sqrt(ex * ex + ey * ey);
            if ((ex * (ry - ay) - ey * (rx - ax)) / len < -eps) return false;
        }
        return true;
    };
    if (inside(px, py) || inside(qx, qy)) return true;
    auto dist_seg = [](double rx, double ry, double ax, double ay, double bx, double by) {
        double ex = bx - ax, ey = by - ay;
        double t = ((rx - ax) * ex + (ry - ay) * ey) / (ex * ex + ey * ey);
        t = fmax(0.0, fmin(1.0, t));
        double dx = ax + t * ex - rx, dy = ay + t * ey - ry;
        return sqrt(dx * dx + dy * dy);
    };
    for (int i = 0; i < nv; i++) {
        const int k = i + 1 == nv ? 0 : i + 1;
        double ax = P[2 * i], ay = P[2 * i + 1], bx = P[2 * k], by = P[2 * k + 1];
        double d1 = (bx - ax) * (py - ay) - (by - ay) * (px - ax);
        double d2 = (bx - ax) * (qy - ay) - (by - ay) * (qx - ax);
        double d3 = (qx - px) * (ay - py) - (qy - py) * (ax - px);
        double d4 = (qx - px) * (by - py) - (qy - py) * (bx - px);
        if (((d1 > 0) != (d2 > 0)) && ((d3 > 0) != (d4 > 0))) return true;
        if (dist_seg(ax, ay, px, py, qx, qy) < eps || dist_seg(px, py, ax, ay, bx, by) < eps ||
            dist_seg(qx, qy, ax, ay, bx, by) < eps)
            return true;
    }
    return false;
}

struct ClassifyPolyArgs {
    const double* xy;  // ring vertices in the clip plane, interleaved
    const int64_t* ring_offsets;
    const int64_t* part_rings;
    const int64_t* geom_parts;
    const int32_t* cand_geom;
    const double* clip;  // [n_cand][nv][2]
    int nv;
    const int32_t* clip_n;  // per candidate: its clip polygon's vertices (<= nv); nullptr: nv each
    int64_t n_cand;
    double eps;
    uint8_t* cls;
};

__global__ void __launch_bounds__(256) k_tess_classify_poly(ClassifyPolyArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t n_waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t c = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; c < a.n_cand; c += n_waves) {
        const int g = a.cand_geom[c];
        const double* P = a.clip + 2 * (int64_t)a.nv * c;
        const int nvk = a.clip_n ? a.clip_n[c] : a.nv;
        const int64_t p0 = a.geom_parts[g], p1 = a.geom_parts[g + 1];
        bool near = false;
        for (int64_t p = p0; p < p1 && !near; p++)
            for (int64_t r = a.part_rings[p]; r < a.part_rings[p + 1]; r++) {
                const int64_t b = a.ring_offsets[r], n = a.ring_offsets[r + 1] - b;
                bool hit = false;
                for (int64_t v = lane; v + 1 < n && !hit; v += 64) {
                    const double* s = a.xy + 2 * (b + v);
                    hit = seg_near_poly(s[0], s[1], s[2], s[3], P, nvk, a.eps);
                }
                if (__ballot(hit)) {
                    near = true;
                    break;
                }
            }
        uint8_t out = 2;
        if (!near) {
            double cx = 0, cy = 0;  // centroid of the clip vertex list, summed in order as the host does
            for (int i = 0; i < nvk; i++) {
                cx += P[2 * i];
                cy += P[2 * i + 1];
            }
            cx /= (double)nvk;
            cy /= (double)nvk;
            bool inside = false;
            for (int64_t p = p0; p < p1 && !inside; p++) {
                bool par = false;
                for (int64_t r = a.part_rings[p]; r < a.part_rings[p + 1]; r++) {
                    const int64_t b = a.ring_offsets[r], n = a.ring_offsets[r + 1] - b;
                    for (int64_t i = lane; i < n; i += 64) {
                        const int64_t j = i == 0 ? n - 1 : i - 1;
                        const double ix = a.xy[2 * (b + i)], iy = a.xy[2 * (b + i) + 1];
                        const double jx = a.xy[2 * (b + j)], jy = a.xy[2 * (b + j) + 1];
                        if (((iy > cy) != (jy > cy)) && (cx < (jx - ix) * (cy - iy) / (jy - iy) + ix)) par = !par;
                    }
                }
                inside = (__popcll(__ballot(par)) & 1) != 0;
            }
            out = inside ? 1 : 0;
        }
        if (lane == 0) a.cls[c] = out;
    }
}

// mosaic_tessellate_gpu's H3 clip polygons generated on the device: candidate k's hexagon around its
// face-plane centre (cxy), each side cut into D pieces -- tessellate.cpp fill_clip's arithmetic
// (corner = centre + offset; a + (b - a) t / D, no contraction), so the same doubles.
struct FillClipArgs {
    const double* cxy;
    int64_t n_cand;
    int D;
    double dx[6], dy[6];
    double* clip;  // [n_cand][6 D][2]
};
__global__ void __launch_bounds__(256) k_tess_fill_clip(FillClipArgs a) {
    const int nv = 6 * a.D;
    const int64_t total = a.n_cand * nv;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < total; w += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = w / nv;
        const int v = (int)(w - k * nv), q = v / a.D, t = v - q * a.D, q1 = q + 1 == 6 ? 0 : q + 1;
        const double cx = a.cxy[2 * k], cy = a.cxy[2 * k + 1];
        const double ax = cx + a.dx[q], ay = cy + a.dy[q], bx = cx + a.dx[q1], by = cy + a.dy[q1];
        a.clip[2 * w] = ax + (bx - ax) * t / a.D;
        a.clip[2 * w + 1] = ay + (by - ay) * t / a.D;
    }
}

}  // namespace tessgpu

// host side of the border clipping (tess_gpu.h)

// The border candidates `tasks` clipped on the device by k_tess_clip_ll (tess_clip.hip) -- geometry
// arrays already on the device (d*), cell polygons from the candidates' H3 ids (d_cid, mode 0) or
// given (d_clip, nv vertices per candidate, mode 1).  Output space: a few points per task beyond the
// typical chip (a task that does not fit goes to the host, status 1), workspaces for at most
// n_cu x 128 lanes.
struct ClipLLBufs {
    DevBuf tasks, wch, wout, out, cnt, rings, parts, status;
    void release() {
        for (DevBuf* b : {&tasks, &wch, &wout, &out, &cnt, &rings, &parts, &status}) b->release();
    }
};
// the ring indexes of the lon / lat clip on the device (llclip::Geom::blk / ring_blk / ring_ccw): block
// offsets by a prefix over the host's ring offsets, envelopes and orientations by k_ring_blocks
struct RingIdxDev {
    DevBuf blk, rblk, ccw;
    int build(ThreadCtx* c, int64_t n_rings, const int64_t* ro, const void* d_ro, const void* d_xy) {
        std::vector<int64_t> rb((size_t)std::max<int64_t>(1, n_rings));
        int64_t t = 0;
        for (int64_t r = 0; r < n_rings; r++) rb[(size_t)r] = t, t += llclip::ring_block_count(ro, r);
        int rc;
        if ((rc = rblk.reserve(rb.size() * 8)) || (rc = blk.reserve((size_t)std::max<int64_t>(1, t) * 32)) ||
            (rc = ccw.reserve((size_t)std::max<int64_t>(16, n_rings))) || (rc = h2d(c, rblk.p, rb.data(), (size_t)n_rings * 8)))
            return rc;
        HIP_TRY(mosaic::tessll::launch_ring_blocks((const int64_t*)d_ro, (const double*)d_xy, n_rings, (const int64_t*)rblk.p,
                                                   (double*)blk.p, (uint8_t*)ccw.p, c->stream));
        return MOSAIC_OK;
    }
    void release() {
        blk.release();
        rblk.release();
        ccw.release();
    }
};

static int run_clip_ll(ThreadCtx* c, ClipLLBufs& B, const void* d_gxy, const void* d_ro, const void* d_pr, const void* d_gp,
                       const void* d_cg, const void* d_cid, const void* d_clip, int nv, int mode,
                       const std::vector<int64_t>& tasks, const int32_t* cand_geom, const int64_t* geom_parts,
                       const int64_t* part_rings, const int64_t* ring_offsets, tessclip::ClipResult* out,
                       const RingIdxDev* ri) {
    const int64_t n_tasks = (int64_t)tasks.size();
    out->status.assign((size_t)n_tasks, 0);
    out->rings.clear();
    out->parts.clear();
    out->verts.clear();
    out->kernel_ms = 0;
    if (n_tasks == 0) return MOSAIC_OK;
    // output bound per task: its geometry's vertices + events and cell vertices, capped near the
    // typical chip size (the rest to the host)
    int64_t bound = 0;
    for (int64_t t = 0; t < n_tasks; t++) {
        const int g = cand_geom[tasks[(size_t)t]];
        bound += ring_offsets[part_rings[geom_parts[g + 1]]] - ring_offsets[part_rings[geom_parts[g]]] + 4 * mosaic::tessll::kLLChains + 32;
    }
    const int64_t out_cap = std::min<int64_t>(bound, n_tasks * 96 + ((int64_t)1 << 20));
    const int64_t ring_cap = n_tasks * mosaic::tessll::kLLOut, part_cap = ring_cap;
    const int64_t lanes = std::max<int64_t>(64, std::min<int64_t>(n_tasks, (int64_t)c->n_cu * 128));
    int rc;
    if ((rc = B.tasks.reserve((size_t)n_tasks * 8)) || (rc = B.wch.reserve((size_t)lanes * mosaic::tessll::kLLChains * sizeof(llclip::Chain))) ||
        (rc = B.wout.reserve((size_t)lanes * mosaic::tessll::kLLOut * sizeof(llclip::Out))) || (rc = B.out.reserve((size_t)out_cap * 16)) ||
        (rc = B.cnt.reserve(32)) || (rc = B.rings.reserve((size_t)ring_cap * sizeof(tessclip::ClipRing))) ||
        (rc = B.parts.reserve((size_t)part_cap * sizeof(tessclip::ClipPart))) || (rc = B.status.reserve((size_t)n_tasks)))
        return rc;
    if ((rc = h2d(c, B.tasks.p, tasks.data(), (size_t)n_tasks * 8))) return rc;
    HIP_TRY(hipMemsetAsync(B.cnt.p, 0, 32, c->stream));
    mosaic::tessll::ClipLLArgs a;
    a.gxy = (const double*)d_gxy;
    a.ring_offsets = (const int64_t*)d_ro;
    a.part_rings = (const int64_t*)d_pr;
    a.geom_parts = (const int64_t*)d_gp;
    a.cand_geom = (const int32_t*)d_cg;
    a.cand_id = (const int64_t*)d_cid;
    a.clip = (const double*)d_clip;
    a.nv = nv;
    a.mode = mode;
    a.tasks = (const int64_t*)B.tasks.p;
    a.n_tasks = n_tasks;
    a.wch = (llclip::Chain*)B.wch.p;
    a.wout = (llclip::Out*)B.wout.p;
    a.out = (double*)B.out.p;
    a.counters = (unsigned long long*)B.cnt.p;
    a.out_cap = out_cap;
    a.ring_cap = ring_cap;
    a.part_cap = part_cap;
    a.rings = (tessclip::ClipRing*)B.rings.p;
    a.parts = (tessclip::ClipPart*)B.parts.p;
    a.status = (uint8_t*)B.status.p;
    a.blk = ri ? (const double*)ri->blk.p : nullptr;
    a.ring_blk = ri ? (const int64_t*)ri->rblk.p : nullptr;
    a.ring_ccw = ri ? (const uint8_t*)ri->ccw.p : nullptr;
    EventGuard ev;
    HIP_TRY(hipEventCreate(&ev.e[0]));
    HIP_TRY(hipEventCreate(&ev.e[1]));
    HIP_TRY(hipEventRecord(ev.e[0], c->stream));
    HIP_TRY(mosaic::tessll::launch_clip_ll(a, lanes, c->stream));
    HIP_TRY(hipEventRecord(ev.e[1], c->stream));
    unsigned long long cnt[3];
    if ((rc = d2h(c, cnt, B.cnt.p, sizeof cnt))) return rc;
    if ((rc = d2h(c, out->status.data(), B.status.p, (size_t)n_tasks))) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    // (counters past a cap: those tasks came back with status 1; the space before is valid)
    const int64_t nv_out = std::min<int64_t>((int64_t)cnt[0], out_cap), nr = std::min<int64_t>((int64_t)cnt[1], ring_cap),
                  np = std::min<int64_t>((int64_t)cnt[2], part_cap);
    out->verts.resize((size_t)nv_out * 2);
    out->rings.resize((size_t)nr);
    out->parts.resize((size_t)np);
    if (nv_out && (rc = d2h(c, out->verts.data(), B.out.p, (size_t)nv_out * 16))) return rc;
    if (nr && (rc = d2h(c, out->rings.data(), B.rings.p, (size_t)nr * sizeof(tessclip::ClipRing)))) return rc;
    if (np && (rc = d2h(c, out->parts.data(), B.parts.p, (size_t)np * sizeof(tessclip::ClipPart)))) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    // drop the records of tasks that went to the host (an overflowing task may have taken ring / part
    // slots before its check failed: it wrote nothing into them)
    {
        std::vector<uint8_t> host(out->status.size());
        std::unordered_map<int64_t, int64_t> pos;
        for (int64_t t = 0; t < n_tasks; t++) pos[tasks[(size_t)t]] = t;
        auto keep_ring = [&](const tessclip::ClipRing& r) { auto it = pos.find(r.cand); return it != pos.end() && out->status[(size_t)it->second] != 1; };
        auto keep_part = [&](const tessclip::ClipPart& r) { auto it = pos.find(r.cand); return it != pos.end() && out->status[(size_t)it->second] != 1; };
        out->rings.erase(std::remove_if(out->rings.begin(), out->rings.end(), [&](const tessclip::ClipRing& r) { return !keep_ring(r); }), out->rings.end());
        out->parts.erase(std::remove_if(out->parts.begin(), out->parts.end(), [&](const tessclip::ClipPart& r) { return !keep_part(r); }), out->parts.end());
    }
    float ms = 0;
    (void)hipEventElapsedTime(&ms, ev.e[0], ev.e[1]);
    out->kernel_ms = ms;
    return MOSAIC_OK;
}

int tessclip::clip_ll(mosaic_ctx* ctx, int64_t n_geoms, const int64_t* geom_parts, const int64_t* part_rings,
                      const int64_t* ring_offsets, const double* xy, const std::vector<int64_t>& tasks,
                      const int32_t* cand_geom, int64_t n_cand, const double* clip, int nv, ClipResult* out) {
    ENTER(ctx);
    if (!out || n_geoms < 0 || nv < 3 || nv > 16) return fail(MOSAIC_E_ARG, "invalid argument");
    for (int64_t k : tasks)
        if (k < 0 || k >= n_cand || cand_geom[k] < 0 || cand_geom[k] >= n_geoms) return fail(MOSAIC_E_ARG, "task out of range");
    if (tasks.empty()) {
        out->status.clear();
        out->rings.clear();
        out->parts.clear();
        out->verts.clear();
        out->kernel_ms = 0;
        return MOSAIC_OK;
    }
    HIP_TRY(hipSetDevice(c->device));
    const int64_t n_parts = geom_parts[n_geoms], n_rings = part_rings[n_parts], n_verts = ring_offsets[n_rings];
    TmpBuf s_gp, s_pr, s_ro, s_xy, s_cg, s_clip;
    ClipLLBufs B;
    struct Rel {
        ClipLLBufs& b;
        ~Rel() { b.release(); }
    } rel{B};
    auto up = [&](TmpBuf& b, const void* src, size_t bytes) -> int {
        int e = b.reserve(std::max<size_t>(bytes, 16));
        if (e) return e;
        if (bytes) if (int e_ = h2d(c, b.p, src, bytes)) return e_;
        return MOSAIC_OK;
    };
    int rc;
    if ((rc = up(s_gp, geom_parts, (size_t)(n_geoms + 1) * 8)) || (rc = up(s_pr, part_rings, (size_t)(n_parts + 1) * 8)) ||
        (rc = up(s_ro, ring_offsets, (size_t)(n_rings + 1) * 8)) || (rc = up(s_xy, xy, (size_t)n_verts * 16)) ||
        (rc = up(s_cg, cand_geom, (size_t)n_cand * 4)) || (rc = up(s_clip, clip, (size_t)n_cand * nv * 16)))
        return rc;
    RingIdxDev ri;
    struct RelRi {
        RingIdxDev& r;
        ~RelRi() { r.release(); }
    } rel_ri{ri};
    if ((rc = ri.build(c, n_rings, ring_offsets, s_ro.p, s_xy.p))) return rc;
    return run_clip_ll(c, B, s_xy.p, s_ro.p, s_pr.p, s_gp.p, s_cg.p, nullptr, s_clip.p, nv, 1, tasks, cand_geom, geom_parts,
                       part_rings, ring_offsets, out, &ri);
}

// ---- mosaic_tessellate_gpu's H3 branch as one device session: the geometry batch is uploaded once,
// each chunk of candidates uploads only its centres (16 B each) and ids (8 B); clip polygons are
// generated on the device (k_tess_fill_clip), classified in the face plane (k_tess_classify_poly)
// and the border ones clipped in lon / lat against their cells' boundaries (k_tess_clip_ll) from the
// same device arrays.
struct tessclip::H3Session {
    mosaic_ctx* ctx;
    int64_t n_geoms, n_parts, n_rings, n_verts, maxn;
    const int64_t *geom_parts, *part_rings, *ring_offsets;
    int res, D;
    double dx[6], dy[6];
    DevBuf d_gp, d_pr, d_ro, d_pxy, d_gxy, d_gf, d_cg, d_cxy, d_clip, d_cls, d_cn, d_cid, d_cnt;
    ClipLLBufs ll;
    RingIdxDev ri;
    void release() {
        for (DevBuf* b : {&d_gp, &d_pr, &d_ro, &d_pxy, &d_gxy, &d_gf, &d_cg, &d_cxy, &d_clip, &d_cls, &d_cn, &d_cid, &d_cnt})
            b->release();
        ll.release();
        ri.release();
    }
};

int tessclip::h3_session_begin(mosaic_ctx* ctx, int64_t n_geoms, const int64_t* geom_parts, const int64_t* part_rings,
                               const int64_t* ring_offsets, const double* pxy, const double* gxy, const int32_t* gface,
                               int res, int D, const double* dx, const double* dy, H3Session** out) {
    ENTER(ctx);
    if (!out || n_geoms < 0 || D < 1 || D > 64 || res < 0 || res > 15) return fail(MOSAIC_E_ARG, "invalid argument");
    H3Session* S = new H3Session();
    S->ctx = ctx;
    S->n_geoms = n_geoms;
    S->n_parts = geom_parts[n_geoms];
    S->n_rings = part_rings[S->n_parts];
    S->n_verts = ring_offsets[S->n_rings];
    S->geom_parts = geom_parts;
    S->part_rings = part_rings;
    S->ring_offsets = ring_offsets;
    S->res = res;
    S->D = D;
    for (int q = 0; q < 6; q++) {
        S->dx[q] = dx[q];
        S->dy[q] = dy[q];
    }
    S->maxn = 1;
    for (int64_t r = 0; r < S->n_rings; r++) S->maxn = std::max<int64_t>(S->maxn, ring_offsets[r + 1] - ring_offsets[r]);
    HIP_TRY(hipSetDevice(c->device));
    auto up = [&](DevBuf& b, const void* src, size_t bytes) -> int {
        int e = b.reserve(std::max<size_t>(bytes, 16));
        if (e) return e;
        if (bytes) if (int e_ = h2d(c, b.p, src, bytes)) return e_;
        return MOSAIC_OK;
    };
    int rc;
    if ((rc = up(S->d_gp, geom_parts, (size_t)(n_geoms + 1) * 8)) || (rc = up(S->d_pr, part_rings, (size_t)(S->n_parts + 1) * 8)) ||
        (rc = up(S->d_ro, ring_offsets, (size_t)(S->n_rings + 1) * 8)) || (rc = up(S->d_pxy, pxy, (size_t)S->n_verts * 16)) ||
        (rc = up(S->d_gxy, gxy, (size_t)S->n_verts * 16)) || (rc = up(S->d_gf, gface, (size_t)n_geoms * 4)) ||
        (rc = S->d_cnt.reserve(32)) || (rc = S->ri.build(c, S->n_rings, ring_offsets, S->d_ro.p, S->d_gxy.p))) {
        S->release();
        delete S;
        return rc;
    }
    *out = S;
    return MOSAIC_OK;
}

void tessclip::h3_session_end(H3Session* S) {
    if (!S) return;
    ThreadCtx* c = enter(S->ctx);
    if (c) {
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
    }
    S->release();
    delete S;
}

int tessclip::h3_session_chunk(H3Session* S, int64_t nc, const int32_t* cand_geom, const double* cxy, double eps,
                               uint8_t* cls, std::vector<int64_t>& tasks, ClipResult* out, const int64_t* cand_id,
                               const double* clip_xy, const int32_t* clip_n, int nv_max) {
    ENTER(S->ctx);
    const bool given = clip_xy != nullptr;  // explicit clip polygons (face pieces) instead of hexagons
    const int nv = given ? nv_max : 6 * S->D;
    tasks.clear();
    out->status.clear();
    out->rings.clear();
    out->parts.clear();
    out->verts.clear();
    out->kernel_ms = 0;
    if (nc <= 0) return MOSAIC_OK;
    HIP_TRY(hipSetDevice(c->device));
    int rc;
    auto up = [&](DevBuf& b, const void* src, size_t bytes) -> int {
        int e = b.reserve(std::max<size_t>(bytes, 16));
        if (e) return e;
        if (bytes) if (int e_ = h2d(c, b.p, src, bytes)) return e_;
        return MOSAIC_OK;
    };
    if ((rc = up(S->d_cg, cand_geom, (size_t)nc * 4)) || (rc = S->d_clip.reserve((size_t)nc * nv * 16)) ||
        (rc = S->d_cls.reserve((size_t)nc)))
        return rc;
    if (given) {
        if ((rc = up(S->d_clip, clip_xy, (size_t)nc * nv * 16)) || (rc = up(S->d_cn, clip_n, (size_t)nc * 4))) return rc;
    } else if ((rc = up(S->d_cxy, cxy, (size_t)nc * 16))) {
        return rc;
    }
    if (cand_id && (rc = up(S->d_cid, cand_id, (size_t)nc * 8))) return rc;
    tessgpu::FillClipArgs fa;
    fa.cxy = (const double*)S->d_cxy.p;
    fa.n_cand = nc;
    fa.D = S->D;
    for (int q = 0; q < 6; q++) {
        fa.dx[q] = S->dx[q];
        fa.dy[q] = S->dy[q];
    }
    fa.clip = (double*)S->d_clip.p;
    const int64_t nfill = nc * nv;
    if (!given)
        hipLaunchKernelGGL(tessgpu::k_tess_fill_clip, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((nfill + 255) / 256, 1 << 20))),
                           dim3(256), 0, c->stream, fa);
    HIP_TRY(hipGetLastError());
    tessgpu::ClassifyPolyArgs ca;
    ca.xy = (const double*)S->d_pxy.p;
    ca.ring_offsets = (const int64_t*)S->d_ro.p;
    ca.part_rings = (const int64_t*)S->d_pr.p;
    ca.geom_parts = (const int64_t*)S->d_gp.p;
    ca.cand_geom = (const int32_t*)S->d_cg.p;
    ca.clip = (const double*)S->d_clip.p;
    ca.nv = nv;
    ca.clip_n = given ? (const int32_t*)S->d_cn.p : nullptr;
    ca.n_cand = nc;
    ca.eps = eps;
    ca.cls = (uint8_t*)S->d_cls.p;
    const int64_t blocks = std::min<int64_t>((nc + 3) / 4, (int64_t)c->n_cu * 16);
    EventGuard ev;
    HIP_TRY(hipEventCreate(&ev.e[0]));
    HIP_TRY(hipEventCreate(&ev.e[1]));
    HIP_TRY(hipEventRecord(ev.e[0], c->stream));
    hipLaunchKernelGGL(tessgpu::k_tess_classify_poly, dim3((unsigned)blocks), dim3(256), 0, c->stream, ca);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ev.e[1], c->stream));
    if (int e_ = d2h(c, cls, S->d_cls.p, (size_t)nc)) return e_;
    HIP_TRY(hipStreamSynchronize(c->stream));
    float cms = 0;
    (void)hipEventElapsedTime(&cms, ev.e[0], ev.e[1]);
    c->last_tess_classify_ms = cms;
    if (!cand_id) return MOSAIC_OK;  // classification only (face pieces)
    // the border candidates, clipped in lon / lat on the device
    for (int64_t k = 0; k < nc; k++)
        if (cls[k] == 2) tasks.push_back(k);
    return run_clip_ll(c, S->ll, S->d_gxy.p, S->d_ro.p, S->d_pr.p, S->d_gp.p, S->d_cg.p, S->d_cid.p, nullptr, 0, 0, tasks,
                       cand_geom, S->geom_parts, S->part_rings, S->ring_offsets, out, &S->ri);
}

int tessclip::h3_cell_vertices(H3Session* S, const std::vector<int64_t>& ids, std::vector<double>& v, std::vector<int32_t>& cnt) {
    ENTER(S->ctx);
    const int64_t n = (int64_t)ids.size();
    v.resize((size_t)n * 20);
    cnt.resize((size_t)n);
    if (n == 0) return MOSAIC_OK;
    HIP_TRY(hipSetDevice(c->device));
    TmpBuf d_i, d_o, d_c, d_f;
    int rc;
    if ((rc = d_i.reserve((size_t)n * 8)) || (rc = d_o.reserve((size_t)n * 160)) || (rc = d_c.reserve((size_t)n * 4)) ||
        (rc = d_f.reserve(16)) || (rc = h2d(c, d_i.p, ids.data(), (size_t)n * 8)))
        return rc;
    HIP_TRY(hipMemsetAsync(d_f.p, 0, 16, c->stream));
    // k_h3_geom mode 1 with JDK 8's toDegrees: the vertices tessellate.cpp's h3_cell_ll computes
    hipLaunchKernelGGL(k_h3_geom, dim3(grid_size(c, n)), dim3(c->block), 0, c->stream, (const int64_t*)d_i.p,
                       (const uint8_t*)nullptr, n, 1, 8, d_o.p, (int32_t*)d_c.p, (unsigned int*)d_f.p);
    HIP_TRY(hipGetLastError());
    if ((rc = d2h(c, cnt.data(), d_c.p, (size_t)n * 4)) || (rc = d2h(c, v.data(), d_o.p, (size_t)n * 160))) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MOSAIC_OK;
}

extern "C" {

// Classification step of mosaic_tessellate_gpu for per-cell convex clip polygons (H3 hexagons in the
// face plane); not part of the public header.  xy holds the rings already in the clip plane.
int mosaic_tess_classify_poly(mosaic_ctx* ctx, int64_t n_geoms, const int64_t* geom_parts, const int64_t* part_rings,
                              const int64_t* ring_offsets, const double* xy, int64_t n_cand, const int32_t* cand_geom,
                              const double* clip, int nv, double eps, uint8_t* cls) {
    ENTER(ctx);
    if (!c || n_geoms < 0 || n_cand < 0 || nv < 3 ||
        (n_cand > 0 && (!geom_parts || !part_rings || !ring_offsets || !xy || !cand_geom || !clip || !cls)))
        return fail(MOSAIC_E_ARG, "invalid argument");
    if (n_cand == 0) {
        c->last_tess_classify_ms = 0;  // (no kernel ran)
        return MOSAIC_OK;
    }
    for (int64_t k = 0; k < n_cand; k++)
        if (cand_geom[k] < 0 || cand_geom[k] >= n_geoms) return fail(MOSAIC_E_ARG, "candidate geometry out of range");
    HIP_TRY(hipSetDevice(c->device));
    const int64_t n_parts = geom_parts[n_geoms], n_rings = part_rings[n_parts], n_verts = ring_offsets[n_rings];
    DevBuf s_gp, s_pr, s_ro, s_xy, s_cg, s_clip, s_cls;
    DevBufGuard guard{{&s_gp, &s_pr, &s_ro, &s_xy, &s_cg, &s_clip, &s_cls}};
    auto done = [&](int rc) { return rc; };  // (the guard releases the buffers)
    int rc;
    const void *dgp, *dpr, *dro, *dxy, *dcg, *dclip;
    if ((rc = to_device(c, s_gp, geom_parts, (size_t)(n_geoms + 1) * 8, &dgp)) ||
        (rc = to_device(c, s_pr, part_rings, (size_t)(n_parts + 1) * 8, &dpr)) ||
        (rc = to_device(c, s_ro, ring_offsets, (size_t)(n_rings + 1) * 8, &dro)) ||
        (rc = to_device(c, s_xy, xy, (size_t)std::max<int64_t>(n_verts, 1) * 16, &dxy)) ||
        (rc = to_device(c, s_cg, cand_geom, (size_t)n_cand * 4, &dcg)) ||
        (rc = to_device(c, s_clip, clip, (size_t)n_cand * nv * 16, &dclip)) || (rc = s_cls.reserve((size_t)n_cand)))
        return done(rc);
    tessgpu::ClassifyPolyArgs a;
    a.xy = (const double*)dxy;
    a.ring_offsets = (const int64_t*)dro;
    a.part_rings = (const int64_t*)dpr;
    a.geom_parts = (const int64_t*)dgp;
    a.cand_geom = (const int32_t*)dcg;
    a.clip = (const double*)dclip;
    a.nv = nv;
    a.clip_n = nullptr;
    a.n_cand = n_cand;
    a.eps = eps;
    a.cls = (uint8_t*)s_cls.p;
    const int64_t blocks = std::min<int64_t>((n_cand + 3) / 4, (int64_t)c->n_cu * 16);
    EventGuard ev;
    HIP_TRY(hipEventCreate(&ev.e[0]));
    HIP_TRY(hipEventCreate(&ev.e[1]));
    hipEvent_t t0 = ev.e[0], t1 = ev.e[1];
    HIP_TRY(hipEventRecord(t0, c->stream));
    hipLaunchKernelGGL(tessgpu::k_tess_classify_poly, dim3((unsigned)blocks), dim3(256), 0, c->stream, a);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(t1, c->stream));
    if (int e_ = d2h(c, cls, s_cls.p, (size_t)n_cand)) return e_;
    HIP_TRY(hipStreamSynchronize(c->stream));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, t0, t1);
    c->last_tess_classify_ms = ms;
    return done(MOSAIC_OK);
}

}  // extern "C"
