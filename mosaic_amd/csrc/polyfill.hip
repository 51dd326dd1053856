// grid_polyfill on the GPU (mosaic_polyfill): the cells of a polygonal geometry whose centre it
// holds, as the reference's IndexSystem.polyfill computes them.
//
// H3 (H3IndexSystem.polyfill, core/index/H3IndexSystem.scala:113-126): per polygon part,
// h3.polyfill(shell, holes, res) = H3 C v3.7 _polyfillInternal, restated as data-parallel rounds
// that reproduce its sequential result exactly:
//   1. k_pf_edge_count / k_pf_edge_sample: every ring edge sampled at lineHexEstimate points
//      (_getEdgeHexagons), each sample's cell kept once at its first sample (a device hash with
//      atomicMin of the sample index) -> the first search frontier, in H3's order.
//   2. rounds of k_pf_expand (kRing(1) of every frontier cell in hexRange order, h3fill::kring1; cells
//      already accepted skipped; each remaining (cell) claimed by its first (frontier position, ring
//      position) with atomicMin) and k_pf_accept (the claimant tests the cell's h3ToGeo centre with
//      H3's pointInsidePolygon, h3_polyfill.h), then a stream compaction in claim order: the next
//      frontier is exactly H3's `found` array of that round, and the accepted cells in round order
//      are exactly H3's insertion sequence into its output table.
//   3. host: that sequence inserted into an open-addressing table of maxPolyfillSize slots (home
//      slot cell % size, linear probing), read in slot order -- the order h3-java returns.  The
//      parts' lists are concatenated per geometry (H3IndexSystem.scala:118-124).
// Where H3's ring walk falls back to _kRingInternal (near the 12 pentagons) kring1 runs that
// fallback too (h3_neighbors.h), in H3's table order.  Rows that hold a non-finite vertex get status
// MOSAIC_POLYFILL_UNSUPPORTED.
//
// BNG (BNGIndexSystem.polyfill, core/index/BNGIndexSystem.scala:185-204): breadth-first from the
// cells of every vertex and of the JTS centroid; a visited cell is kept when the geometry contains
// (JTS, pip_device.h) its square's centroid, and its kLoop(1) cells are visited next.  Rounds of
// k_pf_bng_round over a visited-set hash; the cells are then ordered as the reference's Scala
// 2.12 immutable HashSet iterates them (hash-trie order of the improved Long hash) when there are
// more than four (Set1..Set4 keep insertion order, which is not restated: such rows are ordered
// the same way).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <memory>
#include <string>
#include <unordered_set>
#include <vector>

#include "../../include/mosaic_hip.h"
#include "bng_device.h"
#include "h3_grid.h"
#include "h3_polyfill.h"
#include "pip_device.h"

using namespace mosaic;

extern "C" int mosaic_tess_fail(int code, const char* msg);
extern "C" int mosaic_ctx_exec(mosaic_ctx* ctx, int* device, void** stream, int* jdk, int* n_cu);

struct mosaic_cell_lists {
    std::vector<int64_t> offsets{0};
    std::vector<int64_t> cells;
    std::vector<int32_t> status;
};

namespace {

constexpr uint64_t kEmpty = ~0ull;
constexpr int kPartBits = 12;  // polygon parts (H3) / geometries (BNG) per batch: < 4095
constexpr int64_t kBatch = 4094;

__host__ __device__ inline uint64_t hmix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

// Open-addressing insert; probes bounded by the capacity (flag bit 1 on overflow, never spins).
__device__ inline uint64_t tab_insert(uint64_t* keys, uint64_t mask, uint64_t key, bool* inserted,
                                      unsigned int* flags) {
    uint64_t h = hmix(key) & mask;
    for (uint64_t n = 0; n <= mask; n++, h = (h + 1) & mask) {
        const unsigned long long prev =
            atomicCAS((unsigned long long*)&keys[h], (unsigned long long)kEmpty, (unsigned long long)key);
        if (prev == kEmpty || prev == key) {
            *inserted = prev == kEmpty;
            return h;
        }
    }
    atomicOr(flags, 2u);
    *inserted = false;
    return kEmpty;
}
__device__ inline bool tab_has(const uint64_t* keys, uint64_t mask, uint64_t key) {
    uint64_t h = hmix(key) & mask;
    for (uint64_t n = 0; n <= mask; n++, h = (h + 1) & mask) {
        const uint64_t k = keys[h];
        if (k == key) return true;
        if (k == kEmpty) return false;
    }
    return false;
}

constexpr uint64_t kLow52 = ((uint64_t)1 << 52) - 1;
__host__ __device__ inline uint64_t h3_pack(int part, uint64_t cell) { return (uint64_t)part << 52 | (cell & kLow52); }
__host__ __device__ inline uint64_t h3_unpack(uint64_t key, int res) {
    return (uint64_t)1 << 59 | (uint64_t)res << 52 | (key & kLow52);
}
__host__ __device__ inline int key_part(uint64_t key) { return (int)(key >> 52); }

struct NotEmpty {
    __host__ __device__ bool operator()(const uint64_t& k) const { return k != kEmpty; }
};

// ---- H3 ----
struct H3Args {
    const double* lat;         // vertices (radians), batch-local
    const double* lon;
    const int64_t* ring_off;   // n_rings + 1
    const int32_t* v_ring;     // vertex -> ring
    const int32_t* ring_part;  // ring -> part (batch-local)
    const int64_t* part_ring;  // n_parts + 1
    const h3fill::Box* ring_box;
    int64_t n_verts;
    int res;
    double pent_r;
    int64_t* edge_n;      // per vertex: lineHexEstimate of the edge starting there
    int64_t* sample_off;  // n_verts + 1
    uint64_t* s_key;      // per sample
    uint64_t* s_slot;
    uint32_t* tab_val;    // min claim per slot (samples and rounds)
    uint64_t* tab_keys;   // claim table (samples / round)
    uint64_t tab_mask;
    uint64_t* out_keys;   // accepted set
    uint64_t out_mask;
    unsigned int* flags;  // bit 1: table overflow, bit 2: result overflow
    int32_t* part_fail;
};

__device__ inline bool inside_part(const H3Args& a, int part, double lat, double lon) {
    const int64_t r0 = a.part_ring[part], r1 = a.part_ring[part + 1];
    const int64_t s0 = a.ring_off[r0];
    if (!h3fill::point_inside_loop(a.lat + s0, a.lon + s0, a.ring_off[r0 + 1] - s0, a.ring_box[r0], lat, lon))
        return false;
    for (int64_t r = r0 + 1; r < r1; r++) {
        const int64_t s = a.ring_off[r];
        if (h3fill::point_inside_loop(a.lat + s, a.lon + s, a.ring_off[r + 1] - s, a.ring_box[r], lat, lon))
            return false;
    }
    return true;
}

__device__ inline int64_t next_vertex(const H3Args& a, int64_t v) {
    const int r = a.v_ring[v];
    return v + 1 == a.ring_off[r + 1] ? a.ring_off[r] : v + 1;
}

__global__ void __launch_bounds__(256) k_pf_edge_count(H3Args a) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < a.n_verts; v += (int64_t)gridDim.x * blockDim.x) {
        const int64_t w = next_vertex(a, v);
        a.edge_n[v] = h3fill::line_hex_estimate(a.lat[v], a.lon[v], a.lat[w], a.lon[w], a.pent_r);
    }
}

__global__ void __launch_bounds__(256) k_pf_edge_sample(H3Args a, int64_t n_samples) {
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n_samples; s += (int64_t)gridDim.x * blockDim.x) {
        int64_t lo = 0, hi = a.n_verts;  // largest v with sample_off[v] <= s
        while (hi - lo > 1) {
            const int64_t m = (lo + hi) / 2;
            if (a.sample_off[m] <= s) lo = m;
            else hi = m;
        }
        const int64_t v = lo, w = next_vertex(a, v);
        const int n = (int)a.edge_n[v], j = (int)(s - a.sample_off[v]);
        double lat, lon;
        h3fill::edge_sample(a.lat[v], a.lon[v], a.lat[w], a.lon[w], n, j, &lat, &lon);
        const uint64_t cell = h3::h3_exact(lat, lon, a.res);
        const uint64_t key = h3_pack(a.ring_part[a.v_ring[v]], cell);
        bool ins;
        const uint64_t slot = tab_insert(a.tab_keys, a.tab_mask, key, &ins, a.flags);
        a.s_key[s] = key;
        a.s_slot[s] = slot;
        if (slot != kEmpty) atomicMin(&a.tab_val[slot], (uint32_t)s);
    }
}

// keep[s] = the sample's key at its cell's first sample, else empty
__global__ void __launch_bounds__(256) k_pf_edge_first(H3Args a, int64_t n_samples, uint64_t* keep) {
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n_samples; s += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t slot = a.s_slot[s];
        keep[s] = (slot != kEmpty && a.tab_val[slot] == (uint32_t)s) ? a.s_key[s] : kEmpty;
    }
}

// kRing(1) of each frontier cell: claims (i * 7 + j) on the cells not yet accepted
__global__ void __launch_bounds__(256) k_pf_expand(H3Args a, const uint64_t* frontier, int64_t f, uint64_t* nb,
                                                   uint64_t* nslot) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < f; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t key = frontier[i];
        const int part = key_part(key);
        int64_t ring[7];
        const int n = h3fill::kring1(h3_unpack(key, a.res), a.res, ring);
        if (n < 0) atomicExch(&a.part_fail[part], 1);
        for (int j = 0; j < 7; j++) {
            uint64_t k2 = kEmpty, slot = kEmpty;
            if (j < n) {
                k2 = h3_pack(part, (uint64_t)ring[j]);
                if (tab_has(a.out_keys, a.out_mask, k2)) {
                    k2 = kEmpty;
                } else {
                    bool ins;
                    slot = tab_insert(a.tab_keys, a.tab_mask, k2, &ins, a.flags);
                    if (slot != kEmpty) atomicMin(&a.tab_val[slot], (uint32_t)(i * 7 + j));
                    else k2 = kEmpty;
                }
            }
            nb[i * 7 + j] = k2;
            nslot[i * 7 + j] = slot;
        }
    }
}

// the first claimant of each cell tests its centre
__global__ void __launch_bounds__(256) k_pf_accept(H3Args a, const uint64_t* nb, const uint64_t* nslot, int64_t m,
                                                   uint64_t* keep) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < m; t += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k2 = nb[t];
        uint64_t out = kEmpty;
        if (k2 != kEmpty && a.tab_val[nslot[t]] == (uint32_t)t) {
            double lat, lon;
            h3geom::h3_to_geo(h3_unpack(k2, a.res), &lat, &lon);
            if (inside_part(a, key_part(k2), lat, lon)) out = k2;
        }
        keep[t] = out;
    }
}

__global__ void __launch_bounds__(256) k_pf_commit(H3Args a, const uint64_t* found, int64_t f, uint64_t* result,
                                                   int64_t r_base, int64_t r_cap) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < f; i += (int64_t)gridDim.x * blockDim.x) {
        bool ins;
        tab_insert(a.out_keys, a.out_mask, found[i], &ins, a.flags);
        if (r_base + i < r_cap) result[r_base + i] = found[i];
        else atomicOr(a.flags, 4u);
    }
}

// maxPolyfillSize per part and the pentagon radius, on the device: the glibc restatement's tables
// (glibc_math.h) are device constants, so a HIP translation unit evaluates them only in kernels
__global__ void __launch_bounds__(256) k_pf_part_m(const h3fill::Box* shell_box, const int64_t* total_verts, int64_t np,
                                                   int res, int64_t* m_out, double* pent_r_out) {
    const double pr = h3fill::pentagon_radius_km(res);
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t == 0) pent_r_out[0] = pr;
    for (int64_t p = t; p < np; p += (int64_t)gridDim.x * blockDim.x) {
        if (total_verts[p] == 0) {
            m_out[p] = 0;
            continue;
        }
        int64_t m = h3fill::bbox_hex_estimate(shell_box[p], pr);
        if (m < total_verts[p]) m = total_verts[p];
        m_out[p] = m + h3fill::kPolyfillBuffer;
    }
}

// ---- BNG ----
struct BngArgs {
    pip::GeomStore store;  // batch-local geometries
    int res;
    uint64_t* visited;
    uint64_t mask;
    uint64_t* next;
    unsigned long long* n_next;
    int64_t next_cap;
    uint64_t* result;
    unsigned long long* n_result;
    int64_t result_cap;
    unsigned int* flags;
};
constexpr int kBngShift = 51;
constexpr uint64_t kBngLow = ((uint64_t)1 << kBngShift) - 1;

__device__ inline void bng_visit(const BngArgs& a, uint64_t key) {
    bool ins;
    tab_insert(a.visited, a.mask, key, &ins, a.flags);
    if (!ins) return;
    const unsigned long long at = atomicAdd(a.n_next, 1ull);
    if ((int64_t)at < a.next_cap) a.next[at] = key;
    else atomicOr(a.flags, 4u);
}

// start points: every vertex (then the centroids, given as extra points with their geometry)
__global__ void __launch_bounds__(256) k_pf_bng_start(BngArgs a, const double* px, const double* py, const int32_t* pg,
                                                      int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t id;
        if (!bng::point_to_index(px[i], py[i], a.res, &id)) {
            atomicOr(a.flags, 8u);  // NaN vertex
            continue;
        }
        bng_visit(a, (uint64_t)pg[i] << kBngShift | ((uint64_t)id & kBngLow));
    }
}

__global__ void __launch_bounds__(256) k_pf_bng_round(BngArgs a, const uint64_t* frontier, int64_t f) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < f; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t key = frontier[i];
        const uint32_t g = (uint32_t)(key >> kBngShift);
        const int64_t id = (int64_t)(key & kBngLow);
        int r;
        int32_t e, x, y;
        if (!bng::cell_origin(id, &r, &e, &x, &y)) continue;
        const double cx = (double)x + (double)e / 2, cy = (double)y + (double)e / 2;
        if (!pip::contains(a.store, g, cx, cy)) continue;
        const unsigned long long at = atomicAdd(a.n_result, 1ull);
        if ((int64_t)at < a.result_cap) a.result[at] = key;
        else atomicOr(a.flags, 4u);
        int64_t nb[8];
        const int m = bng::kloop(id, 1, nb);
        for (int j = 0; j < m; j++) bng_visit(a, (uint64_t)g << kBngShift | ((uint64_t)nb[j] & kBngLow));
    }
}

// ---- host helpers ----
struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
    ~Buf() {
        if (p) (void)hipFree(p);
    }
    int reserve(size_t n) {
        if (n <= bytes) return MOSAIC_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        if (hipMalloc(&p, std::max<size_t>(n, 8)) != hipSuccess)
            return mosaic_tess_fail(MOSAIC_E_NOMEM, ("hipMalloc(" + std::to_string(n) + ") failed").c_str());
        bytes = std::max<size_t>(n, 8);
        return MOSAIC_OK;
    }
    template <class T>
    T* as() const {
        return (T*)p;
    }
};

#define PF_TRY(expr)                                                                                   \
    do {                                                                                               \
        hipError_t _e = (expr);                                                                        \
        if (_e != hipSuccess)                                                                          \
            return mosaic_tess_fail(MOSAIC_E_HIP, (std::string(#expr ": ") + hipGetErrorString(_e)).c_str()); \
    } while (0)
#define PF_RC(expr)              \
    do {                         \
        int _rc = (expr);        \
        if (_rc) return _rc;     \
    } while (0)

template <class T>
int upload(Buf& b, const std::vector<T>& v, hipStream_t s) {
    PF_RC(b.reserve(v.size() * sizeof(T)));
    if (!v.empty()) PF_TRY(hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
    return MOSAIC_OK;
}

uint64_t pow2_at_least(uint64_t n) {
    uint64_t c = 1024;
    while (c < n) c <<= 1;
    return c;
}

int blocks_for(int64_t n, int n_cu) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, (int64_t)n_cu * 16)); }

// Compacts the non-empty keys of in[0, n) into out (order kept); returns the count through *count.
int compact(Buf& tmp, const uint64_t* in, int64_t n, uint64_t* out, Buf& count_buf, int64_t* count, hipStream_t s) {
    PF_RC(count_buf.reserve(8));
    size_t bytes = 0;
    PF_TRY(hipcub::DeviceSelect::If(nullptr, bytes, in, out, count_buf.as<int64_t>(), n, NotEmpty(), s));
    PF_RC(tmp.reserve(bytes));
    bytes = tmp.bytes;
    PF_TRY(hipcub::DeviceSelect::If(tmp.p, bytes, in, out, count_buf.as<int64_t>(), n, NotEmpty(), s));
    PF_TRY(hipMemcpyAsync(count, count_buf.p, 8, hipMemcpyDeviceToHost, s));
    PF_TRY(hipStreamSynchronize(s));
    return MOSAIC_OK;
}

// Scala 2.12 immutable.HashSet iteration order of Long elements: the hash-trie walks 5-bit groups
// of improve(elem.##) from the lowest
uint64_t scala_set_order_key(int64_t v) {
    const int32_t iv = (int32_t)v;
    int32_t hc = (int64_t)iv == v ? iv : (int32_t)(v ^ (int64_t)((uint64_t)v >> 32));
    uint32_t h = (uint32_t)hc;
    h = h + ~(h << 9);
    h = h ^ (h >> 14);
    h = h + (h << 4);
    h = h ^ (h >> 10);
    uint64_t k = 0;
    for (int level = 0; level < 7; level++) k = k << 5 | ((h >> (5 * level)) & 31u);
    return k;
}

// JTS 1.19 Orientation.isCCW of a closed ring
__host__ __device__ inline bool jts_is_ccw(const double* xy, int64_t n) {
    const int64_t npts = n - 1;
    if (npts < 3) return false;
    int64_t up_hi = 0, up_low = -1;
    double prev_y = xy[1], hi_y = xy[1];
    for (int64_t i = 1; i <= npts; i++) {
        const double py = xy[2 * i + 1];
        if (py > prev_y && py >= hi_y) {
            up_hi = i;
            hi_y = py;
            up_low = i - 1;
        }
        prev_y = py;
    }
    if (up_hi == 0) return false;
    int64_t down_low = up_hi;
    do {
        down_low = (down_low + 1) % npts;
    } while (down_low != up_hi && xy[2 * down_low + 1] == hi_y);
    const int64_t down_hi = down_low > 0 ? down_low - 1 : npts - 1;
#define PF_EQ2(a, b) (xy[2 * (a)] == xy[2 * (b)] && xy[2 * (a) + 1] == xy[2 * (b) + 1])
    if (PF_EQ2(up_hi, down_hi)) {
        if (PF_EQ2(up_low, up_hi) || PF_EQ2(down_low, up_hi) || PF_EQ2(up_low, down_low)) return false;
#undef PF_EQ2
        return pip::orientation_index(xy[2 * up_low], xy[2 * up_low + 1], xy[2 * up_hi], xy[2 * up_hi + 1],
                                      xy[2 * down_low], xy[2 * down_low + 1]) == 1;
    }
    return xy[2 * down_hi] - xy[2 * up_hi] < 0;
}

// JTS 1.19 Centroid (area part) of geometry g; false when its area is 0
bool jts_centroid(int64_t g, const int64_t* geom_parts, const int64_t* part_rings, const int64_t* ring_offsets,
                  const double* xy, double* cx, double* cy) {
    double sx = 0, sy = 0, a2 = 0, bx = 0, by = 0;
    for (int64_t p = geom_parts[g]; p < geom_parts[g + 1]; p++)
        for (int64_t r = part_rings[p]; r < part_rings[p + 1]; r++) {
            const double* v = xy + 2 * ring_offsets[r];
            const int64_t n = ring_offsets[r + 1] - ring_offsets[r];
            if (n == 0) continue;
            const bool shell = r == part_rings[p];
            if (shell) {
                bx = v[0];
                by = v[1];
            }
            const bool ccw = jts_is_ccw(v, n);
            const double sign = (shell ? !ccw : ccw) ? 1.0 : -1.0;
            for (int64_t i = 0; i + 1 < n; i++) {
                const double p1x = v[2 * i], p1y = v[2 * i + 1], p2x = v[2 * i + 2], p2y = v[2 * i + 3];
                const double tcx = bx + p1x + p2x, tcy = by + p1y + p2y;
                const double area2 = (p1x - bx) * (p2y - by) - (p2x - bx) * (p1y - by);
                sx += sign * area2 * tcx;
                sy += sign * area2 * tcy;
                a2 += sign * area2;
            }
        }
    if (!(fabs(a2) > 0.0)) return false;
    *cx = sx / 3 / a2;
    *cy = sy / 3 / a2;
    return true;
}

// getBufferRadius (H3IndexSystem.scala:73-80) from the geometry's centroid: the centroid's cell
// (geoToH3 after Math.toRadians), its indexToGeometry ring (h3ToGeoBoundary in degrees, closed with
// the first vertex), that polygon's JTS centroid, and the largest distance (Coordinate.distance) of
// a ring point from it
__global__ void __launch_bounds__(256) k_buffer_radius_h3(const double* cx, const double* cy, const uint8_t* ok,
                                                          int64_t n, int res, int jdk, double* out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!ok[i]) {
            out[i] = NAN;
            continue;
        }
        const uint64_t cell = h3::h3_exact(h3::to_radians(cy[i], jdk), h3::to_radians(cx[i], jdk), res);
        double v[20], xy[22];
        const int nv = h3geom::h3_to_geo_boundary(cell, v);
        if (nv <= 0) {
            out[i] = NAN;
            continue;
        }
        for (int k = 0; k < nv; k++) {
            xy[2 * k] = h3geom::to_degrees(v[2 * k + 1], jdk);
            xy[2 * k + 1] = h3geom::to_degrees(v[2 * k], jdk);
        }
        xy[2 * nv] = xy[0];
        xy[2 * nv + 1] = xy[1];
        const int64_t m = nv + 1;
        // JTS Centroid of the polygon (shell only)
        const double bx = xy[0], by = xy[1];
        const double sign = !jts_is_ccw(xy, m) ? 1.0 : -1.0;
        double sx = 0, sy = 0, a2 = 0;
        for (int64_t k = 0; k + 1 < m; k++) {
            const double p1x = xy[2 * k], p1y = xy[2 * k + 1], p2x = xy[2 * k + 2], p2y = xy[2 * k + 3];
            const double area2 = (p1x - bx) * (p2y - by) - (p2x - bx) * (p1y - by);
            sx += sign * area2 * (bx + p1x + p2x);
            sy += sign * area2 * (by + p1y + p2y);
            a2 += sign * area2;
        }
        const double gx = sx / 3 / a2, gy = sy / 3 / a2;
        double r = 0;
        for (int64_t k = 0; k < m; k++) {
            const double dx = xy[2 * k] - gx, dy = xy[2 * k + 1] - gy;
            const double d = sqrt(dx * dx + dy * dy);
            r = d > r ? d : r;
        }
        out[i] = r;
    }
}

struct Input {
    int64_t n_geoms;
    const int64_t *geom_parts, *part_rings, *ring_offsets;
    const double* xy;
};

// H3: parts [p0, p1) of the input (one batch); appends each part's cells (H3 output order) to
// part_cells[p - p0] and sets part_bad[p - p0]
int h3_batch(hipStream_t st, int n_cu, int jdk, int res, const Input& in, int64_t p0, int64_t p1,
             std::vector<std::vector<int64_t>>& part_cells, std::vector<char>& part_bad, double* kernel_ms) {
    const int64_t np = p1 - p0;
    // host: radians, ring boxes (no libm), per-part shell box and vertex count
    std::vector<int64_t> ring_off{0}, part_ring{0}, part_total(np, 0);
    std::vector<int32_t> v_ring, ring_part;
    std::vector<double> lat, lon;
    std::vector<h3fill::Box> boxes, shell_box(np, h3fill::Box{0, 0, 0, 0});
    for (int64_t p = p0; p < p1; p++) {
        const int64_t r0 = in.part_rings[p], r1 = in.part_rings[p + 1];
        bool empty = r1 == r0 || in.ring_offsets[r0 + 1] == in.ring_offsets[r0];
        bool finite = true;
        for (int64_t v = in.ring_offsets[r0]; !empty && v < in.ring_offsets[r1]; v++)
            finite &= std::isfinite(in.xy[2 * v]) && std::isfinite(in.xy[2 * v + 1]);
        if (empty || !finite) {
            part_bad[p - p0] = !finite;
            part_ring.push_back(part_ring.back());
            continue;
        }
        int64_t total = 0;
        for (int64_t r = r0; r < r1; r++) {
            const int64_t s = (int64_t)lat.size();
            for (int64_t v = in.ring_offsets[r]; v < in.ring_offsets[r + 1]; v++) {
                lat.push_back(h3::to_radians(in.xy[2 * v + 1], jdk));
                lon.push_back(h3::to_radians(in.xy[2 * v], jdk));
                v_ring.push_back((int32_t)ring_part.size());
            }
            const int64_t n = (int64_t)lat.size() - s;
            total += n;
            boxes.push_back(h3fill::bbox_from_loop(lat.data() + s, lon.data() + s, n));
            ring_part.push_back((int32_t)(p - p0));
            ring_off.push_back((int64_t)lat.size());
        }
        shell_box[p - p0] = boxes[part_ring.back()];
        part_ring.push_back((int64_t)ring_part.size());
        part_total[p - p0] = total;
    }
    const int64_t nv = (int64_t)lat.size();
    if (nv == 0) return MOSAIC_OK;
    if (nv >= ((int64_t)1 << 31)) return mosaic_tess_fail(MOSAIC_E_CAPACITY, "polyfill: too many vertices in a batch");
    std::vector<int64_t> part_m(np, 0);
    double pent_r = 0;
    {
        Buf d_sb, d_tot, d_m, d_pr;
        PF_RC(upload(d_sb, shell_box, st));
        PF_RC(upload(d_tot, part_total, st));
        PF_RC(d_m.reserve((size_t)np * 8));
        PF_RC(d_pr.reserve(8));
        hipLaunchKernelGGL(k_pf_part_m, dim3(blocks_for(np, n_cu)), dim3(256), 0, st, d_sb.as<h3fill::Box>(),
                           d_tot.as<int64_t>(), np, res, d_m.as<int64_t>(), d_pr.as<double>());
        PF_TRY(hipGetLastError());
        PF_TRY(hipMemcpyAsync(part_m.data(), d_m.p, (size_t)np * 8, hipMemcpyDeviceToHost, st));
        PF_TRY(hipMemcpyAsync(&pent_r, d_pr.p, 8, hipMemcpyDeviceToHost, st));
        PF_TRY(hipStreamSynchronize(st));
    }
    uint64_t m_sum = 0;
    for (int64_t m : part_m) m_sum += (uint64_t)m;
    Buf d_lat, d_lon, d_roff, d_vring, d_rpart, d_pring, d_box, d_en, d_soff, d_flags, d_fail, d_tmp, d_cnt;
    PF_RC(upload(d_lat, lat, st));
    PF_RC(upload(d_lon, lon, st));
    PF_RC(upload(d_roff, ring_off, st));
    PF_RC(upload(d_vring, v_ring, st));
    PF_RC(upload(d_rpart, ring_part, st));
    PF_RC(upload(d_pring, part_ring, st));
    PF_RC(upload(d_box, boxes, st));
    PF_RC(d_en.reserve((size_t)nv * 8));
    PF_RC(d_soff.reserve((size_t)(nv + 1) * 8));
    PF_RC(d_flags.reserve(4));
    PF_RC(d_fail.reserve((size_t)np * 4));
    PF_TRY(hipMemsetAsync(d_flags.p, 0, 4, st));
    PF_TRY(hipMemsetAsync(d_fail.p, 0, (size_t)np * 4, st));
    H3Args a{};
    a.lat = d_lat.as<double>();
    a.lon = d_lon.as<double>();
    a.ring_off = d_roff.as<int64_t>();
    a.v_ring = d_vring.as<int32_t>();
    a.ring_part = d_rpart.as<int32_t>();
    a.part_ring = d_pring.as<int64_t>();
    a.ring_box = d_box.as<h3fill::Box>();
    a.n_verts = nv;
    a.res = res;
    a.pent_r = pent_r;
    a.edge_n = d_en.as<int64_t>();
    a.sample_off = d_soff.as<int64_t>();
    a.flags = d_flags.as<unsigned int>();
    a.part_fail = d_fail.as<int32_t>();
    hipEvent_t e0, e1;
    PF_TRY(hipEventCreate(&e0));
    PF_TRY(hipEventCreate(&e1));
    struct EvGuard {
        hipEvent_t a, b;
        ~EvGuard() {
            (void)hipEventDestroy(a);
            (void)hipEventDestroy(b);
        }
    } evg{e0, e1};
    PF_TRY(hipEventRecord(e0, st));
    // 1. edge samples -> first frontier
    hipLaunchKernelGGL(k_pf_edge_count, dim3(blocks_for(nv, n_cu)), dim3(256), 0, st, a);
    PF_TRY(hipGetLastError());
    PF_TRY(hipMemsetAsync(a.sample_off, 0, 8, st));
    {
        size_t bytes = 0;
        PF_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, bytes, a.edge_n, a.sample_off + 1, nv, st));
        PF_RC(d_tmp.reserve(bytes));
        bytes = d_tmp.bytes;
        PF_TRY(hipcub::DeviceScan::InclusiveSum(d_tmp.p, bytes, a.edge_n, a.sample_off + 1, nv, st));
    }
    int64_t n_samples = 0;
    PF_TRY(hipMemcpyAsync(&n_samples, a.sample_off + nv, 8, hipMemcpyDeviceToHost, st));
    PF_TRY(hipStreamSynchronize(st));
    if (n_samples >= ((int64_t)1 << 31)) return mosaic_tess_fail(MOSAIC_E_CAPACITY, "polyfill: too many edge samples");
    Buf d_skey, d_sslot, d_tkeys, d_tval, d_keep, d_front, d_nb, d_nslot, d_okeys, d_result;
    PF_RC(d_skey.reserve((size_t)n_samples * 8));
    PF_RC(d_sslot.reserve((size_t)n_samples * 8));
    PF_RC(d_keep.reserve((size_t)n_samples * 8));
    PF_RC(d_front.reserve((size_t)n_samples * 8));
    uint64_t tcap = pow2_at_least(2 * (uint64_t)n_samples);
    PF_RC(d_tkeys.reserve(tcap * 8));
    PF_RC(d_tval.reserve(tcap * 4));
    PF_TRY(hipMemsetAsync(d_tkeys.p, 0xff, tcap * 8, st));
    PF_TRY(hipMemsetAsync(d_tval.p, 0xff, tcap * 4, st));
    a.s_key = d_skey.as<uint64_t>();
    a.s_slot = d_sslot.as<uint64_t>();
    a.tab_keys = d_tkeys.as<uint64_t>();
    a.tab_val = d_tval.as<uint32_t>();
    a.tab_mask = tcap - 1;
    hipLaunchKernelGGL(k_pf_edge_sample, dim3(blocks_for(n_samples, n_cu)), dim3(256), 0, st, a, n_samples);
    PF_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_pf_edge_first, dim3(blocks_for(n_samples, n_cu)), dim3(256), 0, st, a, n_samples,
                       d_keep.as<uint64_t>());
    PF_TRY(hipGetLastError());
    int64_t f = 0;
    PF_RC(compact(d_tmp, d_keep.as<uint64_t>(), n_samples, d_front.as<uint64_t>(), d_cnt, &f, st));
    // 2. breadth-first rounds
    const uint64_t ocap = pow2_at_least(2 * m_sum);
    if (ocap > ((uint64_t)1 << 31)) return mosaic_tess_fail(MOSAIC_E_CAPACITY, "polyfill: result too large for one call");
    PF_RC(d_okeys.reserve(ocap * 8));
    PF_TRY(hipMemsetAsync(d_okeys.p, 0xff, ocap * 8, st));
    PF_RC(d_result.reserve(m_sum * 8));
    a.out_keys = d_okeys.as<uint64_t>();
    a.out_mask = ocap - 1;
    int64_t r_total = 0;
    while (f > 0) {
        const int64_t m = 7 * f;
        PF_RC(d_nb.reserve((size_t)m * 8));
        PF_RC(d_nslot.reserve((size_t)m * 8));
        if (d_keep.bytes < (size_t)m * 8) PF_RC(d_keep.reserve((size_t)m * 8));
        const uint64_t need = pow2_at_least(2 * (uint64_t)m);
        if (need > tcap) {
            tcap = need;
            PF_RC(d_tkeys.reserve(tcap * 8));
            PF_RC(d_tval.reserve(tcap * 4));
        }
        a.tab_keys = d_tkeys.as<uint64_t>();
        a.tab_val = d_tval.as<uint32_t>();
        a.tab_mask = need - 1;
        PF_TRY(hipMemsetAsync(d_tkeys.p, 0xff, need * 8, st));
        PF_TRY(hipMemsetAsync(d_tval.p, 0xff, need * 4, st));
        hipLaunchKernelGGL(k_pf_expand, dim3(blocks_for(f, n_cu)), dim3(256), 0, st, a, d_front.as<uint64_t>(), f,
                           d_nb.as<uint64_t>(), d_nslot.as<uint64_t>());
        PF_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_pf_accept, dim3(blocks_for(m, n_cu)), dim3(256), 0, st, a, d_nb.as<uint64_t>(),
                           d_nslot.as<uint64_t>(), m, d_keep.as<uint64_t>());
        PF_TRY(hipGetLastError());
        if (d_front.bytes < (size_t)m * 8) PF_RC(d_front.reserve((size_t)m * 8));
        PF_RC(compact(d_tmp, d_keep.as<uint64_t>(), m, d_front.as<uint64_t>(), d_cnt, &f, st));
        if (f > 0) {
            hipLaunchKernelGGL(k_pf_commit, dim3(blocks_for(f, n_cu)), dim3(256), 0, st, a, d_front.as<uint64_t>(), f,
                               d_result.as<uint64_t>(), r_total, (int64_t)m_sum);
            PF_TRY(hipGetLastError());
        }
        r_total += f;
        if (r_total > (int64_t)m_sum) break;
    }
    PF_TRY(hipEventRecord(e1, st));
    unsigned int flags = 0;
    std::vector<int32_t> fails(np);
    std::vector<uint64_t> result((size_t)std::min<int64_t>(r_total, (int64_t)m_sum));
    PF_TRY(hipMemcpyAsync(&flags, d_flags.p, 4, hipMemcpyDeviceToHost, st));
    PF_TRY(hipMemcpyAsync(fails.data(), d_fail.p, (size_t)np * 4, hipMemcpyDeviceToHost, st));
    if (!result.empty())
        PF_TRY(hipMemcpyAsync(result.data(), d_result.p, result.size() * 8, hipMemcpyDeviceToHost, st));
    PF_TRY(hipStreamSynchronize(st));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    *kernel_ms += ms;
    if (flags & 2u) return mosaic_tess_fail(MOSAIC_E_CAPACITY, "polyfill: device hash table overflow");
    if ((flags & 4u) || r_total > (int64_t)m_sum)
        return mosaic_tess_fail(MOSAIC_E_CAPACITY, "polyfill: more cells than maxPolyfillSize");
    // 3. H3's output table order per part
    std::vector<std::vector<uint64_t>> seq(np);
    for (uint64_t k : result) seq[key_part(k)].push_back(h3_unpack(k, res));
    for (int64_t q = 0; q < np; q++) {
        if (fails[q]) part_bad[q] = 1;
        if (part_bad[q] || seq[q].empty()) continue;
        const uint64_t M = (uint64_t)part_m[q];
        // H3 v3.7 _polyfillInternal gives up when its table of maxPolyfillSize slots is full (its
        // probe loop stops at loopCount > numHexagons) and polyfill returns no cells for the part;
        // the placement below would otherwise probe forever
        if (seq[q].size() > M) continue;
        std::unordered_set<uint64_t> used;
        used.reserve(seq[q].size() * 2);
        std::vector<std::pair<uint64_t, uint64_t>> placed;
        placed.reserve(seq[q].size());
        for (uint64_t cell : seq[q]) {
            uint64_t loc = cell % M;
            while (used.count(loc)) loc = (loc + 1) % M;
            used.insert(loc);
            placed.emplace_back(loc, cell);
        }
        std::sort(placed.begin(), placed.end());
        auto& out = part_cells[q];
        out.reserve(placed.size());
        for (auto& pc : placed) out.push_back((int64_t)pc.second);
    }
    return MOSAIC_OK;
}

// BNG: geometries [g0, g1) (one batch); appends each geometry's cells to cells[g - g0]
int bng_batch(hipStream_t st, int n_cu, int res, const Input& in, int64_t g0, int64_t g1,
              std::vector<std::vector<int64_t>>& cells, std::vector<char>& bad, double* kernel_ms) {
    const int64_t ng = g1 - g0;
    // pip store of the batch (pip_device.h layout) + start points
    std::vector<pip::Vec2> verts;
    std::vector<uint32_t> ring_start{0}, part_ring{0}, geom_part{0};
    std::vector<pip::Box> ring_box, geom_box;
    std::vector<double> px, py;
    std::vector<int32_t> pg;
    uint64_t visit_bound = 0;
    const double e = (double)bng::edge_size(res);
    for (int64_t g = g0; g < g1; g++) {
        pip::Box gb{INFINITY, INFINITY, -INFINITY, -INFINITY};
        const int64_t v0 = in.ring_offsets[in.part_rings[in.geom_parts[g]]];
        const int64_t v1 = in.ring_offsets[in.part_rings[in.geom_parts[g + 1]]];
        double cx = 0, cy = 0;
        const bool has = v1 > v0 && jts_centroid(g, in.geom_parts, in.part_rings, in.ring_offsets, in.xy, &cx, &cy);
        if (v1 > v0 && !has) bad[g - g0] = 1;  // no area (the reference would take a line centroid)
        for (int64_t p = in.geom_parts[g]; has && p < in.geom_parts[g + 1]; p++) {
            for (int64_t r = in.part_rings[p]; r < in.part_rings[p + 1]; r++) {
                pip::Box rb{INFINITY, INFINITY, -INFINITY, -INFINITY};
                for (int64_t v = in.ring_offsets[r]; v < in.ring_offsets[r + 1]; v++) {
                    const double x = in.xy[2 * v], y = in.xy[2 * v + 1];
                    verts.push_back({x, y});
                    rb.minx = std::min(rb.minx, x);
                    rb.maxx = std::max(rb.maxx, x);
                    rb.miny = std::min(rb.miny, y);
                    rb.maxy = std::max(rb.maxy, y);
                    px.push_back(x);
                    py.push_back(y);
                    pg.push_back((int32_t)(g - g0));
                }
                ring_box.push_back(rb);
                ring_start.push_back((uint32_t)verts.size());
                gb.minx = std::min(gb.minx, rb.minx);
                gb.maxx = std::max(gb.maxx, rb.maxx);
                gb.miny = std::min(gb.miny, rb.miny);
                gb.maxy = std::max(gb.maxy, rb.maxy);
            }
            part_ring.push_back((uint32_t)ring_box.size());
        }
        if (has) {
            px.push_back(cx);
            py.push_back(cy);
            pg.push_back((int32_t)(g - g0));
            // visited cells lie within one cell of the bbox (accepted centres are inside it)
            const double w = (gb.maxx - gb.minx) / e + 3, h = (gb.maxy - gb.miny) / e + 3;
            if (!(w * h < 4e9)) return mosaic_tess_fail(MOSAIC_E_CAPACITY, "polyfill: geometry too large for BNG res");
            visit_bound += (uint64_t)(w * h) + 2;
        }
        geom_part.push_back((uint32_t)(part_ring.size() - 1));
        geom_box.push_back(gb);
    }
    if (verts.size() >= ((size_t)1 << 32)) return mosaic_tess_fail(MOSAIC_E_CAPACITY, "polyfill: too many vertices");
    if (px.empty()) return MOSAIC_OK;
    const uint64_t vcap = pow2_at_least(2 * visit_bound);
    if (vcap > ((uint64_t)1 << 31)) return mosaic_tess_fail(MOSAIC_E_CAPACITY, "polyfill: result too large for one call");
    Buf d_verts, d_rs, d_rb, d_pr, d_gp, d_gb, d_px, d_py, d_pg, d_vis, d_f0, d_f1, d_res, d_cnt, d_flags;
    PF_RC(upload(d_verts, verts, st));
    PF_RC(upload(d_rs, ring_start, st));
    PF_RC(upload(d_rb, ring_box, st));
    PF_RC(upload(d_pr, part_ring, st));
    PF_RC(upload(d_gp, geom_part, st));
    PF_RC(upload(d_gb, geom_box, st));
    PF_RC(upload(d_px, px, st));
    PF_RC(upload(d_py, py, st));
    PF_RC(upload(d_pg, pg, st));
    PF_RC(d_vis.reserve(vcap * 8));
    PF_RC(d_f0.reserve(visit_bound * 8));
    PF_RC(d_f1.reserve(visit_bound * 8));
    PF_RC(d_res.reserve(visit_bound * 8));
    PF_RC(d_cnt.reserve(16));
    PF_RC(d_flags.reserve(4));
    PF_TRY(hipMemsetAsync(d_vis.p, 0xff, vcap * 8, st));
    PF_TRY(hipMemsetAsync(d_cnt.p, 0, 16, st));
    PF_TRY(hipMemsetAsync(d_flags.p, 0, 4, st));
    BngArgs a{};
    a.store = pip::GeomStore{d_verts.as<pip::Vec2>(), d_rs.as<uint32_t>(), d_rb.as<pip::Box>(), d_pr.as<uint32_t>(),
                             d_gp.as<uint32_t>(), d_gb.as<pip::Box>()};
    a.res = res;
    a.visited = d_vis.as<uint64_t>();
    a.mask = vcap - 1;
    a.next_cap = (int64_t)visit_bound;
    a.result = d_res.as<uint64_t>();
    a.n_result = d_cnt.as<unsigned long long>() + 1;
    a.result_cap = (int64_t)visit_bound;
    a.flags = d_flags.as<unsigned int>();
    hipEvent_t e0, e1;
    PF_TRY(hipEventCreate(&e0));
    PF_TRY(hipEventCreate(&e1));
    struct EvGuard {
        hipEvent_t a, b;
        ~EvGuard() {
            (void)hipEventDestroy(a);
            (void)hipEventDestroy(b);
        }
    } evg{e0, e1};
    PF_TRY(hipEventRecord(e0, st));
    Buf* cur = &d_f0;
    Buf* nxt = &d_f1;
    a.next = cur->as<uint64_t>();
    a.n_next = d_cnt.as<unsigned long long>();
    const int64_t np = (int64_t)px.size();
    hipLaunchKernelGGL(k_pf_bng_start, dim3(blocks_for(np, n_cu)), dim3(256), 0, st, a, d_px.as<double>(),
                       d_py.as<double>(), d_pg.as<int32_t>(), np);
    PF_TRY(hipGetLastError());
    unsigned long long f = 0;
    PF_TRY(hipMemcpyAsync(&f, d_cnt.p, 8, hipMemcpyDeviceToHost, st));
    PF_TRY(hipStreamSynchronize(st));
    while (f > 0 && (int64_t)f <= a.next_cap) {
        PF_TRY(hipMemsetAsync(d_cnt.p, 0, 8, st));
        a.next = nxt->as<uint64_t>();
        hipLaunchKernelGGL(k_pf_bng_round, dim3(blocks_for((int64_t)f, n_cu)), dim3(256), 0, st, a,
                           cur->as<uint64_t>(), (int64_t)f);
        PF_TRY(hipGetLastError());
        PF_TRY(hipMemcpyAsync(&f, d_cnt.p, 8, hipMemcpyDeviceToHost, st));
        PF_TRY(hipStreamSynchronize(st));
        std::swap(cur, nxt);
    }
    PF_TRY(hipEventRecord(e1, st));
    unsigned int flags = 0;
    unsigned long long n_res = 0;
    PF_TRY(hipMemcpyAsync(&flags, d_flags.p, 4, hipMemcpyDeviceToHost, st));
    PF_TRY(hipMemcpyAsync(&n_res, (char*)d_cnt.p + 8, 8, hipMemcpyDeviceToHost, st));
    PF_TRY(hipStreamSynchronize(st));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    *kernel_ms += ms;
    if (flags & 8u) return mosaic_tess_fail(MOSAIC_E_NAN, "NaN coordinates are not supported.");
    if ((flags & 6u) || (int64_t)n_res > a.result_cap)
        return mosaic_tess_fail(MOSAIC_E_CAPACITY, "polyfill: device table overflow");
    std::vector<uint64_t> result((size_t)n_res);
    if (n_res) PF_TRY(hipMemcpy(result.data(), d_res.p, (size_t)n_res * 8, hipMemcpyDeviceToHost));
    for (uint64_t k : result) cells[(size_t)(k >> kBngShift)].push_back((int64_t)(k & kBngLow));
    for (auto& v : cells) {
        std::vector<std::pair<uint64_t, int64_t>> o;
        o.reserve(v.size());
        for (int64_t id : v) o.emplace_back(scala_set_order_key(id), id);
        std::sort(o.begin(), o.end());
        for (size_t i = 0; i < o.size(); i++) v[i] = o[i].second;
    }
    return MOSAIC_OK;
}

thread_local double g_last_polyfill_ms = 0;

}  // namespace

extern "C" {

int mosaic_polyfill(mosaic_ctx* ctx, int grid, int res, int64_t n_geoms, const int64_t* geom_parts,
                    const int64_t* part_rings, const int64_t* ring_offsets, const double* xy, mosaic_cell_lists** out) {
    if (!ctx || !out || n_geoms < 0 || (n_geoms > 0 && (!geom_parts || !part_rings || !ring_offsets)))
        return mosaic_tess_fail(MOSAIC_E_ARG, "invalid argument");
    *out = nullptr;
    if (grid == MOSAIC_GRID_H3 ? (res < 0 || res > 15) : (grid == MOSAIC_GRID_BNG ? !bng::valid_resolution(res) : true))
        return mosaic_tess_fail(grid == MOSAIC_GRID_H3 || grid == MOSAIC_GRID_BNG ? MOSAIC_E_RES : MOSAIC_E_ARG,
                                "invalid grid or resolution");
    int device = 0, jdk = 8, n_cu = 256;
    void* stream = nullptr;
    PF_RC(mosaic_ctx_exec(ctx, &device, &stream, &jdk, &n_cu));
    hipStream_t st = (hipStream_t)stream;
    const Input in{n_geoms, geom_parts, part_rings, ring_offsets, xy};
    std::unique_ptr<mosaic_cell_lists> lists(new mosaic_cell_lists());
    lists->status.assign((size_t)n_geoms, MOSAIC_POLYFILL_OK);
    double ms = 0;
    if (grid == MOSAIC_GRID_H3) {
        const int64_t n_parts = n_geoms > 0 ? geom_parts[n_geoms] - geom_parts[0] : 0;
        const int64_t pbase = n_geoms > 0 ? geom_parts[0] : 0;
        std::vector<std::vector<int64_t>> part_cells((size_t)n_parts);
        std::vector<char> part_bad((size_t)n_parts, 0);
        for (int64_t b = 0; b < n_parts; b += kBatch) {
            const int64_t e = std::min(n_parts, b + kBatch);
            std::vector<std::vector<int64_t>> pc((size_t)(e - b));
            std::vector<char> pb((size_t)(e - b), 0);
            PF_RC(h3_batch(st, n_cu, jdk, res, in, pbase + b, pbase + e, pc, pb, &ms));
            for (int64_t q = b; q < e; q++) {
                part_cells[q].swap(pc[q - b]);
                part_bad[q] = pb[q - b];
            }
        }
        for (int64_t g = 0; g < n_geoms; g++) {
            bool bad = false;
            for (int64_t p = geom_parts[g]; p < geom_parts[g + 1]; p++) bad |= part_bad[p - pbase] != 0;
            if (bad) {
                lists->status[g] = MOSAIC_POLYFILL_UNSUPPORTED;
            } else {
                for (int64_t p = geom_parts[g]; p < geom_parts[g + 1]; p++)
                    lists->cells.insert(lists->cells.end(), part_cells[p - pbase].begin(), part_cells[p - pbase].end());
            }
            lists->offsets.push_back((int64_t)lists->cells.size());
        }
    } else {
        for (int64_t b = 0; b < n_geoms; b += kBatch) {
            const int64_t e = std::min(n_geoms, b + kBatch);
            std::vector<std::vector<int64_t>> gc((size_t)(e - b));
            std::vector<char> gb((size_t)(e - b), 0);
            PF_RC(bng_batch(st, n_cu, res, in, b, e, gc, gb, &ms));
            for (int64_t g = b; g < e; g++) {
                if (gb[g - b]) lists->status[g] = MOSAIC_POLYFILL_UNSUPPORTED;
                else lists->cells.insert(lists->cells.end(), gc[g - b].begin(), gc[g - b].end());
                lists->offsets.push_back((int64_t)lists->cells.size());
            }
        }
    }
    g_last_polyfill_ms = ms;
    *out = lists.release();
    return MOSAIC_OK;
}

int mosaic_cell_lists_info(const mosaic_cell_lists* l, int64_t* n_rows, int64_t* n_cells) {
    if (!l) return mosaic_tess_fail(MOSAIC_E_ARG, "null cell lists");
    if (n_rows) *n_rows = (int64_t)l->status.size();
    if (n_cells) *n_cells = (int64_t)l->cells.size();
    return MOSAIC_OK;
}

int mosaic_cell_lists_export(const mosaic_cell_lists* l, int64_t* offsets, int64_t* cells, int32_t* status) {
    if (!l) return mosaic_tess_fail(MOSAIC_E_ARG, "null cell lists");
    if (offsets) std::copy(l->offsets.begin(), l->offsets.end(), offsets);
    if (cells) std::copy(l->cells.begin(), l->cells.end(), cells);
    if (status) std::copy(l->status.begin(), l->status.end(), status);
    return MOSAIC_OK;
}

int mosaic_cell_lists_destroy(mosaic_cell_lists* l) {
    delete l;
    return MOSAIC_OK;
}

double mosaic_polyfill_last_ms(void) { return g_last_polyfill_ms; }

int mosaic_buffer_radius(mosaic_ctx* ctx, int grid, int res, int64_t n_geoms, const int64_t* geom_parts,
                         const int64_t* part_rings, const int64_t* ring_offsets, const double* xy, double* out) {
    if (!ctx || !out || n_geoms < 0 || (n_geoms > 0 && (!geom_parts || !part_rings || !ring_offsets)))
        return mosaic_tess_fail(MOSAIC_E_ARG, "invalid argument");
    if (grid == MOSAIC_GRID_BNG) {
        if (!bng::valid_resolution(res)) return mosaic_tess_fail(MOSAIC_E_RES, "invalid BNG resolution");
        const double r = (double)bng::edge_size(res) * 1.4142135623730951 / 2;  // size * math.sqrt(2) / 2
        for (int64_t g = 0; g < n_geoms; g++) out[g] = r;
        return MOSAIC_OK;
    }
    if (grid != MOSAIC_GRID_H3 || res < 0 || res > 15)
        return mosaic_tess_fail(grid == MOSAIC_GRID_H3 ? MOSAIC_E_RES : MOSAIC_E_ARG, "invalid grid or resolution");
    if (n_geoms == 0) return MOSAIC_OK;
    int device = 0, jdk = 8, n_cu = 256;
    void* stream = nullptr;
    PF_RC(mosaic_ctx_exec(ctx, &device, &stream, &jdk, &n_cu));
    hipStream_t st = (hipStream_t)stream;
    std::vector<double> cx((size_t)n_geoms, 0), cy((size_t)n_geoms, 0);
    std::vector<uint8_t> ok((size_t)n_geoms, 0);
    for (int64_t g = 0; g < n_geoms; g++)
        ok[g] = jts_centroid(g, geom_parts, part_rings, ring_offsets, xy, &cx[g], &cy[g]) ? 1 : 0;
    Buf d_cx, d_cy, d_ok, d_out;
    PF_RC(upload(d_cx, cx, st));
    PF_RC(upload(d_cy, cy, st));
    PF_RC(upload(d_ok, ok, st));
    PF_RC(d_out.reserve((size_t)n_geoms * 8));
    hipLaunchKernelGGL(k_buffer_radius_h3, dim3(blocks_for(n_geoms, n_cu)), dim3(256), 0, st, d_cx.as<double>(),
                       d_cy.as<double>(), d_ok.as<uint8_t>(), n_geoms, res, jdk, d_out.as<double>());
    PF_TRY(hipGetLastError());
    PF_TRY(hipMemcpyAsync(out, d_out.p, (size_t)n_geoms * 8, hipMemcpyDeviceToHost, st));
    PF_TRY(hipStreamSynchronize(st));
    return MOSAIC_OK;
}

}  // extern "C"
