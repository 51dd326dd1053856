// Chip production (the build side of the chip join) on the host: grid_tessellateexplode.
//
// Reference: MosaicExplode.eval (expressions/index/MosaicExplode.scala:70-79) -> Mosaic.getChips /
// mosaicFill (core/Mosaic.scala:21-87) -> IndexSystem.getBorderChips / getCoreChips
// (core/index/IndexSystem.scala:152-186).  The reference carves the polygon with JTS
// buffer(-radius), polyfills, and intersects border cells with JTS overlay.  This producer reaches
// the same contract -- every cell that meets the polygon gets one chip; a core chip's cell lies in
// the polygon's interior (so its points are accepted without a test); a border chip carries
// polygon n cell -- by exact per-cell classification instead:
//   * H3: the polygon is projected into its icosahedron face's gnomonic hex2d plane at the target
//     resolution (where H3 cells are exact hexagons); candidate lattice cells come from the
//     projected bounding box; each ring is clipped against the convex hexagon (Sutherland-Hodgman)
//     and clip vertices are mapped back to lon/lat.  Original polygon vertices are kept bit-exact.
//     Hexagon edges are densified (H3 cell edges are great-circle arcs; straight lon/lat chords
//     would leave slivers).  Cell ids are _faceIjkToH3 of the lattice cell (h3_device.h).
//   * BNG: cells are axis-aligned squares in the native plane; same clipping.
// Polygons spanning icosahedron faces are cut into per-face pieces (tessellate_h3_multiface); the
// GPU producer (mosaic_tessellate_gpu) classifies and clips single-face geometries on the device and
// runs the same host routine for face-spanning ones, so both give the same chip set.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <string>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/mosaic_hip.h"
#include "tess_gpu.h"
#include "bng_device.h"
#include "h3_device.h"
#include "h3_geom.h"
#include "isect_geom.h"
#include "llclip.h"

#include <unordered_map>

using namespace mosaic;

extern "C" int mosaic_tess_fail(int code, const char* msg);  // defined in mosaic_hip.hip
extern "C" int mosaic_tess_classify_bng(mosaic_ctx* c, int64_t n_geoms, const int64_t* geom_parts,
                                        const int64_t* part_rings, const int64_t* ring_offsets, const double* xy,
                                        int64_t n_cand, const int32_t* cand_geom, const int64_t* cand_ij, double e,
                                        double eps, uint8_t* cls);  // mosaic_hip.hip
extern "C" int mosaic_tess_classify_poly(mosaic_ctx* c, int64_t n_geoms, const int64_t* geom_parts,
                                         const int64_t* part_rings, const int64_t* ring_offsets, const double* xy,
                                         int64_t n_cand, const int32_t* cand_geom, const double* clip, int nv,
                                         double eps, uint8_t* cls);  // mosaic_hip.hip

namespace {

// phase trace (measurement only): MOSAIC_BUILD_TRACE=1 prints phase wall times to stderr
struct TessTrace {
    bool on = getenv("MOSAIC_BUILD_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    double acc[6] = {0, 0, 0, 0, 0, 0};
    void mark(const char* what) {
        if (!on) return;
        fprintf(stderr, "[tess] %-28s %8.3f ms\n", what,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count());
        t = std::chrono::steady_clock::now();
    }
    void add(int k) {  // accumulate the time since the last mark into acc[k]
        if (!on) return;
        acc[k] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
        t = std::chrono::steady_clock::now();
    }
};

struct P2 {
    double x, y;
};

// ---- H3 face-plane helpers (host) ----
struct FacePlane {
    int face, res;
    const double *fc, *ei, *ep;
    double S;
    void init(int f, int r) {
        face = f;
        res = r;
        const double* b = h3::kH3FastBasis[f];
        fc = b;
        ei = b + ((r & 1) ? 9 : 3);
        ep = b + ((r & 1) ? 12 : 6);
        S = h3::kH3FastScale[r];
    }
    static void unit(double lon_deg, double lat_deg, double p[3]) {
        double la = lat_deg * (M_PI / 180.0), lo = lon_deg * (M_PI / 180.0);
        p[0] = cos(lo) * cos(la);
        p[1] = sin(lo) * cos(la);
        p[2] = sin(la);
    }
    P2 to_hex(double lon, double lat) const {
        double p[3];
        unit(lon, lat, p);
        return to_hex_unit(p);
    }
    P2 to_hex_unit(const double p[3]) const {
        double d = fc[0] * p[0] + fc[1] * p[1] + fc[2] * p[2];
        return {S * (ei[0] * p[0] + ei[1] * p[1] + ei[2] * p[2]) / d, S * (ep[0] * p[0] + ep[1] * p[1] + ep[2] * p[2]) / d};
    }
    P2 to_geo(P2 h) const {
        double t[3];
        for (int k = 0; k < 3; k++) t[k] = fc[k] + (h.x * ei[k] + h.y * ep[k]) / S;
        // (latitude as atan2(z, |xy|): the same function as the longitude, so the GPU clipper's
        // restatement of glibc atan2 (glibc_math.h) maps computed vertices bit for bit)
        return {atan2(t[1], t[0]) * (180.0 / M_PI), atan2(t[2], sqrt(t[0] * t[0] + t[1] * t[1])) * (180.0 / M_PI)};
    }
};

int face_of_unit(const double p[3]) {
    int best = 0;
    double bd = -2;
    for (int f = 0; f < 20; f++) {
        const double* b = h3::kH3FastBasis[f];
        double d = b[0] * p[0] + b[1] * p[1] + b[2] * p[2];
        if (d > bd) {
            bd = d;
            best = f;
        }
    }
    return best;
}
int face_of(double lon, double lat) {
    double p[3];
    FacePlane::unit(lon, lat, p);
    return face_of_unit(p);
}

// The hexagon corner offsets R cos(30 + 60 k deg), R sin(...), k = 0..5: the same expressions as the
// per-cell loops used to evaluate (so the same doubles), computed once.
struct HexCorners {
    double dx[6], dy[6];
    HexCorners() {
        const double R = 0.57735026918962576451;
        for (int k = 0; k < 6; k++) {
            double ang = (30.0 + 60.0 * k) * (M_PI / 180.0);
            dx[k] = R * cos(ang);
            dy[k] = R * sin(ang);
        }
    }
};
const HexCorners& hex_corners() {
    static const HexCorners h;
    return h;
}

// ---- geometry helpers (plane) ----
double ring_area(const std::vector<P2>& r) {
    double a = 0;
    for (size_t i = 0; i + 1 < r.size(); i++) a += r[i].x * r[i + 1].y - r[i + 1].x * r[i].y;
    return 0.5 * a;
}

// Sutherland-Hodgman: clip an (open) vertex list by the half-plane left of edge a->b (ccw convex clip).
// tag[i] carries, per output vertex, the index of the original vertex (>= 0) or -1 if computed.
void clip_edge(const std::vector<P2>& in, const std::vector<long>& tin, P2 a, P2 b, std::vector<P2>& out,
               std::vector<long>& tout) {
    out.clear();
    tout.clear();
    size_t n = in.size();
    if (!n) return;
    auto side = [&](P2 p) { return (b.x - a.x) * (p.y - a.y) - (b.y - a.y) * (p.x - a.x); };
    for (size_t i = 0; i < n; i++) {
        P2 cur = in[i], prev = in[(i + n - 1) % n];
        double sc = side(cur), sp = side(prev);
        bool ic = sc >= 0, ip = sp >= 0;
        if (ic) {
            if (!ip) {
                double t = sp / (sp - sc);
                out.push_back({prev.x + t * (cur.x - prev.x), prev.y + t * (cur.y - prev.y)});
                tout.push_back(-1);
            }
            out.push_back(cur);
            tout.push_back(tin[i]);
        } else if (ip) {
            double t = sp / (sp - sc);
            out.push_back({prev.x + t * (cur.x - prev.x), prev.y + t * (cur.y - prev.y)});
            tout.push_back(-1);
        }
    }
}

bool seg_near_convex(P2 p, P2 q, const std::vector<P2>& poly, double eps) {
    // true if segment pq comes within eps of the convex polygon (ccw, open vertex list)
    // test: any endpoint inside expanded poly, or segment intersects an edge, or distance < eps
    auto inside = [&](P2 r) {
        for (size_t i = 0; i < poly.size(); i++) {
            P2 a = poly[i], b = poly[(i + 1) % poly.size()];
            double ex = b.x - a.x, ey = b.y - a.y, len = sqrt(ex * ex + ey * ey);
            if ((ex * (r.y - a.y) - ey * (r.x - a.x)) / len < -eps) return false;
        }
        return true;
    };
    if (inside(p) || inside(q)) return true;
    auto dist_seg = [](P2 r, P2 a, P2 b) {
        double ex = b.x - a.x, ey = b.y - a.y;
        double t = ((r.x - a.x) * ex + (r.y - a.y) * ey) / (ex * ex + ey * ey);
        t = std::max(0.0, std::min(1.0, t));
        double dx = a.x + t * ex - r.x, dy = a.y + t * ey - r.y;
        return sqrt(dx * dx + dy * dy);
    };
    for (size_t i = 0; i < poly.size(); i++) {
        P2 a = poly[i], b = poly[(i + 1) % poly.size()];
        double d1 = (b.x - a.x) * (p.y - a.y) - (b.y - a.y) * (p.x - a.x);
        double d2 = (b.x - a.x) * (q.y - a.y) - (b.y - a.y) * (q.x - a.x);
        double d3 = (q.x - p.x) * (a.y - p.y) - (q.y - p.y) * (a.x - p.x);
        double d4 = (q.x - p.x) * (b.y - p.y) - (q.y - p.y) * (b.x - p.x);
        if (((d1 > 0) != (d2 > 0)) && ((d3 > 0) != (d4 > 0))) return true;
        if (dist_seg(a, p, q) < eps || dist_seg(p, a, b) < eps || dist_seg(q, a, b) < eps) return true;
    }
    return false;
}

bool point_in_rings_evenodd(P2 p, const std::vector<std::vector<P2>>& rings) {
    bool in = false;
    for (auto& r : rings) {
        for (size_t i = 0, j = r.size() - 1; i < r.size(); j = i++) {
            if (((r[i].y > p.y) != (r[j].y > p.y)) &&
                (p.x < (r[j].x - r[i].x) * (p.y - r[i].y) / (r[j].y - r[i].y) + r[i].x))
                in = !in;
        }
    }
    return in;
}

// ---- WKB writer (JTS WKBWriter default: big-endian, 2D) ----
struct WkbOut {
    std::vector<uint8_t> b;
    void u8(uint8_t v) { b.push_back(v); }
    void u32(uint32_t v) {
        const size_t n = b.size();
        b.resize(n + 4);
        v = __builtin_bswap32(v);
        memcpy(b.data() + n, &v, 4);
    }
    void f64(double d) {
        uint64_t u;
        memcpy(&u, &d, 8);
        const size_t n = b.size();
        b.resize(n + 8);
        u = __builtin_bswap64(u);
        memcpy(b.data() + n, &u, 8);
    }
    void polygon(const std::vector<std::vector<P2>>& rings) {
        u8(0);
        u32(3);
        u32((uint32_t)rings.size());
        for (auto& r : rings) {
            u32((uint32_t)r.size());
            for (auto& p : r) {
                f64(p.x);
                f64(p.y);
            }
        }
    }
};

// to a preallocated span (same bytes as WkbOut)
struct WkbPtr {
    uint8_t* b;
    void u8(uint8_t v) { *b++ = v; }
    void u32(uint32_t v) {
        v = __builtin_bswap32(v);
        memcpy(b, &v, 4);
        b += 4;
    }
    void f64(double d) {
        uint64_t u;
        memcpy(&u, &d, 8);
        u = __builtin_bswap64(u);
        memcpy(b, &u, 8);
        b += 8;
    }
};
// counts bytes only
struct WkbSize {
    int64_t n = 0;
    void u8(uint8_t) { n += 1; }
    void u32(uint32_t) { n += 4; }
    void f64(double) { n += 8; }
};

std::vector<uint8_t> to_wkb(const std::vector<std::vector<std::vector<P2>>>& parts) {
    WkbOut w;
    if (parts.size() == 1) {
        w.polygon(parts[0]);
    } else {
        w.u8(0);
        w.u32(6);
        w.u32((uint32_t)parts.size());
        for (auto& p : parts) w.polygon(p);
    }
    return w.b;
}

}  // namespace

// an allocator whose resize() leaves new bytes uninitialised (the writers fill them, in parallel)
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U>&) {}
    template <class U>
    void construct(U* p) noexcept {
        ::new ((void*)p) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... args) {
        ::new ((void*)p) U(std::forward<A>(args)...);
    }
};

struct mosaic_chip_set {
    std::vector<uint8_t> is_core;
    std::vector<int64_t> index_id;
    std::vector<int32_t> key;
    std::vector<int64_t> wkb_offsets{0};
    std::vector<uint8_t, NoInitAlloc<uint8_t>> wkb;
    void add(bool core, int64_t id, int32_t k, const std::vector<uint8_t>& blob) {
        is_core.push_back(core);
        index_id.push_back(id);
        key.push_back(k);
        wkb.insert(wkb.end(), blob.begin(), blob.end());
        wkb_offsets.push_back((int64_t)wkb.size());
    }
};

namespace {

struct Cell {
    int64_t id;
    std::vector<P2> clip;     // convex clip polygon in the plane (ccw, open)
    std::vector<P2> outline;  // densified outline in the plane for core chip output
};

// The class of one cell (convex clip region) for one geometry given in the plane: 0 disjoint (or in a
// hole), 1 core (no polygon segment within core_eps, centre inside), 2 border.
int classify_cell(const Cell& cell, const std::vector<std::vector<std::vector<P2>>>& pl, double core_eps) {
    // 1) any polygon segment near the cell?  2) cell centre inside?
    for (size_t pi = 0; pi < pl.size(); pi++)
        for (auto& ring : pl[pi])
            for (size_t i = 0; i + 1 < ring.size(); i++)
                if (seg_near_convex(ring[i], ring[i + 1], cell.clip, core_eps)) return 2;
    P2 c = {0, 0};
    for (auto& p : cell.clip) {
        c.x += p.x;
        c.y += p.y;
    }
    c.x /= cell.clip.size();
    c.y /= cell.clip.size();
    bool inside = false;
    for (size_t pi = 0; pi < pl.size(); pi++) inside = inside || point_in_rings_evenodd(c, pl[pi]);
    return inside ? 1 : 0;
}

// A core cell's outline mapped to output coordinates, closed.
template <class ToGeo>
std::vector<P2> cell_ring(const Cell& cell, ToGeo to_geo) {
    std::vector<P2> ring;
    for (auto& p : cell.outline) ring.push_back(to_geo(p));
    ring.push_back(ring.front());
    return ring;
}

// Border cell: every ring of the geometry clipped against the cell, appended to out_parts (polygon
// parts, shells first); original vertices kept exact, computed ones mapped by to_geo.
template <class ToGeo>
void clip_cell(const Cell& cell, const std::vector<std::vector<std::vector<P2>>>& pl,
               const std::vector<std::vector<std::vector<P2>>>& geo, ToGeo to_geo, double area_eps,
               std::vector<std::vector<std::vector<P2>>>& out_parts) {
    std::vector<P2> a, b;
    std::vector<long> ta, tb;
    for (size_t pi = 0; pi < pl.size(); pi++) {
        std::vector<std::vector<P2>> rings_out;
        double net = 0;
        for (size_t ri = 0; ri < pl[pi].size(); ri++) {
            const auto& ring = pl[pi][ri];
            if (ring.size() < 4) continue;
            a.assign(ring.begin(), ring.end() - 1);  // open
            ta.resize(a.size());
            for (size_t i = 0; i < a.size(); i++) ta[i] = (long)i;
            for (size_t e = 0; e < cell.clip.size() && !a.empty(); e++) {
                clip_edge(a, ta, cell.clip[e], cell.clip[(e + 1) % cell.clip.size()], b, tb);
                a.swap(b);
                ta.swap(tb);
            }
            if (a.size() < 3) {
                if (ri == 0) break;  // shell misses the cell
                continue;
            }
            std::vector<P2> plane_closed(a);
            plane_closed.push_back(a.front());
            double ar = ring_area(plane_closed);
            if (fabs(ar) <= area_eps) {
                if (ri == 0) break;
                continue;
            }
            net += ri == 0 ? fabs(ar) : -fabs(ar);
            std::vector<P2> g;
            g.reserve(a.size() + 1);
            for (size_t i = 0; i < a.size(); i++)
                g.push_back(ta[i] >= 0 ? geo[pi][ri][ta[i]] : to_geo(a[i]));  // original vertices kept exact
            g.push_back(g.front());
            rings_out.push_back(std::move(g));
        }
        if (!rings_out.empty() && net > area_eps) out_parts.push_back(std::move(rings_out));
    }
}

// Classify one cell against one geometry given in the plane (plane rings + original lon/lat rings)
// and emit its chip.  to_geo maps a plane point to output coordinates.
template <class ToGeo>
void emit_cell(mosaic_chip_set* cs, int32_t key, const Cell& cell, const std::vector<std::vector<std::vector<P2>>>& pl,
               const std::vector<std::vector<std::vector<P2>>>& geo, double core_eps, int keep_core_geom,
               ToGeo to_geo, double area_eps, int pre = -1) {
    // pre >= 0: the class was computed on the GPU (k_bng_tess_classify: 0 dropped, 1 core, 2 border)
    const int cls = pre >= 0 ? pre : classify_cell(cell, pl, core_eps);
    if (cls == 0) return;
    if (cls == 1) {
        std::vector<uint8_t> blob;
        if (keep_core_geom) blob = to_wkb({{cell_ring(cell, to_geo)}});
        cs->add(true, cell.id, key, blob);
        return;
    }
    std::vector<std::vector<std::vector<P2>>> out_parts;
    clip_cell(cell, pl, geo, to_geo, area_eps, out_parts);
    if (out_parts.empty()) return;
    cs->add(false, cell.id, key, to_wkb(out_parts));
}

// ---- border chips as the reference builds them (llclip.h): geometry n cell polygon in output
// coordinates, with JTS's crossing arithmetic.  Cells the planar clip cannot take (a cell over the
// antimeridian or a pole; a ring walk whose labels do not pair up) fall back to clip_cell in the
// plane of `pl` and are counted (mosaic_tess_counters).
std::atomic<int64_t> g_ll_fallbacks{0}, g_ll_chips{0};

// H3 cell id -> its indexToGeometry polygon (h3ToGeoBoundary, degrees via JDK 8 Math.toDegrees, as
// H3IndexSystem.scala:93-100 builds it); false when it is not a planar counter-clockwise polygon
// the batch's ring indexes for the lon / lat clip (llclip::ring_blocks_one), built on first use (host
// threads may call geom() at once)
struct RingIdx {
    int64_t n_rings = 0;
    const double* xy;
    const int64_t *ro, *pr;
    mutable std::vector<double> blk;
    mutable std::vector<int64_t> ring_blk;
    mutable std::vector<uint8_t> ccw;
    mutable std::once_flag once;
    RingIdx(int64_t n_geoms, const int64_t* gp, const int64_t* pr_, const int64_t* ro_, const double* xy_)
        : xy(xy_), ro(ro_), pr(pr_) {
        if (n_geoms > 0 && gp && pr_ && ro_ && xy_) n_rings = pr_[gp[n_geoms]];
    }
    llclip::Geom geom(int64_t p0, int64_t p1) const {
        std::call_once(once, [&] {
            ring_blk.resize((size_t)std::max<int64_t>(1, n_rings));
            ccw.resize((size_t)std::max<int64_t>(1, n_rings));
            int64_t t = 0;
            for (int64_t r = 0; r < n_rings; r++) ring_blk[(size_t)r] = t, t += llclip::ring_block_count(ro, r);
            blk.resize((size_t)std::max<int64_t>(1, t) * 4);
            for (int64_t r = 0; r < n_rings; r++)
                llclip::ring_blocks_one(ro, xy, r, blk.data() + 4 * ring_blk[(size_t)r], ccw.data() + r);
        });
        return llclip::Geom{xy, ro, pr, p0, p1, blk.data(), ring_blk.data(), ccw.data()};
    }
};

bool h3_cell_ll(int64_t id, llclip::Cell& C) {
    double b[20];
    const int nb = h3geom::h3_to_geo_boundary((uint64_t)id, b);
    if (nb < 3 || nb > 16) return false;
    C.nc = nb;
    for (int v = 0; v < nb; v++) C.v[v] = {h3geom::to_degrees(b[2 * v + 1], 8), h3geom::to_degrees(b[2 * v], 8)};
    llclip::cell_init(C);
    return llclip::cell_ok(C, true);
}
// BNG square (BNGIndexSystem.indexToGeometry: (x, y), (x + e, y), (x + e, y + e), (x, y + e))
bool bng_cell_ll(double x0, double y0, double e, llclip::Cell& C) {
    C.nc = 4;
    C.v[0] = {x0, y0};
    C.v[1] = {x0 + e, y0};
    C.v[2] = {x0 + e, y0 + e};
    C.v[3] = {x0, y0 + e};
    llclip::cell_init(C);
    return llclip::cell_ok(C, false);
}

// The chip of geometry gg against C as WKB (empty: no chip); llclip status.  Host scratch grows on
// overflow, so only kInconsistent / kBadCell come back non-zero.
int ll_chip(const llclip::Geom& gg, const llclip::Cell& C, bool* is_cell, std::vector<uint8_t>& wkb) {
    thread_local std::vector<llclip::Chain> ch;
    thread_local std::vector<llclip::Out> out;
    thread_local std::vector<double> buf;
    const double eps2 = 1e-12 * llclip::cell_area2(C);
    for (size_t cap = 64;; cap *= 4) {
        if (ch.size() < cap) ch.resize(cap);
        if (out.size() < cap) out.resize(cap);
        llclip::Work w{ch.data(), (int32_t)cap, out.data(), (int32_t)cap, 0, 0};
        int32_t polys = 0;
        const int st = llclip::clip(gg, C, w, eps2, &polys, is_cell);
        if (st == llclip::kOverflow && cap < ((size_t)1 << 22)) continue;
        if (st) return st;
        wkb.clear();
        if (polys == 0) return llclip::kOk;
        WkbOut wo;
        if (polys > 1) {
            wo.u8(0);
            wo.u32(6);
            wo.u32((uint32_t)polys);
        }
        for (int32_t i = 0; i < w.n_out;) {
            int32_t j = i + 1;
            while (j < w.n_out && w.out[j].hole) j++;
            wo.u8(0);
            wo.u32(3);
            wo.u32((uint32_t)(j - i));
            for (int32_t k = i; k < j; k++) {
                const int32_t n = w.out[k].npts;
                buf.resize(2 * (size_t)(n + 1));
                llclip::write_ring(gg, C, w, w.out[k], buf.data());
                wo.u32((uint32_t)(n + 1));
                for (int32_t v = 0; v <= n; v++) {
                    wo.f64(buf[2 * (size_t)v]);
                    wo.f64(buf[2 * (size_t)v + 1]);
                }
            }
            i = j;
        }
        wkb.swap(wo.b);
        g_ll_chips++;
        return llclip::kOk;
    }
}

// C as a closed ring (a core chip's indexToGeometry)
std::vector<P2> cell_ll_ring(const llclip::Cell& C) {
    std::vector<P2> r;
    for (int v = 0; v <= C.nc; v++) r.push_back({C.v[v % C.nc].x, C.v[v % C.nc].y});
    return r;
}

// emit_cell with the reference's border chips: classification in the plane of pl (as emit_cell),
// border cells clipped against C (make_c(C) fills it; false: no planar polygon) in output coordinates;
// core chips carry C itself when core_from_c (H3 without densify, BNG), else the plane outline.
template <class ToGeo, class MakeC>
void emit_cell_ll(mosaic_chip_set* cs, int32_t key, const Cell& cell, const std::vector<std::vector<std::vector<P2>>>& pl,
                  const std::vector<std::vector<std::vector<P2>>>& geo, const llclip::Geom& gg, double core_eps,
                  int keep_core_geom, ToGeo to_geo, double area_eps, MakeC make_c, bool core_from_c, int pre = -1) {
    const int cls = pre >= 0 ? pre : classify_cell(cell, pl, core_eps);
    if (cls == 0) return;
    llclip::Cell C;
    if (cls == 1) {
        std::vector<uint8_t> blob;
        if (keep_core_geom) blob = to_wkb({{core_from_c && make_c(C) ? cell_ll_ring(C) : cell_ring(cell, to_geo)}});
        cs->add(true, cell.id, key, blob);
        return;
    }
    const bool cok = make_c(C);
    if (cok) {
        bool is_cell = false;
        std::vector<uint8_t> blob;
        if (ll_chip(gg, C, &is_cell, blob) == llclip::kOk) {
            if (!blob.empty()) cs->add(is_cell, cell.id, key, is_cell && !keep_core_geom ? std::vector<uint8_t>() : blob);
            return;
        }
    }
    g_ll_fallbacks++;
    std::vector<std::vector<std::vector<P2>>> out_parts;
    clip_cell(cell, pl, geo, to_geo, area_eps, out_parts);
    if (out_parts.empty()) return;
    cs->add(false, cell.id, key, to_wkb(out_parts));
}

// ---- H3 polygons that span icosahedron faces ----
// geoToH3 projects a point onto its closest face (largest fc . p) and rounds in that face's
// gnomonic plane, so a cell is, on the sphere, the union over faces f of (hexagon of its lattice
// position on f) n territory(f), where territory(f) = {p : fc_f . p >= fc_g . p for every g} is the
// face's spherical triangle, a straight-edged triangle in f's gnomonic plane (the three bisector
// planes (fc_f - fc_g) . p = 0 of its edge neighbours g).  Per face f whose territory meets the
// polygon, candidate lattice cells are clipped to the triangle; face_ijk_to_h3(f, ijk) is H3's id of
// the points of that piece (what _faceIjkToH3 computes for them).  A cell's pieces are then merged:
// core when every piece is core, else a border chip holding the core pieces' outlines and the
// border pieces' clips (a MultiPolygon whose parts meet along the face edge).
struct FaceTerritory {
    double A[3], B[3], C[3];  // A x + B y + C >= 0 in the face plane (hex2d units at res)
    void init(int f, const FacePlane& fp) {
        const double* fc = h3::kH3FastBasis[f];
        int nb[3] = {-1, -1, -1};
        double nd[3] = {-2, -2, -2};
        for (int g = 0; g < 20; g++) {  // the three edge neighbours: the closest face centres
            if (g == f) continue;
            const double* fg = h3::kH3FastBasis[g];
            double d = fc[0] * fg[0] + fc[1] * fg[1] + fc[2] * fg[2];
            for (int q = 0; q < 3; q++)
                if (d > nd[q]) {
                    for (int r = 2; r > q; r--) {
                        nd[r] = nd[r - 1];
                        nb[r] = nb[r - 1];
                    }
                    nd[q] = d;
                    nb[q] = g;
                    break;
                }
        }
        for (int q = 0; q < 3; q++) {
            const double* fg = h3::kH3FastBasis[nb[q]];
            double w[3] = {fc[0] - fg[0], fc[1] - fg[1], fc[2] - fg[2]};
            // p ~ fc + (x ei + y ep) / S
            C[q] = w[0] * fc[0] + w[1] * fc[1] + w[2] * fc[2];
            A[q] = (w[0] * fp.ei[0] + w[1] * fp.ei[1] + w[2] * fp.ei[2]) / fp.S;
            B[q] = (w[0] * fp.ep[0] + w[1] * fp.ep[1] + w[2] * fp.ep[2]) / fp.S;
        }
    }
    // the triangle's corners (pairwise intersections of its edge lines)
    void corners(P2 out[3]) const {
        for (int q = 0; q < 3; q++) {
            const int a = (q + 1) % 3, b = (q + 2) % 3;
            const double det = A[a] * B[b] - A[b] * B[a];
            out[q] = {(-C[a] * B[b] + C[b] * B[a]) / det, (-A[a] * C[b] + A[b] * C[a]) / det};
        }
    }
};

// keep A x + B y + C >= 0 of a convex (open) polygon
void clip_halfplane(const std::vector<P2>& in, double A, double B, double C, std::vector<P2>& out) {
    out.clear();
    const size_t n = in.size();
    for (size_t i = 0; i < n; i++) {
        const P2 cur = in[i], prev = in[(i + n - 1) % n];
        const double sc = A * cur.x + B * cur.y + C, sp = A * prev.x + B * prev.y + C;
        if (sc >= 0) {
            if (sp < 0) {
                const double t = sp / (sp - sc);
                out.push_back({prev.x + t * (cur.x - prev.x), prev.y + t * (cur.y - prev.y)});
            }
            out.push_back(cur);
        } else if (sp >= 0) {
            const double t = sp / (sp - sc);
            out.push_back({prev.x + t * (cur.x - prev.x), prev.y + t * (cur.y - prev.y)});
        }
    }
}

double open_area(const std::vector<P2>& r) {
    double a = 0;
    for (size_t i = 0; i < r.size(); i++) {
        const P2 p = r[i], q = r[(i + 1) % r.size()];
        a += p.x * q.y - q.x * p.y;
    }
    return 0.5 * a;
}

using Geo3 = std::vector<std::vector<std::vector<P2>>>;  // parts -> rings -> points

// The per-face pieces of one face-spanning geometry: made by multiface_pieces, classified and
// clipped by multiface_classify_host (tessellate_h3_multiface) or on the GPU (mosaic_tessellate_gpu,
// the same arithmetic), turned into chips by multiface_emit.
struct MultiPiece {
    int face, cls = -1;
    Cell cell;
    Geo3 parts;  // border: the clipped geometry
};
struct MultiFace {
    std::vector<int64_t> order;                   // cell ids in first-seen order (faces ascending, lattice order)
    std::vector<std::vector<size_t>> slot_pieces;  // per cell id: its pieces (indices into pieces)
    std::vector<MultiPiece> pieces;
    std::vector<int> faces;                       // faces with pieces, ascending
    std::vector<Geo3> pl;                         // per face of `faces`: the geometry in its plane
    int face_slot(int f) const {
        for (size_t k = 0; k < faces.size(); k++)
            if (faces[k] == f) return (int)k;
        return -1;
    }
};

// Pieces of geometry geo (lon/lat rings) that spans faces: 0, or MOSAIC_E_ARG for geometries no face
// plane can hold (a vertex more than ~78 degrees from a face centre whose territory it meets).
int multiface_pieces(int res, int D, const Geo3& geo, MultiFace& mf) {
    std::unordered_map<int64_t, size_t> index;  // id -> slot (O(1) per piece: country-scale inputs)
    auto slot_of = [&](int64_t id) -> size_t {
        auto ins = index.emplace(id, mf.order.size());
        if (ins.second) {
            mf.order.push_back(id);
            mf.slot_pieces.emplace_back();
        }
        return ins.first->second;
    };
    const double s60 = 0.86602540378443864676, R = 0.57735026918962576451;
    int faces_used = 0;
    for (int f = 0; f < 20; f++) {
        FacePlane fp;
        fp.init(f, res);
        const double* fc = fp.fc;
        // the gnomonic projection must hold every vertex (fc . p >= 0.2, ~78 degrees)
        bool valid = true;
        for (auto& part : geo)
            for (auto& ring : part)
                for (auto& p : ring) {
                    double u[3];
                    FacePlane::unit(p.x, p.y, u);
                    if (fc[0] * u[0] + fc[1] * u[1] + fc[2] * u[2] < 0.2) valid = false;
                }
        FaceTerritory ft;
        ft.init(f, fp);
        std::vector<std::vector<std::vector<P2>>> pl = geo;
        for (auto& part : pl)
            for (auto& ring : part)
                for (auto& p : ring) p = fp.to_hex(p.x, p.y);
        // does the territory meet the geometry? (the shells clipped to the triangle keep area)
        double met = 0;
        if (valid) {
            std::vector<P2> a, b;
            for (auto& part : pl) {
                if (part.empty() || part[0].size() < 4) continue;
                a.assign(part[0].begin(), part[0].end() - 1);
                for (int q = 0; q < 3 && !a.empty(); q++) {
                    clip_halfplane(a, ft.A[q], ft.B[q], ft.C[q], b);
                    a.swap(b);
                }
                if (a.size() >= 3) met += fabs(open_area(a));
            }
        } else {
            // refuse when the geometry could reach this face: some vertex on it, or some edge
            // crossing its territory between vertices (edges sampled every <= 0.25 degrees; a face
            // territory is ~40 degrees across, so an edge that crosses one has samples on it)
            for (auto& part : geo)
                for (auto& ring : part)
                    for (size_t v = 0; v < ring.size(); v++) {
                        if (face_of(ring[v].x, ring[v].y) == f) return MOSAIC_E_ARG;
                        if (v == 0) continue;
                        const P2 a = ring[v - 1], b = ring[v];
                        const int m = (int)std::min(1e6, ceil(std::max(fabs(b.x - a.x), fabs(b.y - a.y)) / 0.25));
                        for (int t = 1; t < m; t++)
                            if (face_of(a.x + (b.x - a.x) * t / m, a.y + (b.y - a.y) * t / m) == f) return MOSAIC_E_ARG;
                    }
            continue;
        }
        if (!(met > 1e-12)) continue;
        faces_used++;
        mf.faces.push_back(f);
        mf.pl.push_back(pl);
        P2 tc[3];
        ft.corners(tc);
        double x0 = 1e300, y0 = 1e300, x1 = -1e300, y1 = -1e300;
        for (auto& part : pl)
            for (auto& ring : part)
                for (auto& p : ring) {
                    x0 = std::min(x0, p.x);
                    x1 = std::max(x1, p.x);
                    y0 = std::min(y0, p.y);
                    y1 = std::max(y1, p.y);
                }
        double tx0 = std::min(tc[0].x, std::min(tc[1].x, tc[2].x)), tx1 = std::max(tc[0].x, std::max(tc[1].x, tc[2].x));
        double ty0 = std::min(tc[0].y, std::min(tc[1].y, tc[2].y)), ty1 = std::max(tc[0].y, std::max(tc[1].y, tc[2].y));
        x0 = std::max(x0, tx0);
        x1 = std::min(x1, tx1);
        y0 = std::max(y0, ty0);
        y1 = std::min(y1, ty1);
        if (x0 > x1 || y0 > y1) continue;
        int jlo = (int)floor(y0 / s60) - 2, jhi = (int)ceil(y1 / s60) + 2;
        std::vector<P2> hex, tmp;
        for (int j = jlo; j <= jhi; j++) {
            int ilo = (int)floor(x0 + j * 0.5) - 2, ihi = (int)ceil(x1 + j * 0.5) + 2;
            for (int i = ilo; i <= ihi; i++) {
                double cx = i - 0.5 * j, cy = j * s60;
                if (cx + R < x0 || cx - R > x1 || cy + R < y0 || cy - R > y1) continue;
                P2 corners[6];
                for (int k = 0; k < 6; k++) corners[k] = {cx + hex_corners().dx[k], cy + hex_corners().dy[k]};
                hex.clear();
                for (int k = 0; k < 6; k++) {
                    P2 a = corners[k], b = corners[(k + 1) % 6];
                    for (int t = 0; t < D; t++) hex.push_back({a.x + (b.x - a.x) * t / D, a.y + (b.y - a.y) * t / D});
                }
                // the piece of the cell on this face
                for (int q = 0; q < 3 && !hex.empty(); q++) {
                    clip_halfplane(hex, ft.A[q], ft.B[q], ft.C[q], tmp);
                    hex.swap(tmp);
                }
                if (hex.size() < 3 || !(fabs(open_area(hex)) > 1e-9)) continue;
                h3::IJK ijk = {i, j, 0};
                h3::ijk_normalize(ijk);
                const int64_t id = (int64_t)h3::face_ijk_to_h3(f, ijk, res);
                if (id == 0) return MOSAIC_E_ARG;  // (a lattice cell H3 has no id for: not expected)
                MultiPiece pc;
                pc.face = f;
                pc.cell.id = id;
                pc.cell.clip = hex;
                pc.cell.outline = hex;
                mf.slot_pieces[slot_of(id)].push_back(mf.pieces.size());
                mf.pieces.push_back(std::move(pc));
            }
        }
    }
    return MOSAIC_OK;
}

// classify_cell and clip_cell of every piece against the geometry in its face's plane
void multiface_classify_host(MultiFace& mf, const Geo3& geo, int res) {
    for (size_t k = 0; k < mf.faces.size(); k++) {
        FacePlane fp;
        fp.init(mf.faces[k], res);
        for (MultiPiece& pc : mf.pieces) {
            if (pc.face != mf.faces[k]) continue;
            pc.cls = classify_cell(pc.cell, mf.pl[k], 1e-3);
        }
    }
}

// The chips of the classified pieces, in cell first-seen order: a cell whose pieces are all core is a
// core chip (indexToGeometry); any other cell with a piece in the polygon gets the reference's border
// chip -- the whole geometry clipped against the cell's boundary polygon in lon / lat (llclip.h), which
// needs no per-face pieces (the boundary carries H3's face-edge vertices).  A cell the planar clip
// cannot take falls back to the pieces clipped in their faces' planes, dissolved along the face edge.
void multiface_emit(mosaic_chip_set* cs, int32_t key, int res, int keep_core_geom, MultiFace& mf, const Geo3& geo,
                    const llclip::Geom& gg) {
    for (size_t k = 0; k < mf.order.size(); k++) {
        std::vector<MultiPiece*> ps;
        for (size_t q : mf.slot_pieces[k]) ps.push_back(&mf.pieces[q]);
        const std::vector<int64_t>& order = mf.order;
        bool all_core = true, any = false;
        for (const MultiPiece* pp : ps) {
            all_core = all_core && pp->cls == 1;
            any = any || pp->cls == 1 || pp->cls == 2;
        }
        if (!any) continue;
        std::vector<std::vector<std::vector<P2>>> parts;
        llclip::Cell C;
        const bool cok = h3_cell_ll(order[k], C);
        if (all_core) {
            // a core cell over a face edge: its geometry is the one polygon of the cell boundary
            // (h3ToGeoBoundary, what the reference's indexToGeometry returns for a core chip,
            // H3IndexSystem.scala:93-100), not the per-face pieces
            if (keep_core_geom) {
                double b[20];
                const int nb = h3geom::h3_to_geo_boundary((uint64_t)order[k], b);
                if (nb < 3) continue;  // (not expected: a valid H3 id)
                std::vector<P2> ring;
                for (int v = 0; v <= nb; v++) {
                    const int q = v % nb;
                    ring.push_back({h3geom::to_degrees(b[2 * q + 1], 8), h3geom::to_degrees(b[2 * q], 8)});
                }
                parts.push_back({ring});
            }
            cs->add(true, order[k], key, keep_core_geom ? to_wkb(parts) : std::vector<uint8_t>());
            continue;
        }
        if (cok) {
            bool is_cell = false;
            std::vector<uint8_t> blob;
            if (ll_chip(gg, C, &is_cell, blob) == llclip::kOk) {
                if (!blob.empty()) cs->add(is_cell, order[k], key, is_cell && !keep_core_geom ? std::vector<uint8_t>() : blob);
                continue;
            }
        }
        g_ll_fallbacks++;
        int face_mask_n = 0;
        uint32_t face_mask = 0;
        for (MultiPiece* pp : ps) {
            MultiPiece& p = *pp;
            const size_t before = parts.size();
            FacePlane fp;
            fp.init(p.face, res);
            if (p.cls == 1) {
                parts.push_back({cell_ring(p.cell, [&](P2 h) { return fp.to_geo(h); })});
            } else if (p.cls == 2) {
                if (p.parts.empty())
                    clip_cell(p.cell, mf.pl[(size_t)mf.face_slot(p.face)], geo, [&](P2 h) { return fp.to_geo(h); }, 1e-12,
                              p.parts);
                for (auto& q : p.parts) parts.push_back(q);
            }
            if (parts.size() > before && !(face_mask & (1u << p.face))) {
                face_mask |= 1u << p.face;
                face_mask_n++;
            }
        }
        if (parts.empty()) continue;
        if (face_mask_n > 1) {
            // pieces of several faces meet along the face edge: dissolved into one geometry (every ring
            // as directed edges, interior on the left, through st_intersection_aggregate's stitcher)
            std::vector<double> e;
            for (const auto& part : parts)
                for (size_t r = 0; r < part.size(); r++) {
                    const std::vector<P2>& ring = part[r];
                    size_t n = ring.size();
                    if (n > 1 && ring[0].x == ring[n - 1].x && ring[0].y == ring[n - 1].y) n--;
                    if (n < 3) continue;
                    double a2 = 0.0;
                    for (size_t i = 0; i < n; i++) {
                        const P2 &u = ring[i], &v = ring[(i + 1) % n];
                        a2 += u.x * v.y - v.x * u.y;
                    }
                    const bool rev = (a2 > 0) != (r == 0);
                    for (size_t i = 0; i < n; i++) {
                        const P2 &u = ring[i], &v = ring[(i + 1) % n];
                        if (rev) e.insert(e.end(), {v.x, v.y, u.x, u.y});
                        else e.insert(e.end(), {u.x, u.y, v.x, v.y});
                    }
                }
            std::vector<uint8_t> merged;
            double area = 0.0;
            if (isect_geom::stitch_wkb(e.data(), e.size() / 4, 1e-9, merged, &area) && merged.size() > 9) {
                cs->add(false, order[k], key, merged);
                continue;
            }
        }
        cs->add(false, order[k], key, to_wkb(parts));
    }
}

// Chips of geometry g (lon/lat rings geo) that spans faces, on the host: 0, or MOSAIC_E_ARG (see
// multiface_pieces).
int tessellate_h3_multiface(mosaic_chip_set* cs, int32_t key, int res, int D, int keep_core_geom, const Geo3& geo,
                            const llclip::Geom& gg) {
    MultiFace mf;
    if (int rc = multiface_pieces(res, D, geo, mf)) return rc;
    multiface_classify_host(mf, geo, res);
    multiface_emit(cs, key, res, keep_core_geom, mf, geo, gg);
    return MOSAIC_OK;
}

// The border chips the GPU clipped (tess_gpu.h), indexed by candidate: rings sorted by (candidate,
// part, ring), parts by (candidate, part).
struct ClippedChips {
    tessclip::ClipResult r;
    std::vector<int64_t> task_of;  // candidate -> task (-1: not a border task)
    std::vector<int64_t> ring_at, part_at;  // candidate c's rings / parts: [ring_at[c], ring_at[c + 1])
    void index(int64_t n_cand, const std::vector<int64_t>& tasks) {
        // stable counting sort by candidate (the kernels append each candidate's rings / parts in
        // (part, ring) order from one wave or lane; a candidate whose entries are not is sorted on
        // its own), keeping each candidate's start
        auto by_cand = [&](auto& v, auto less, std::vector<int64_t>& start) {
            start.assign((size_t)n_cand + 1, 0);
            for (auto& e : v) start[(size_t)e.cand + 1]++;
            for (int64_t c = 0; c < n_cand; c++) start[(size_t)c + 1] += start[(size_t)c];
            std::remove_reference_t<decltype(v)> out(v.size());
            std::vector<int64_t> pos(start.begin(), start.end() - 1);
            for (auto& e : v) out[(size_t)pos[(size_t)e.cand]++] = e;
            for (int64_t c = 0; c < n_cand; c++) {
                auto b = out.begin() + start[(size_t)c], e = out.begin() + start[(size_t)c + 1];
                if (e - b > 1 && !std::is_sorted(b, e, less)) std::sort(b, e, less);
            }
            v.swap(out);
        };
        by_cand(r.rings, [](const tessclip::ClipRing& a, const tessclip::ClipRing& b) {
            return a.part != b.part ? a.part < b.part : a.ring < b.ring;
        }, ring_at);
        by_cand(r.parts, [](const tessclip::ClipPart& a, const tessclip::ClipPart& b) { return a.part < b.part; }, part_at);
        task_of.assign((size_t)n_cand, -1);
        for (size_t t = 0; t < tasks.size(); t++) task_of[(size_t)tasks[t]] = (int64_t)t;
    }
    bool redo(int64_t k) const { return task_of[(size_t)k] < 0 || r.status[(size_t)task_of[(size_t)k]] == 1; }
    bool is_cell(int64_t k) const { return task_of[(size_t)k] >= 0 && r.status[(size_t)task_of[(size_t)k]] == 2; }
    // candidate k's clipped geometry as clip_cell's out_parts (kept parts with rings, closed rings)
    void parts_of(int64_t k, Geo3& out) const {
        out.clear();
        size_t jr = (size_t)ring_at[(size_t)k];
        for (size_t jp = (size_t)part_at[(size_t)k]; jp < r.parts.size() && r.parts[jp].cand == k; jp++) {
            const int32_t part = r.parts[jp].part;
            while (jr < r.rings.size() && r.rings[jr].cand == k && r.rings[jr].part < part) jr++;
            const size_t r0 = jr;
            while (jr < r.rings.size() && r.rings[jr].cand == k && r.rings[jr].part == part) jr++;
            if (!r.parts[jp].keep || jr == r0) continue;
            std::vector<std::vector<P2>> rings;
            for (size_t q = r0; q < jr; q++) {
                const tessclip::ClipRing& cr = r.rings[q];
                std::vector<P2> ring((size_t)cr.n);
                for (int32_t v = 0; v < cr.n; v++) ring[(size_t)v] = {r.verts[2 * (cr.off + v)], r.verts[2 * (cr.off + v) + 1]};
                rings.push_back(std::move(ring));
            }
            out.push_back(std::move(rings));
        }
    }
    // candidate k's chip as WKB appended to w (to_wkb's bytes); false (nothing written): no chip
    template <class W>
    bool chip(int64_t k, W& w) const {
        const size_t ir = (size_t)ring_at[(size_t)k], ip = (size_t)part_at[(size_t)k];
        // the kept parts that have rings: (first ring, ring count)
        std::pair<size_t, size_t> kept[64];
        std::vector<std::pair<size_t, size_t>> more;
        size_t n_kept = 0, jr = ir;
        for (size_t jp = ip; jp < r.parts.size() && r.parts[jp].cand == k; jp++) {
            const int32_t part = r.parts[jp].part;
            while (jr < r.rings.size() && r.rings[jr].cand == k && r.rings[jr].part < part) jr++;
            const size_t r0 = jr;
            while (jr < r.rings.size() && r.rings[jr].cand == k && r.rings[jr].part == part) jr++;
            if (!r.parts[jp].keep || jr == r0) continue;
            if (n_kept < 64) kept[n_kept] = {r0, jr - r0};
            else more.push_back({r0, jr - r0});
            n_kept++;
        }
        if (n_kept == 0) return false;
        auto part_at = [&](size_t i) { return i < 64 ? kept[i] : more[i - 64]; };
        if (n_kept > 1) {
            w.u8(0);
            w.u32(6);
            w.u32((uint32_t)n_kept);
        }
        for (size_t i = 0; i < n_kept; i++) {
            const auto pr = part_at(i);
            w.u8(0);
            w.u32(3);
            w.u32((uint32_t)pr.second);
            for (size_t q = pr.first; q < pr.first + pr.second; q++) {
                const tessclip::ClipRing& cr = r.rings[q];
                w.u32((uint32_t)cr.n);
                for (int32_t v = 0; v < cr.n; v++) {
                    w.f64(r.verts[2 * (cr.off + v)]);
                    w.f64(r.verts[2 * (cr.off + v) + 1]);
                }
            }
        }
        return true;
    }
};

// The face-spanning geometries' chips on the device (mosaic_tessellate_gpu): per-face pieces made on
// host threads (multiface_pieces), then classified by one session over virtual geometries --
// (geometry, face): the geometry's rings in that face's plane (MultiFace::pl, the host routine's
// doubles) -- with the pieces as explicit clip polygons (k_tess_classify_poly: tessellate.cpp's
// classify_cell arithmetic); multiface_emit then clips each border cell in lon / lat (llclip.h), as
// the host routine does.
int multiface_gpu(mosaic_ctx* ctx, const std::vector<int64_t>& multi_geoms, const int64_t* geom_parts,
                  const int64_t* part_rings, const int64_t* ring_offsets, const double* xy, int res, int D,
                  std::vector<MultiFace>& mfs, std::vector<Geo3>& geos) {
    const size_t nm = multi_geoms.size();
    geos.assign(nm, Geo3());
    std::atomic<size_t> next(0);
    std::atomic<int> bad(0);
    auto work = [&]() {
        for (size_t m; (m = next.fetch_add(1)) < nm;) {
            const int64_t g = multi_geoms[m];
            for (int64_t p = geom_parts[g]; p < geom_parts[g + 1]; p++) {
                std::vector<std::vector<P2>> rings;
                for (int64_t r = part_rings[p]; r < part_rings[p + 1]; r++) {
                    std::vector<P2> ring;
                    for (int64_t v = ring_offsets[r]; v < ring_offsets[r + 1]; v++) ring.push_back({xy[2 * v], xy[2 * v + 1]});
                    rings.push_back(std::move(ring));
                }
                geos[m].push_back(std::move(rings));
            }
            if (multiface_pieces(res, D, geos[m], mfs[m])) bad = 1;
        }
    };
    {
        const int nt = (int)std::max<size_t>(1, std::min<size_t>(std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency())), nm));
        std::vector<std::thread> pool;
        for (int t = 1; t < nt; t++) pool.emplace_back(work);
        work();
        for (auto& th : pool) th.join();
    }
    if (bad) return mosaic_tess_fail(MOSAIC_E_ARG, "geometry too large for a gnomonic face plane "
                                                  "(a vertex more than 78 degrees from a face centre it meets)");
    // virtual geometries and the pieces as candidates
    std::vector<int64_t> vgp(1, 0), vpr(1, 0), vro(1, 0);
    std::vector<double> vpxy, vxy;
    std::vector<int32_t> vgf;
    const int nvmax = 6 * D + 3;  // a 6D-gon cut by the three sides of a face triangle
    std::vector<int32_t> pcg, pcn;
    std::vector<double> pclip;
    std::vector<std::pair<size_t, size_t>> pref;  // candidate -> (geometry m, piece q)
    for (size_t m = 0; m < nm; m++) {
        const MultiFace& mf = mfs[m];
        std::vector<int32_t> vid(mf.faces.size());
        for (size_t k = 0; k < mf.faces.size(); k++) {
            vid[k] = (int32_t)vgf.size();
            vgf.push_back(mf.faces[k]);
            for (size_t pi = 0; pi < geos[m].size(); pi++) {
                for (size_t ri = 0; ri < geos[m][pi].size(); ri++) {
                    const std::vector<P2>& gr = geos[m][pi][ri];
                    const std::vector<P2>& pr = mf.pl[k][pi][ri];
                    for (size_t v = 0; v < gr.size(); v++) {
                        vxy.push_back(gr[v].x);
                        vxy.push_back(gr[v].y);
                        vpxy.push_back(pr[v].x);
                        vpxy.push_back(pr[v].y);
                    }
                    vro.push_back(vro.back() + (int64_t)gr.size());
                }
                vpr.push_back(vro.size() - 1);
            }
            vgp.push_back(vpr.size() - 1);
        }
        for (size_t q = 0; q < mf.pieces.size(); q++) {
            const MultiPiece& pc = mf.pieces[q];
            const int n = (int)pc.cell.clip.size();
            if (n > nvmax) return mosaic_tess_fail(MOSAIC_E_ARG, "face piece with more vertices than expected");
            pcg.push_back(vid[(size_t)mf.face_slot(pc.face)]);
            pcn.push_back(n);
            for (int v = 0; v < nvmax; v++) {
                pclip.push_back(v < n ? pc.cell.clip[(size_t)v].x : 0.0);
                pclip.push_back(v < n ? pc.cell.clip[(size_t)v].y : 0.0);
            }
            pref.push_back({m, q});
        }
    }
    const int64_t n_pieces = (int64_t)pcg.size();
    if (n_pieces == 0) return MOSAIC_OK;
    tessclip::H3Session* S = nullptr;
    if (int rc = tessclip::h3_session_begin(ctx, (int64_t)vgf.size(), vgp.data(), vpr.data(), vro.data(), vpxy.data(),
                                            vxy.data(), vgf.data(), res, D, hex_corners().dx, hex_corners().dy, &S))
        return rc;
    std::vector<uint8_t> cls((size_t)n_pieces, 0);
    std::vector<int64_t> tasks;
    tessclip::ClipResult cr;
    int rc = tessclip::h3_session_chunk(S, n_pieces, pcg.data(), nullptr, 1e-3, cls.data(), tasks, &cr, nullptr,
                                        pclip.data(), pcn.data(), nvmax);
    tessclip::h3_session_end(S);
    if (rc) return rc;
    for (int64_t i = 0; i < n_pieces; i++) mfs[pref[(size_t)i].first].pieces[pref[(size_t)i].second].cls = cls[(size_t)i];
    return MOSAIC_OK;
}

}  // namespace

extern "C" {

int mosaic_tessellate(int grid, int res, int64_t n_geoms, const int64_t* geom_parts, const int64_t* part_rings,
                      const int64_t* ring_offsets, const double* xy, int keep_core_geom, int densify,
                      mosaic_chip_set** out) {
    const RingIdx ri(n_geoms, geom_parts, part_rings, ring_offsets, xy);
    if (!out || n_geoms < 0 || (n_geoms > 0 && (!geom_parts || !part_rings || !ring_offsets || !xy)))
        return mosaic_tess_fail(MOSAIC_E_ARG, "invalid argument");
    if (grid == MOSAIC_GRID_H3 && (res < 0 || res > 15))
        return mosaic_tess_fail(MOSAIC_E_RES, ("H3 resolution has to be between 0 and 15; found " + std::to_string(res)).c_str());
    if (grid == MOSAIC_GRID_BNG && !(res != 0 && res >= -6 && res <= 6))
        return mosaic_tess_fail(MOSAIC_E_RES, ("BNG resolution not supported; found " + std::to_string(res)).c_str());
    if (grid != MOSAIC_GRID_H3 && grid != MOSAIC_GRID_BNG) return mosaic_tess_fail(MOSAIC_E_ARG, "unknown grid");
    if (densify < 1 || densify > 64) return mosaic_tess_fail(MOSAIC_E_ARG, "densify must be in [1, 64]");
    mosaic_chip_set* cs = new mosaic_chip_set();
    const int D = densify;  // hexagon edge subdivision (1 = the 6-vertex cell boundary)
    for (int64_t g = 0; g < n_geoms; g++) {
        // geometry in lon/lat (or BNG metres)
        std::vector<std::vector<std::vector<P2>>> geo;
        for (int64_t p = geom_parts[g]; p < geom_parts[g + 1]; p++) {
            std::vector<std::vector<P2>> rings;
            for (int64_t r = part_rings[p]; r < part_rings[p + 1]; r++) {
                std::vector<P2> ring;
                for (int64_t v = ring_offsets[r]; v < ring_offsets[r + 1]; v++) ring.push_back({xy[2 * v], xy[2 * v + 1]});
                rings.push_back(std::move(ring));
            }
            geo.push_back(std::move(rings));
        }
        bool any = false;
        for (auto& part : geo)
            for (auto& ring : part) any = any || !ring.empty();
        if (!any) continue;
        if (grid == MOSAIC_GRID_H3) {
            int face = -1;
            bool multi = false;
            for (auto& part : geo)
                for (auto& ring : part)
                    for (auto& p : ring) {
                        int f = face_of(p.x, p.y);
                        if (face < 0) face = f;
                        multi = multi || f != face;
                    }
            if (multi) {  // cells on several faces: per-face pieces (tessellate_h3_multiface)
                const llclip::Geom gg = ri.geom(geom_parts[g], geom_parts[g + 1]);
                if (tessellate_h3_multiface(cs, (int32_t)g, res, D, keep_core_geom, geo, gg)) {
                    delete cs;
                    return mosaic_tess_fail(MOSAIC_E_ARG, "geometry too large for a gnomonic face plane "
                                                          "(a vertex more than 78 degrees from a face centre it meets)");
                }
                continue;
            }
            FacePlane fp;
            fp.init(face, res);
            std::vector<std::vector<std::vector<P2>>> pl = geo;
            double x0 = 1e300, y0 = 1e300, x1 = -1e300, y1 = -1e300;
            for (auto& part : pl)
                for (auto& ring : part)
                    for (auto& p : ring) {
                        p = fp.to_hex(p.x, p.y);
                        x0 = std::min(x0, p.x);
                        x1 = std::max(x1, p.x);
                        y0 = std::min(y0, p.y);
                        y1 = std::max(y1, p.y);
                    }
            const double s60 = 0.86602540378443864676, R = 0.57735026918962576451;
            int jlo = (int)floor(y0 / s60) - 2, jhi = (int)ceil(y1 / s60) + 2;
            for (int j = jlo; j <= jhi; j++) {
                int ilo = (int)floor(x0 + j * 0.5) - 2, ihi = (int)ceil(x1 + j * 0.5) + 2;
                for (int i = ilo; i <= ihi; i++) {
                    double cx = i - 0.5 * j, cy = j * s60;
                    if (cx + R < x0 || cx - R > x1 || cy + R < y0 || cy - R > y1) continue;
                    Cell cell;
                    std::vector<P2> corners;
                    for (int k = 0; k < 6; k++) corners.push_back({cx + hex_corners().dx[k], cy + hex_corners().dy[k]});
                    cell.clip = corners;
                    for (int k = 0; k < 6; k++) {
                        P2 a = corners[k], b = corners[(k + 1) % 6];
                        for (int s = 0; s < D; s++)
                            cell.outline.push_back({a.x + (b.x - a.x) * s / D, a.y + (b.y - a.y) * s / D});
                    }
                    h3::IJK ijk = {i, j, 0};
                    h3::ijk_normalize(ijk);
                    cell.id = (int64_t)h3::face_ijk_to_h3(face, ijk, res);
                    // densified clip polygon: SH on the densified (still convex) hexagon keeps the
                    // cell boundary within ~1/D^2 of the great-circle arcs once mapped back
                    cell.clip = cell.outline;
                    const llclip::Geom gg = ri.geom(geom_parts[g], geom_parts[g + 1]);
                    emit_cell_ll(cs, (int32_t)g, cell, pl, geo, gg, 1e-3, keep_core_geom,
                                 [&](P2 h) { return fp.to_geo(h); }, 1e-12,
                                 [&](llclip::Cell& C) { return h3_cell_ll(cell.id, C); }, D == 1);
                }
            }
        } else {
            static const double edge_by_res[] = {0, 100000, 10000, 1000, 100, 10, 1};
            int ar = res < 0 ? -res : res;
            double e = res > 0 ? edge_by_res[ar] : edge_by_res[ar - 1] / 2.0;  // negative res: quadrants
            if (res == -1) e = 500000;
            double x0 = 1e300, y0 = 1e300, x1 = -1e300, y1 = -1e300;
            for (auto& part : geo)
                for (auto& ring : part)
                    for (auto& p : ring) {
                        x0 = std::min(x0, p.x);
                        x1 = std::max(x1, p.x);
                        y0 = std::min(y0, p.y);
                        y1 = std::max(y1, p.y);
                    }
            long ilo = (long)floor(x0 / e), ihi = (long)floor(x1 / e), jlo = (long)floor(y0 / e), jhi = (long)floor(y1 / e);
            for (long j = jlo; j <= jhi; j++)
                for (long i = ilo; i <= ihi; i++) {
                    Cell cell;
                    double cx0 = i * e, cy0 = j * e;
                    cell.clip = {{cx0, cy0}, {cx0 + e, cy0}, {cx0 + e, cy0 + e}, {cx0, cy0 + e}};
                    cell.outline = cell.clip;
                    int64_t id;
                    if (!bng::point_to_index(cx0 + 0.5 * e, cy0 + 0.5 * e, res, &id)) continue;
                    cell.id = id;
                    const llclip::Geom gg = ri.geom(geom_parts[g], geom_parts[g + 1]);
                    emit_cell_ll(cs, (int32_t)g, cell, geo, geo, gg, 1e-9 * e, keep_core_geom, [](P2 h) { return h; },
                                 1e-12 * e * e, [&](llclip::Cell& C) { return bng_cell_ll(cx0, cy0, e, C); }, true);
                }
        }
    }
    *out = cs;
    return MOSAIC_OK;
}

// H3 branch of mosaic_tessellate_gpu: candidates, hexagon clip polygons and face-plane rings exactly as
// mosaic_tessellate's H3 branch builds them; the classification runs in k_tess_classify_poly.
static int tessellate_gpu_h3(mosaic_ctx* ctx, int res, int64_t n_geoms, const int64_t* geom_parts,
                             const int64_t* part_rings, const int64_t* ring_offsets, const double* xy,
                             int keep_core_geom, int densify, mosaic_chip_set** out) {
    const RingIdx ri(n_geoms, geom_parts, part_rings, ring_offsets, xy);
    if (res < 0 || res > 15)
        return mosaic_tess_fail(MOSAIC_E_RES, ("H3 resolution has to be between 0 and 15; found " + std::to_string(res)).c_str());
    if (densify < 1 || densify > 64) return mosaic_tess_fail(MOSAIC_E_ARG, "densify must be in [1, 64]");
    TessTrace trace;
    const int D = densify, nv = 6 * D;
    const int64_t n_verts = n_geoms ? ring_offsets[part_rings[geom_parts[n_geoms]]] : 0;
    std::vector<double> pxy((size_t)std::max<int64_t>(n_verts, 1) * 2);
    std::vector<int> gface(n_geoms, -1);
    std::vector<int32_t> cg;
    std::vector<double> cxy;  // candidate hexagon centres in the face plane
    std::vector<int64_t> cid;
    std::vector<int64_t> multi_geoms;  // geometries spanning icosahedron faces
    const double s60 = 0.86602540378443864676, R = 0.57735026918962576451;
    // candidate k's (densified) hexagon clip polygon, nv points: the host producer's arithmetic
    auto fill_clip = [&](int64_t k, double* out_pts) {
        const double cx = cxy[2 * (size_t)k], cy = cxy[2 * (size_t)k + 1];
        P2 corners[6];
        for (int q = 0; q < 6; q++) corners[q] = {cx + hex_corners().dx[q], cy + hex_corners().dy[q]};
        int m = 0;
        for (int q = 0; q < 6; q++) {
            P2 a = corners[q], b = corners[(q + 1) % 6];
            for (int t = 0; t < D; t++) {
                out_pts[m++] = a.x + (b.x - a.x) * t / D;
                out_pts[m++] = a.y + (b.y - a.y) * t / D;
            }
        }
    };
    // per geometry (host threads, independent): face check, face-plane vertices (disjoint ranges of
    // pxy) and the lattice window; then the candidates counted, offsets by a prefix sum, and filled in
    // place (geometry order) by the threads again -- no per-geometry vectors, no concatenation
    struct GeomWin {
        int face = -1, jlo = 0, jhi = -1;
        bool multi = false;
        double x0 = 0, y0 = 0, x1 = 0, y1 = 0;
        int64_t count = 0;
    };
    std::vector<GeomWin> gw((size_t)n_geoms);
    auto window_of = [&](int64_t g, std::vector<double>& u) {
        GeomWin& w = gw[(size_t)g];
        const int64_t v0 = ring_offsets[part_rings[geom_parts[g]]], v1 = ring_offsets[part_rings[geom_parts[g + 1]]];
        if (v0 == v1) return;
        int face = -1;
        // unit vectors once per vertex (face test and projection: the same doubles as face_of / to_hex)
        u.resize((size_t)(v1 - v0) * 3);
        for (int64_t v = v0; v < v1; v++) {
            double* pu = u.data() + 3 * (v - v0);
            FacePlane::unit(xy[2 * v], xy[2 * v + 1], pu);
            int f = face_of_unit(pu);
            if (face < 0) face = f;
            w.multi = w.multi || f != face;
        }
        if (w.multi) return;  // spans faces: the host's per-face pieces (tessellate_h3_multiface)
        w.face = face;
        FacePlane fp;
        fp.init(face, res);
        double x0 = 1e300, y0 = 1e300, x1 = -1e300, y1 = -1e300;
        for (int64_t v = v0; v < v1; v++) {
            P2 p = fp.to_hex_unit(u.data() + 3 * (v - v0));
            pxy[2 * v] = p.x;
            pxy[2 * v + 1] = p.y;
            x0 = std::min(x0, p.x);
            x1 = std::max(x1, p.x);
            y0 = std::min(y0, p.y);
            y1 = std::max(y1, p.y);
        }
        w.x0 = x0, w.y0 = y0, w.x1 = x1, w.y1 = y1;
        w.jlo = (int)floor(y0 / s60) - 2;
        w.jhi = (int)ceil(y1 / s60) + 2;
        int64_t cnt = 0;
        for (int j = w.jlo; j <= w.jhi; j++) {
            int ilo = (int)floor(x0 + j * 0.5) - 2, ihi = (int)ceil(x1 + j * 0.5) + 2;
            for (int i = ilo; i <= ihi; i++) {
                double cx = i - 0.5 * j, cy = j * s60;
                if (cx + R < x0 || cx - R > x1 || cy + R < y0 || cy - R > y1) continue;
                cnt++;
            }
        }
        w.count = cnt;
    };
    std::vector<int64_t> cand0((size_t)n_geoms + 1, 0);
    auto fill_of = [&](int64_t g) {
        const GeomWin& w = gw[(size_t)g];
        if (w.multi || w.face < 0) return;
        int64_t o = cand0[(size_t)g];
        for (int j = w.jlo; j <= w.jhi; j++) {
            int ilo = (int)floor(w.x0 + j * 0.5) - 2, ihi = (int)ceil(w.x1 + j * 0.5) + 2;
            for (int i = ilo; i <= ihi; i++) {
                double cx = i - 0.5 * j, cy = j * s60;
                if (cx + R < w.x0 || cx - R > w.x1 || cy + R < w.y0 || cy - R > w.y1) continue;
                cxy[2 * (size_t)o] = cx;
                cxy[2 * (size_t)o + 1] = cy;
                h3::IJK ijk = {i, j, 0};
                h3::ijk_normalize(ijk);
                cid[(size_t)o] = (int64_t)h3::face_ijk_to_h3(w.face, ijk, res);
                cg[(size_t)o] = (int32_t)g;
                o++;
            }
        }
    };
    {
        const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(
            std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency())), n_geoms / 8));
        auto pool_run = [&](auto body) {
            std::atomic<int64_t> next(0);
            auto work = [&]() {
                std::vector<double> u;
                for (int64_t g0; (g0 = next.fetch_add(64)) < n_geoms;)
                    for (int64_t g = g0; g < std::min<int64_t>(g0 + 64, n_geoms); g++) body(g, u);
            };
            std::vector<std::thread> pool;
            for (int k = 1; k < nt; k++) pool.emplace_back(work);
            work();
            for (auto& th : pool) th.join();
        };
        pool_run([&](int64_t g, std::vector<double>& u) { window_of(g, u); });
        for (int64_t g = 0; g < n_geoms; g++) {
            cand0[(size_t)g + 1] = cand0[(size_t)g] + gw[(size_t)g].count;
            if (gw[(size_t)g].multi) multi_geoms.push_back(g);
            gface[g] = gw[(size_t)g].face;
        }
        const int64_t total = cand0[(size_t)n_geoms];
        cxy.resize((size_t)total * 2);
        cid.resize((size_t)total);
        cg.resize((size_t)total);
        pool_run([&](int64_t g, std::vector<double>&) { fill_of(g); });
    }
    gw.clear();
    trace.mark("h3 candidates (host)");
    // candidates in chunks, so the clip polygons staged on the host and the device stay bounded
    // (<= 64 MB of them per chunk) for any densify and envelope; chips come out in candidate order
    const int64_t n_cand = (int64_t)cg.size();
    const int64_t chunk = std::max<int64_t>(1, ((int64_t)64 << 20) / ((int64_t)nv * 16));
    std::vector<uint8_t> cls;
    std::vector<int64_t> tasks;
    mosaic_chip_set* cs = new mosaic_chip_set();
    // the face-spanning geometries before geometry `upto`, emitted where the host producer emits them
    size_t next_multi = 0;
    // face-spanning geometries: their per-face pieces made on the host (multiface_pieces), classified
    // and clipped on the device like every other candidate -- one session over virtual geometries
    // (geometry, face), the pieces as explicit clip polygons -- and emitted in geometry order
    // (multiface_emit), so the chips are the host producer's
    std::vector<MultiFace> mfs(multi_geoms.size());
    std::vector<Geo3> mgeos;
    if (!multi_geoms.empty()) {
        if (int rc = multiface_gpu(ctx, multi_geoms, geom_parts, part_rings, ring_offsets, xy, res, D, mfs, mgeos)) {
            delete cs;
            return rc;
        }
    }
    trace.mark("face-spanning pieces (GPU)");
    auto flush_multi = [&](int64_t upto) -> int {
        for (; next_multi < multi_geoms.size() && multi_geoms[next_multi] < upto; next_multi++)
        {
            const int64_t g = multi_geoms[next_multi];
            const llclip::Geom gg = ri.geom(geom_parts[g], geom_parts[g + 1]);
            multiface_emit(cs, (int32_t)g, res, keep_core_geom, mfs[next_multi], mgeos[next_multi], gg);
        }
        return MOSAIC_OK;
    };
    // one device session for the batch: geometry uploaded once, per chunk only the candidate centres;
    // clip polygons generated, classified and the border ones clipped on the device
    tessclip::H3Session* S = nullptr;
    struct SessionEnd {
        tessclip::H3Session*& s;
        ~SessionEnd() { tessclip::h3_session_end(s); }
    } session_end{S};
    if (n_cand > 0) {
        if (int rc = tessclip::h3_session_begin(ctx, n_geoms, geom_parts, part_rings, ring_offsets, pxy.data(), xy,
                                                gface.data(), res, D, hex_corners().dx, hex_corners().dy, &S)) {
            delete cs;
            return rc;
        }
    }
    trace.mark("h3 session upload");
    double clip_kernel_ms = 0;
    for (int64_t k0 = 0; k0 < n_cand; k0 += chunk) {
        const int64_t nc = std::min<int64_t>(chunk, n_cand - k0);
        cls.assign((size_t)nc, 0);
        trace.add(0);
        ClippedChips cc;
        int rc = tessclip::h3_session_chunk(S, nc, cg.data() + k0, cxy.data() + 2 * (size_t)k0, 1e-3, cls.data(), tasks,
                                            &cc.r, cid.data() + k0);
        trace.add(1);
        clip_kernel_ms += cc.r.kernel_ms;
        if (rc) {
            delete cs;
            return rc;
        }
        trace.add(2);
        cc.index(nc, tasks);
        // core chips' geometry (indexToGeometry of the cell) from the device: h3ToGeoBoundary costs ~56
        // us per cell on the host (x87-exact steps emulated), the whole res-11 NYC build on 16 threads
        std::vector<int64_t> core_ids;
        std::vector<int32_t> core_idx, core_cnt;
        std::vector<double> core_v;
        if (keep_core_geom && D == 1) {
            core_idx.assign((size_t)nc, -1);
            for (int64_t kk = 0; kk < nc; kk++)
                if (cls[kk] == 1) core_idx[(size_t)kk] = (int32_t)core_ids.size(), core_ids.push_back(cid[k0 + kk]);
            if ((rc = tessclip::h3_cell_vertices(S, core_ids, core_v, core_cnt))) {
                delete cs;
                return rc;
            }
        }
        trace.add(3);
        // the chunk's chips on host threads (each candidate's chip is independent: GPU-clipped border
        // chips to WKB, core chips' outlines, cells the GPU clipper left to the host).  Thread t takes
        // candidates [nc t / nt, nc (t + 1) / nt): GPU-clipped chips are sized first and written in
        // place into the chip set afterwards (offsets by a prefix sum); the others are built into the
        // thread's buffer and copied.  (With face-spanning geometries in the batch, whose chips are
        // emitted between these, every chip goes through the thread buffers and is appended in order.)
        struct OneChip {
            int64_t off = 0;   // in the thread's buffer (built chips), then in the chip set's wkb
            int32_t len = -1;  // -1: no chip
            uint8_t core = 0, built = 0;
        };
        std::vector<OneChip> chips((size_t)nc);
        const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(
            std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency())), nc / 256));
        std::vector<WkbOut> bufs((size_t)nt);
        const bool direct = multi_geoms.empty();
        {
            auto work = [&](int t) {
                std::vector<std::vector<std::vector<P2>>> geo, pl;
                FacePlane fp;
                fp.init(0, res);
                int64_t cur = -1;
                mosaic_chip_set tmp;
                std::vector<double> P((size_t)nv * 2);  // the cell's clip polygon (core / host-clipped cells)
                WkbOut& w = bufs[(size_t)t];
                for (int64_t kk = nc * t / nt; kk < nc * (t + 1) / nt; kk++) {
                    const int64_t k = k0 + kk;
                    OneChip& o = chips[(size_t)kk];
                    if (!cls[kk]) continue;
                    o.off = (int64_t)w.b.size();
                    if (cls[kk] == 2 && !cc.redo(kk)) {
                        // (a chip equal to its cell is a core chip, geometry kept only with keep_core_geom)
                        o.core = cc.is_cell(kk);
                        if (o.core && !keep_core_geom) {
                            WkbSize z;
                            if (cc.chip(kk, z)) o.len = 0;
                        } else if (direct) {
                            WkbSize z;
                            if (cc.chip(kk, z)) o.len = (int32_t)z.n;
                        } else {
                            o.built = 1;
                            if (cc.chip(kk, w)) o.len = (int32_t)((int64_t)w.b.size() - o.off);
                        }
                        continue;
                    }
                    o.built = 1;
                    if (cls[kk] == 1 && !core_idx.empty()) {
                        // (h3_cell_ll's cell from the device's vertices; a cell that is not a planar polygon
                        // takes emit_cell_ll below, whose core chip is then the face-plane outline)
                        const int32_t ci = core_idx[(size_t)kk], nb = core_cnt[(size_t)ci];
                        llclip::Cell C;
                        if (nb >= 3 && nb <= 10) {
                            C.nc = nb;
                            for (int q = 0; q < nb; q++) C.v[q] = {core_v[20 * (size_t)ci + 2 * q], core_v[20 * (size_t)ci + 2 * q + 1]};
                            llclip::cell_init(C);
                            if (llclip::cell_ok(C, true)) {
                                const std::vector<uint8_t> blob = to_wkb({{cell_ll_ring(C)}});
                                o.core = 1;
                                w.b.insert(w.b.end(), blob.begin(), blob.end());
                                o.len = (int32_t)blob.size();
                                continue;
                            }
                        }
                    }
                    if (cg[k] != cur) {
                        cur = cg[k];
                        fp.init(gface[cur], res);
                        geo.clear();
                        pl.clear();
                        for (int64_t p = geom_parts[cur]; p < geom_parts[cur + 1]; p++) {
                            std::vector<std::vector<P2>> rings, prings;
                            for (int64_t r = part_rings[p]; r < part_rings[p + 1]; r++) {
                                std::vector<P2> ring, pring;
                                for (int64_t v = ring_offsets[r]; v < ring_offsets[r + 1]; v++) {
                                    ring.push_back({xy[2 * v], xy[2 * v + 1]});
                                    pring.push_back({pxy[2 * v], pxy[2 * v + 1]});
                                }
                                rings.push_back(std::move(ring));
                                prings.push_back(std::move(pring));
                            }
                            geo.push_back(std::move(rings));
                            pl.push_back(std::move(prings));
                        }
                    }
                    Cell cell;
                    fill_clip(k, P.data());
                    for (int v = 0; v < nv; v++) cell.outline.push_back({P[2 * v], P[2 * v + 1]});
                    cell.clip = cell.outline;
                    cell.id = cid[k];
                    tmp.is_core.clear();
                    tmp.index_id.clear();
                    tmp.key.clear();
                    tmp.wkb_offsets.assign(1, 0);
                    tmp.wkb.clear();
                    const llclip::Geom gg = ri.geom(geom_parts[cur], geom_parts[cur + 1]);
                    emit_cell_ll(&tmp, (int32_t)cur, cell, pl, geo, gg, 1e-3, keep_core_geom, [&](P2 h) { return fp.to_geo(h); },
                                 1e-12, [&](llclip::Cell& C) { return h3_cell_ll(cell.id, C); }, D == 1, (int)cls[kk]);
                    if (!tmp.index_id.empty()) {
                        o.core = tmp.is_core[0] != 0;
                        w.b.insert(w.b.end(), tmp.wkb.begin(), tmp.wkb.end());
                        o.len = (int32_t)tmp.wkb.size();
                    }
                }
            };
            std::vector<std::thread> pool;
            for (int t = 1; t < nt; t++) pool.emplace_back(work, t);
            work(0);
            for (auto& th : pool) th.join();
        }
        if (direct) {
            // offsets, index columns, then the WKB written in place by the threads
            int64_t n_chips = 0, n_bytes = 0;
            for (auto& o : chips)
                if (o.len >= 0) n_chips++, n_bytes += o.len;
            const size_t c0 = cs->index_id.size(), w0 = cs->wkb.size();
            cs->is_core.resize(c0 + (size_t)n_chips);
            cs->index_id.resize(c0 + (size_t)n_chips);
            cs->key.resize(c0 + (size_t)n_chips);
            cs->wkb_offsets.resize(c0 + 1 + (size_t)n_chips);
            cs->wkb.resize(w0 + (size_t)n_bytes);
            std::vector<int64_t> src_off((size_t)nc, 0);
            size_t ci = c0;
            int64_t wo = (int64_t)w0;
            for (int64_t kk = 0; kk < nc; kk++) {
                OneChip& o = chips[(size_t)kk];
                if (o.len < 0) continue;
                cs->is_core[ci] = o.core;
                cs->index_id[ci] = cid[k0 + kk];
                cs->key[ci] = cg[k0 + kk];
                src_off[(size_t)kk] = o.off;
                o.off = wo;
                wo += o.len;
                cs->wkb_offsets[++ci] = wo;
            }
            trace.add(4);
            auto write = [&](int t) {
                for (int64_t kk = nc * t / nt; kk < nc * (t + 1) / nt; kk++) {
                    const OneChip& o = chips[(size_t)kk];
                    if (o.len <= 0) continue;
                    if (o.built) {
                        memcpy(cs->wkb.data() + o.off, bufs[(size_t)t].b.data() + src_off[(size_t)kk], (size_t)o.len);
                    } else {
                        WkbPtr w{cs->wkb.data() + o.off};
                        cc.chip(kk, w);
                    }
                }
            };
            std::vector<std::thread> pool;
            for (int t = 1; t < nt; t++) pool.emplace_back(write, t);
            write(0);
            for (auto& th : pool) th.join();
            trace.add(5);
            continue;
        }
        trace.add(4);
        int64_t n_chips = 0, n_bytes = 0;
        for (auto& o : chips)
            if (o.len >= 0) n_chips++, n_bytes += o.len;
        cs->is_core.reserve(cs->is_core.size() + (size_t)n_chips);
        cs->index_id.reserve(cs->index_id.size() + (size_t)n_chips);
        cs->key.reserve(cs->key.size() + (size_t)n_chips);
        cs->wkb_offsets.reserve(cs->wkb_offsets.size() + (size_t)n_chips);
        cs->wkb.reserve(cs->wkb.size() + (size_t)n_bytes);
        for (int t = 0; t < nt; t++) {
            const std::vector<uint8_t>& b = bufs[(size_t)t].b;
            const size_t wkb0 = cs->wkb.size();
            // face-spanning geometries are emitted between chips: then chip by chip
            const bool interleaved = !multi_geoms.empty();
            for (int64_t kk = nc * t / nt; kk < nc * (t + 1) / nt; kk++) {
                const int64_t k = k0 + kk;
                if (interleaved && (rc = flush_multi(cg[k]))) {
                    delete cs;
                    return rc;
                }
                const OneChip& o = chips[(size_t)kk];
                if (o.len < 0) continue;
                cs->is_core.push_back(o.core);
                cs->index_id.push_back(cid[k]);
                cs->key.push_back(cg[k]);
                if (interleaved) {
                    cs->wkb.insert(cs->wkb.end(), b.begin() + o.off, b.begin() + o.off + o.len);
                    cs->wkb_offsets.push_back((int64_t)cs->wkb.size());
                } else {
                    cs->wkb_offsets.push_back((int64_t)(wkb0 + (size_t)o.off + (size_t)o.len));
                }
            }
            if (!interleaved) cs->wkb.insert(cs->wkb.end(), b.begin(), b.end());
        }
        trace.add(5);
    }
    if (int rc = flush_multi(n_geoms)) {
        delete cs;
        return rc;
    }
    trace.add(5);
    if (trace.on)
        fprintf(stderr, "[tess] chunk setup %.3f ms, device classify + clip %.3f ms (clip kernel %.3f ms), index clips %.3f ms, "
                        "chip WKB (threads) %.3f ms, append %.3f ms\n",
                trace.acc[0], trace.acc[1], clip_kernel_ms, trace.acc[3], trace.acc[4], trace.acc[5]);
    *out = cs;
    return MOSAIC_OK;
}

// grid_tessellateexplode with the per-cell classification (the O(segments x cells)
// part of the producer) on the GPU (k_bng_tess_classify); border cells are clipped on the host
// exactly as mosaic_tessellate does, so the chip set is identical row for row and byte for byte.
int mosaic_tessellate_gpu(mosaic_ctx* ctx, int grid, int res, int64_t n_geoms, const int64_t* geom_parts,
                          const int64_t* part_rings, const int64_t* ring_offsets, const double* xy,
                          int keep_core_geom, int densify, mosaic_chip_set** out) {
    const RingIdx ri(n_geoms, geom_parts, part_rings, ring_offsets, xy);
    if (!ctx || !out || n_geoms < 0 || (n_geoms > 0 && (!geom_parts || !part_rings || !ring_offsets || !xy)))
        return mosaic_tess_fail(MOSAIC_E_ARG, "invalid argument");
    if (grid == MOSAIC_GRID_H3)
        return tessellate_gpu_h3(ctx, res, n_geoms, geom_parts, part_rings, ring_offsets, xy, keep_core_geom, densify,
                                 out);
    if (grid != MOSAIC_GRID_BNG) return mosaic_tess_fail(MOSAIC_E_ARG, "unknown grid");
    if (!(res != 0 && res >= -6 && res <= 6))
        return mosaic_tess_fail(MOSAIC_E_RES, ("BNG resolution not supported; found " + std::to_string(res)).c_str());
    static const double edge_by_res[] = {0, 100000, 10000, 1000, 100, 10, 1};
    const int ar = res < 0 ? -res : res;
    double e = res > 0 ? edge_by_res[ar] : edge_by_res[ar - 1] / 2.0;  // negative res: quadrants
    if (res == -1) e = 500000;
    // candidates in mosaic_tessellate's order: geometry, then row j, then column i
    std::vector<int32_t> cg;
    std::vector<int64_t> cij, cid;
    for (int64_t g = 0; g < n_geoms; g++) {
        double x0 = 1e300, y0 = 1e300, x1 = -1e300, y1 = -1e300;
        bool any = false;
        for (int64_t p = geom_parts[g]; p < geom_parts[g + 1]; p++)
            for (int64_t r = part_rings[p]; r < part_rings[p + 1]; r++)
                for (int64_t v = ring_offsets[r]; v < ring_offsets[r + 1]; v++) {
                    any = true;
                    x0 = std::min(x0, xy[2 * v]);
                    x1 = std::max(x1, xy[2 * v]);
                    y0 = std::min(y0, xy[2 * v + 1]);
                    y1 = std::max(y1, xy[2 * v + 1]);
                }
        if (!any) continue;
        long ilo = (long)floor(x0 / e), ihi = (long)floor(x1 / e), jlo = (long)floor(y0 / e), jhi = (long)floor(y1 / e);
        for (long j = jlo; j <= jhi; j++)
            for (long i = ilo; i <= ihi; i++) {
                double cx0 = i * e, cy0 = j * e;
                int64_t id;
                if (!bng::point_to_index(cx0 + 0.5 * e, cy0 + 0.5 * e, res, &id)) continue;
                cg.push_back((int32_t)g);
                cij.push_back(i);
                cij.push_back(j);
                cid.push_back(id);
            }
    }
    const int64_t n_cand = (int64_t)cg.size();
    std::vector<uint8_t> cls(n_cand);
    int rc = mosaic_tess_classify_bng(ctx, n_geoms, geom_parts, part_rings, ring_offsets, xy, n_cand, cg.data(),
                                      cij.data(), e, 1e-9 * e, cls.data());
    if (rc) return rc;
    // border cells clipped on the GPU (k_tess_clip_ll) against their squares, as emit_cell_ll does
    std::vector<int64_t> tasks;
    for (int64_t k = 0; k < n_cand; k++)
        if (cls[k] == 2) tasks.push_back(k);
    std::vector<double> sq((size_t)n_cand * 8);
    for (int64_t k = 0; k < n_cand; k++) {
        llclip::Cell C;
        bng_cell_ll(cij[2 * k] * e, cij[2 * k + 1] * e, e, C);
        for (int v = 0; v < 4; v++) {
            sq[8 * (size_t)k + 2 * v] = C.v[v].x;
            sq[8 * (size_t)k + 2 * v + 1] = C.v[v].y;
        }
    }
    ClippedChips cc;
    if ((rc = tessclip::clip_ll(ctx, n_geoms, geom_parts, part_rings, ring_offsets, xy, tasks, cg.data(), n_cand, sq.data(), 4,
                                &cc.r)))
        return rc;
    cc.index(n_cand, tasks);
    mosaic_chip_set* cs = new mosaic_chip_set();
    std::vector<std::vector<std::vector<P2>>> geo;
    int64_t cur = -1;
    for (int64_t k = 0; k < n_cand; k++) {
        if (!cls[k]) continue;
        if (cls[k] == 2 && !cc.redo(k)) {
            WkbOut w;
            const bool core = cc.is_cell(k);
            if (cc.chip(k, w)) cs->add(core, cid[k], cg[k], core && !keep_core_geom ? std::vector<uint8_t>() : w.b);
            continue;
        }
        if (cg[k] != cur) {
            cur = cg[k];
            geo.clear();
            for (int64_t p = geom_parts[cur]; p < geom_parts[cur + 1]; p++) {
                std::vector<std::vector<P2>> rings;
                for (int64_t r = part_rings[p]; r < part_rings[p + 1]; r++) {
                    std::vector<P2> ring;
                    for (int64_t v = ring_offsets[r]; v < ring_offsets[r + 1]; v++) ring.push_back({xy[2 * v], xy[2 * v + 1]});
                    rings.push_back(std::move(ring));
                }
                geo.push_back(std::move(rings));
            }
        }
        Cell cell;
        const double cx0 = cij[2 * k] * e, cy0 = cij[2 * k + 1] * e;
        cell.clip = {{cx0, cy0}, {cx0 + e, cy0}, {cx0 + e, cy0 + e}, {cx0, cy0 + e}};
        cell.outline = cell.clip;
        cell.id = cid[k];
        const llclip::Geom gg = ri.geom(geom_parts[cur], geom_parts[cur + 1]);
        emit_cell_ll(cs, (int32_t)cur, cell, geo, geo, gg, 1e-9 * e, keep_core_geom, [](P2 h) { return h; }, 1e-12 * e * e,
                     [&](llclip::Cell& C) { return bng_cell_ll(cx0, cy0, e, C); }, true, (int)cls[k]);
    }
    *out = cs;
    return MOSAIC_OK;
}

// chips clipped by the reference-style clip on the host, and cells that fell back to the plane clip
// (process-wide counters; tests assert no fallback on their inputs)
int mosaic_tess_counters(int64_t* ll_chips, int64_t* ll_fallbacks) {
    if (ll_chips) *ll_chips = g_ll_chips.load();
    if (ll_fallbacks) *ll_fallbacks = g_ll_fallbacks.load();
    return MOSAIC_OK;
}

int mosaic_chip_set_info(const mosaic_chip_set* cs, int64_t* n_chips, int64_t* wkb_bytes) {
    if (!cs || !n_chips || !wkb_bytes) return mosaic_tess_fail(MOSAIC_E_ARG, "null argument");
    *n_chips = (int64_t)cs->index_id.size();
    *wkb_bytes = (int64_t)cs->wkb.size();
    return MOSAIC_OK;
}

int mosaic_chip_set_columns(const mosaic_chip_set* cs, const uint8_t** is_core, const int64_t** index_id,
                            const int32_t** key, const int64_t** wkb_offsets, const uint8_t** wkb) {
    if (!cs || !is_core || !index_id || !key || !wkb_offsets || !wkb) return mosaic_tess_fail(MOSAIC_E_ARG, "null argument");
    *is_core = cs->is_core.data();
    *index_id = cs->index_id.data();
    *key = cs->key.data();
    *wkb_offsets = cs->wkb_offsets.data();
    *wkb = cs->wkb.data();
    return MOSAIC_OK;
}

int mosaic_chip_set_export(const mosaic_chip_set* cs, uint8_t* is_core, int64_t* index_id, int32_t* key,
                           int64_t* wkb_offsets, uint8_t* wkb) {
    if (!cs) return mosaic_tess_fail(MOSAIC_E_ARG, "null chip set");
    size_t n = cs->index_id.size();
    if (is_core) memcpy(is_core, cs->is_core.data(), n);
    if (index_id) memcpy(index_id, cs->index_id.data(), n * 8);
    if (key) memcpy(key, cs->key.data(), n * 4);
    if (wkb_offsets) memcpy(wkb_offsets, cs->wkb_offsets.data(), (n + 1) * 8);
    if (wkb && !cs->wkb.empty()) memcpy(wkb, cs->wkb.data(), cs->wkb.size());
    return MOSAIC_OK;
}

int mosaic_chip_set_destroy(mosaic_chip_set* cs) {
    delete cs;
    return MOSAIC_OK;
}

}  // extern "C"
