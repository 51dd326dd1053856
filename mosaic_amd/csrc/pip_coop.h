// Wave-cooperative JTS contains for gfx950: all 64 lanes of a wavefront evaluate ONE
// (point, chip) test, one ring edge per lane, with coalesced 16-byte vertex loads, then reduce with
// ballot / popcount.  Used by the fused join kernel: after the cell probe, a wave walks its lanes'
// border-chip work items one by one (wave-uniform), instead of every lane running its own divergent
// edge loop over gathered vertices.
//
// Equivalence with the sequential JTS restatement (pip_device.h / oracle/pip.c): RayCrossingCounter
// returns BOUNDARY as soon as any segment reports "on segment", otherwise the crossing parity; every
// segment's contribution (on-segment flag, crossing flag) depends on that segment and the point
// only.  So "any lane on-segment -> BOUNDARY, else parity of the summed crossings" is the same
// answer, whatever the order.  Ring-envelope checks only skip rings whose crossing count is even
// and that cannot touch the point, so they are optional; they are kept (wave-uniform) for speed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pip_device.h"

namespace mosaic {
namespace pip {

__device__ inline int lane_id() { return (int)(threadIdx.x & 63); }

__device__ inline uint32_t readlane_u32(uint32_t v, int src) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, src);
}
__device__ inline double readlane_f64(double v, int src) {
    unsigned long long u = __double_as_longlong(v);
    uint32_t lo = readlane_u32((uint32_t)u, src), hi = readlane_u32((uint32_t)(u >> 32), src);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Ring r of the store, point (px, py) uniform across the wave: LOC_* (wave-uniform).
__device__ inline int coop_locate_in_ring(const GeomStore& s, uint32_t v0, uint32_t n, double px, double py) {
    bool boundary = false;
    int crossings = 0;
    const int lane = lane_id();
    for (uint32_t base = 1; base < n; base += 64) {
        uint32_t i = base + lane;
        bool on = false, cross = false;
        if (i < n) {
            Vec2 p1 = s.verts[v0 + i];
            Vec2 p2 = s.verts[v0 + i - 1];
            if (!(p1.x < px && p2.x < px)) {
                if (px == p2.x && py == p2.y) {
                    on = true;
                } else if (p1.y == py && p2.y == py) {
                    double minx = p1.x < p2.x ? p1.x : p2.x;
                    double maxx = p1.x < p2.x ? p2.x : p1.x;
                    on = (px >= minx && px <= maxx);
                } else if (((p1.y > py) && (p2.y <= py)) || ((p2.y > py) && (p1.y <= py))) {
                    int orient = orientation_index(p1.x, p1.y, p2.x, p2.y, px, py);
                    if (orient == 0) {
                        on = true;
                    } else {
                        if (p2.y < p1.y) orient = -orient;
                        cross = orient == 1;
                    }
                }
            }
        }
        boundary = boundary || (__ballot(on) != 0ULL);
        crossings += __popcll(__ballot(cross));
    }
    if (boundary) return LOC_BOUNDARY;
    return (crossings & 1) ? LOC_INTERIOR : LOC_EXTERIOR;
}

__device__ inline int coop_locate_in_polygon(const GeomStore& s, uint32_t part, double px, double py) {
    uint32_t r0 = s.part_ring[part], r1 = s.part_ring[part + 1];
    if (r1 <= r0) return LOC_EXTERIOR;
    uint32_t v0 = s.ring_start[r0], v1 = s.ring_start[r0 + 1];
    if (v1 <= v0) return LOC_EXTERIOR;
    if (box_excludes(s.ring_bbox[r0], px, py)) return LOC_EXTERIOR;
    int shell = coop_locate_in_ring(s, v0, v1 - v0, px, py);
    if (shell != LOC_INTERIOR) return shell;
    for (uint32_t r = r0 + 1; r < r1; r++) {
        if (box_excludes(s.ring_bbox[r], px, py)) continue;
        uint32_t a = s.ring_start[r], b = s.ring_start[r + 1];
        int hole = coop_locate_in_ring(s, a, b - a, px, py);
        if (hole == LOC_INTERIOR) return LOC_EXTERIOR;
        if (hole == LOC_BOUNDARY) return LOC_BOUNDARY;
    }
    return LOC_INTERIOR;
}

// Geometry.contains(POINT(px py)) for geometry g; g, px, py wave-uniform; result wave-uniform.
__device__ inline bool coop_contains(const GeomStore& s, uint32_t g, double px, double py) {
    uint32_t p0 = s.geom_part[g], p1 = s.geom_part[g + 1];
    if (p1 <= p0) return false;
    if (box_excludes(s.geom_bbox[g], px, py)) return false;
    if (p1 - p0 == 1) return coop_locate_in_polygon(s, p0, px, py) == LOC_INTERIOR;
    bool is_in = false;
    int nb = 0;
    for (uint32_t p = p0; p < p1; p++) {
        int loc = coop_locate_in_polygon(s, p, px, py);
        if (loc == LOC_INTERIOR) is_in = true;
        if (loc == LOC_BOUNDARY) nb++;
    }
    if (nb & 1) return false;
    return nb > 0 || is_in;
}

// Per-edge flags of edge i (1 <= i < n) of ring v[0..n) for point (px, py): the RayCrossingCounter
// contribution of segment (v[i], v[i-1]).
__device__ inline void edge_flags(const Vec2* v, uint32_t i, double px, double py, bool& on, bool& cross) {
    on = false;
    cross = false;
    Vec2 p1 = v[i];
    Vec2 p2 = v[i - 1];
    if (p1.x < px && p2.x < px) return;
    if (px == p2.x && py == p2.y) {
        on = true;
    } else if (p1.y == py && p2.y == py) {
        double minx = p1.x < p2.x ? p1.x : p2.x;
        double maxx = p1.x < p2.x ? p2.x : p1.x;
        on = (px >= minx && px <= maxx);
    } else if (((p1.y > py) && (p2.y <= py)) || ((p2.y > py) && (p1.y <= py))) {
        int orient = orientation_index(p1.x, p1.y, p2.x, p2.y, px, py);
        if (orient == 0) {
            on = true;
        } else {
            if (p2.y < p1.y) orient = -orient;
            cross = orient == 1;
        }
    }
}

// Packed evaluation of up to 4 "simple" work items (chip = one Polygon with one shell ring whose
// envelope already contains the point), each with at most G - 1... G edges: item k owns lanes
// [k*G, (k+1)*G) and lane k*G + j evaluates edge j + 1.  Lanes fetch their item's point and ring
// through ds_bpermute from the owning lane src_k.  ng, G (16 or 32) and src_k are wave-uniform.
// Returns the on-segment and crossing ballots; item k is contained iff its G-bit slice of `on` is
// empty and its slice of `cross` has odd population.
__device__ inline void coop_packed(const Vec2* verts, int ng, int G, int s0, int s1, int s2, int s3, double x, double y,
                                   uint32_t vstart, uint32_t nv, unsigned long long& onm, unsigned long long& crm) {
    const int lane = lane_id();
    const int grp = G == 32 ? (lane >> 5) : (lane >> 4);
    const int gl = lane & (G - 1);
    int my_src = grp == 0 ? s0 : (grp == 1 ? s1 : (grp == 2 ? s2 : s3));
    double px = __shfl(x, my_src, 64);
    double py = __shfl(y, my_src, 64);
    uint32_t vs = (uint32_t)__shfl((int)vstart, my_src, 64);
    uint32_t n = (uint32_t)__shfl((int)nv, my_src, 64);
    uint32_t i = 1u + (uint32_t)gl;
    bool on = false, cross = false;
    if (grp < ng && i < n) edge_flags(verts + vs, i, px, py, on, cross);
    onm = __ballot(on);
    crm = __ballot(cross);
}

// ---- slab-filtered edges --------------------------------------------------------------------
// A ring's segment (p1 = ring[i], p2 = ring[i-1]) can only report "on segment" or "crossing" for a
// point whose y lies in [min(p1.y, p2.y), max(p1.y, p2.y)] (every RayCrossingCounter branch that
// sets a flag requires it).  The chip table therefore keeps, per chip and per horizontal slab of
// its envelope, the list of segments whose y-range meets the (slightly widened) slab, as explicit
// 32-byte records {p1.x, p1.y, p2.x, p2.y}.  Evaluating only the point's slab list gives exactly
// the flags of the whole ring.
// Edge / edge_rec_flags: pip_device.h (shared with the host-side raster self-check).

}  // namespace pip
}  // namespace mosaic
