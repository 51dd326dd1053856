// CPU build of the st_intersection_aggregate area code (mosaic_amd/csrc/isect_area.h, the device
// code compiled by g++): area(A n B) for two polygonal geometries, the lanes' edge loop run
// sequentially, so tests/test_intersection_agg.py can compare it with the exact oracle without a GPU.
#include <stdint.h>

#include <vector>

#include "isect_area.h"

using namespace mosaic;

namespace {
struct Store {
    std::vector<pip::Vec2> v;
    std::vector<uint32_t> rs{0}, pr{0}, gp{0};
    std::vector<pip::Box> rb, gb;
    // one geometry: n_rings rings with ring_off[n_rings + 1] into xy, part_rings[n_parts + 1]
    Store(const double* xy, const int64_t* ring_off, int n_rings, const int64_t* part_rings, int n_parts) {
        pip::Box g{1e300, 1e300, -1e300, -1e300};
        for (int r = 0; r < n_rings; r++) {
            pip::Box b{1e300, 1e300, -1e300, -1e300};
            for (int64_t i = ring_off[r]; i < ring_off[r + 1]; i++) {
                const double x = xy[2 * i], y = xy[2 * i + 1];
                v.push_back({x, y});
                b.minx = x < b.minx ? x : b.minx;
                b.miny = y < b.miny ? y : b.miny;
                b.maxx = x > b.maxx ? x : b.maxx;
                b.maxy = y > b.maxy ? y : b.maxy;
            }
            rb.push_back(b);
            rs.push_back((uint32_t)v.size());
            g.minx = b.minx < g.minx ? b.minx : g.minx;
            g.miny = b.miny < g.miny ? b.miny : g.miny;
            g.maxx = b.maxx > g.maxx ? b.maxx : g.maxx;
            g.maxy = b.maxy > g.maxy ? b.maxy : g.maxy;
        }
        for (int p = 1; p <= n_parts; p++) pr.push_back((uint32_t)part_rings[p]);
        gp.push_back((uint32_t)n_parts);
        gb.push_back(g);
    }
    pip::GeomStore view() const { return pip::GeomStore{v.data(), rs.data(), rb.data(), pr.data(), gp.data(), gb.data()}; }
};
}  // namespace

extern "C" double isect_area_host(const double* xa, const int64_t* ra, int nra, const int64_t* pa, int npa,
                                  const double* xb, const int64_t* rb, int nrb, const int64_t* pb, int npb) {
    Store A(xa, ra, nra, pa, npa), B(xb, rb, nrb, pb, npb);
    const pip::GeomStore sa = A.view(), sb = B.view();
    const uint32_t na = isect::edge_count(sa, 0);
    const pip::Vec2 o{fmin(sa.geom_bbox[0].minx, sb.geom_bbox[0].minx), fmin(sa.geom_bbox[0].miny, sb.geom_bbox[0].miny)};
    double sum = 0;
    for (uint32_t e = 0; e < na; e++) {
        uint32_t r, v;
        bool shell;
        isect::edge_at(sa, 0, e, &r, &v, &shell);
        const double sga = isect::ring_sign(sa, r, shell);
        for (uint32_t p = sb.geom_part[0]; p < sb.geom_part[1]; p++)
            for (uint32_t rb = sb.part_ring[p]; rb < sb.part_ring[p + 1]; rb++) {
                const double sgb = isect::ring_sign(sb, rb, rb == sb.part_ring[p]);
                for (uint32_t i = sb.ring_start[rb]; i + 1 < sb.ring_start[rb + 1]; i++)
                    sum += isect::pair_term(sa.verts[v].x - o.x, sa.verts[v].y - o.y, sa.verts[v + 1].x - o.x,
                                            sa.verts[v + 1].y - o.y, sga, sb.verts[i].x - o.x, sb.verts[i].y - o.y,
                                            sb.verts[i + 1].x - o.x, sb.verts[i + 1].y - o.y, sgb);
            }
    }
    return sum;
}
