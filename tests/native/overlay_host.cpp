// CPU build of the st_intersection_aggregate unit overlay (mosaic_amd/csrc/overlay.h, the device code
// compiled by g++), so tests/test_intersection_agg.py can check it against the exact oracle without a
// GPU: the boundary of (union of A's parts) n (union of B's parts) as directed edges, and its area.
#include <stdint.h>

#include <vector>

#include "overlay.h"

using namespace mosaic;

namespace {
struct Store {
    std::vector<pip::Vec2> v;
    std::vector<uint32_t> rs{0}, pr{0}, gp{0};
    std::vector<pip::Box> rb, gb;
    // parts: n_rings rings with ring_off[n_rings + 1] into xy, part_rings[n_parts + 1]; one geometry
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

// need: 1 = A, 2 = B, 3 = both (a set not needed has no parts passed: it covers everything).
// Returns the edge count (out: 4 doubles per edge, cap edges), -1 on overflow; *area the shoelace area.
extern "C" int overlay_host(const double* xa, const int64_t* ra, int nra, const int64_t* pa, int npa, const double* xb,
                            const int64_t* rb, int nrb, const int64_t* pb, int npb, int need, double* out, int cap,
                            double* area) {
    Store A(xa, ra, nra, pa, npa), B(xb, rb, nrb, pb, npb);
    const pip::GeomStore st[2] = {A.view(), B.view()};
    std::vector<overlay::PartRef> parts;
    int ne = 0;
    if (need & overlay::kNeedA)
        for (int p = 0; p < npa; p++) parts.push_back({(uint32_t)p, 0, 0, 0}), ne += overlay::part_edges(st[0], p);
    if (need & overlay::kNeedB)
        for (int p = 0; p < npb; p++) parts.push_back({(uint32_t)p, 1, 0, 0}), ne += overlay::part_edges(st[1], p);
    std::vector<char> buf((size_t)overlay::scratch_bytes(ne) + 64);
    overlay::Scratch sc = overlay::make_scratch((void*)(((uintptr_t)buf.data() + 63) & ~(uintptr_t)63), ne);
    return overlay::unit_boundary(st, parts.data(), (int)parts.size(), need, sc, out, cap, area);
}
