// CPU build of the H3 polyfill kernel pieces (mosaic_amd/csrc/h3_polyfill.h, h3_grid.h kRing(1),
// h3_device.h h3_exact, h3_geom.h h3ToGeo -- the device code compiled by g++), driven by H3 C v3.7's
// sequential _polyfillInternal loop, so tests/test_polyfill.py can compare the kernel code with the
// oracle (oracle/polyfill.c) without a GPU.  One polygon part: rings of (lat, lon) radians.
#include <stdint.h>

#include <unordered_set>
#include <vector>

#include "h3_polyfill.h"

using namespace mosaic;

// returns the count (H3 output order) or -1 (pentagon met / cap)
extern "C" int64_t h3_polyfill_host(const double* lat, const double* lon, const int64_t* ring_off, int n_rings, int res,
                                    int64_t* out, int64_t cap) {
    std::vector<h3fill::Box> boxes;
    int64_t total = 0;
    for (int r = 0; r < n_rings; r++) {
        boxes.push_back(h3fill::bbox_from_loop(lat + ring_off[r], lon + ring_off[r], ring_off[r + 1] - ring_off[r]));
        total += ring_off[r + 1] - ring_off[r];
    }
    const double pr = h3fill::pentagon_radius_km(res);
    int64_t M = h3fill::bbox_hex_estimate(boxes[0], pr);
    if (M < total) M = total;
    M += h3fill::kPolyfillBuffer;
    auto inside = [&](double la, double lo) {
        if (!h3fill::point_inside_loop(lat + ring_off[0], lon + ring_off[0], ring_off[1] - ring_off[0], boxes[0], la, lo))
            return false;
        for (int r = 1; r < n_rings; r++)
            if (h3fill::point_inside_loop(lat + ring_off[r], lon + ring_off[r], ring_off[r + 1] - ring_off[r], boxes[r],
                                          la, lo))
                return false;
        return true;
    };
    std::vector<uint64_t> search;
    std::unordered_set<uint64_t> seen;
    for (int r = 0; r < n_rings; r++) {
        const int64_t s = ring_off[r], n = ring_off[r + 1] - s;
        for (int64_t i = 0; i < n; i++) {
            const int64_t w = i == n - 1 ? s : s + i + 1;
            const int est = h3fill::line_hex_estimate(lat[s + i], lon[s + i], lat[w], lon[w], pr);
            for (int j = 0; j < est; j++) {
                double la, lo;
                h3fill::edge_sample(lat[s + i], lon[s + i], lat[w], lon[w], est, j, &la, &lo);
                const uint64_t h = h3::h3_exact(la, lo, res);
                if (seen.insert(h).second) search.push_back(h);
            }
        }
    }
    std::vector<uint64_t> table((size_t)M, 0), order;
    std::unordered_set<uint64_t> acc;
    while (!search.empty()) {
        std::vector<uint64_t> found;
        for (uint64_t sh : search) {
            int64_t ring[7];
            const int nr = h3fill::kring1(sh, res, ring);
            if (nr < 0) return -1;
            for (int j = 0; j < nr; j++) {
                const uint64_t h = (uint64_t)ring[j];
                if (acc.count(h)) continue;
                double la, lo;
                h3geom::h3_to_geo(h, &la, &lo);
                if (!inside(la, lo)) continue;
                acc.insert(h);
                found.push_back(h);
                uint64_t loc = h % (uint64_t)M;
                while (table[loc]) loc = (loc + 1) % (uint64_t)M;
                table[loc] = h;
            }
        }
        search.swap(found);
    }
    int64_t n = 0;
    for (uint64_t h : table)
        if (h) {
            if (n >= cap) return -1;
            out[n++] = (int64_t)h;
        }
    return n;
}
