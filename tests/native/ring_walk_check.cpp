// CPU check of the tile join's ring walks (mosaic_amd/csrc/ring_walk.h): the branch-free walk with
// its filter fallback, and the exact walk, equal pip::locate_in_ring == INTERIOR (JTS semantics) on
// random rings and adversarial points (vertices, points on edges, horizontal edges, points on the
// rays through vertices, collinear vertices).  Prints: cases, mismatches.
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

#include "../../mosaic_amd/csrc/ring_walk.h"

using namespace mosaic;

int main(int argc, char** argv) {
    const int n_rings = argc > 1 ? atoi(argv[1]) : 20000;
    std::mt19937_64 rng(11);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    long cases = 0, bad = 0;
    for (int r = 0; r < n_rings; r++) {
        // a ring of 4-12 vertices around (cx, cy): lon/lat-like magnitudes, some on a coarse grid
        // (axis-aligned and collinear edges), closed
        const int m = 4 + (int)(rng() % 9);
        const bool grid = (r % 3) == 0;
        const double cx = -74.0 + 0.5 * U(rng), cy = 40.7 + 0.5 * U(rng), sc = 1e-4 * (1.0 + 9.0 * (U(rng) + 1.0));
        std::vector<ringwalk::V2> v((size_t)m + 1);
        for (int k = 0; k < m; k++) {
            const double a = 6.283185307179586 * (k + 0.3 * U(rng)) / m, rad = sc * (0.5 + 0.5 * (U(rng) + 1.0));
            double x = cx + rad * cos(a), y = cy + rad * sin(a);
            if (grid) {
                x = cx + sc * 0.25 * (double)(long)(4.0 * (x - cx) / sc);
                y = cy + sc * 0.25 * (double)(long)(4.0 * (y - cy) / sc);
            }
            v[(size_t)k] = {x, y};
        }
        v[(size_t)m] = v[0];
        std::vector<pip::Vec2> pv((size_t)m + 1);
        for (int k = 0; k <= m; k++) pv[(size_t)k] = {v[(size_t)k].x, v[(size_t)k].y};
        std::vector<std::pair<double, double>> pts;
        for (int q = 0; q < 24; q++) pts.push_back({cx + 1.3 * sc * U(rng), cy + 1.3 * sc * U(rng)});
        for (int k = 0; k < m; k++) {
            const ringwalk::V2 a = v[(size_t)k], b = v[(size_t)k + 1];
            pts.push_back({a.x, a.y});                                   // vertex
            pts.push_back({0.5 * (a.x + b.x), 0.5 * (a.y + b.y)});       // (near) edge midpoint
            pts.push_back({a.x + sc * 0.1 * U(rng), a.y});               // on the ray through a vertex
            pts.push_back({a.x + 0.25 * (b.x - a.x), a.y + 0.25 * (b.y - a.y)});
        }
        for (auto& p : pts) {
            const bool want = pip::locate_in_ring(pv.data(), (uint32_t)m + 1, p.first, p.second) == pip::LOC_INTERIOR;
            const bool ex = ringwalk::ring_interior_exact((const double*)v.data(), (uint32_t)m + 1, p.first, p.second);
            const bool bf = ringwalk::ring_interior((const double*)v.data(), (uint32_t)m + 1, p.first, p.second);
            cases++;
            bad += (ex != want) + (bf != want);
        }
    }
    printf("%ld %ld\n", cases, bad);
    return 0;
}
