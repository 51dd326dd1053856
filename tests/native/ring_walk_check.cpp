// CPU check of the tile join's ring walks (mosaic_amd/csrc/ring_walk.h): the branch-free walk with
// its filter fallback, and the exact walk, equal pip::locate_in_ring == INTERIOR (JTS semantics) on
// random rings and adversarial points (vertices, points on edges, horizontal edges, points on the
// rays through vertices, collinear vertices); and the f32 walk, where it decides, equals it too.
// Prints: cases, mismatches, f32 cases, f32 undecided, f32 cases of the random points, undecided
// ones among them.
#include <math.h>
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
    long cases = 0, bad = 0, f32_cases = 0, f32_undecided = 0, f32_random = 0, f32_random_undecided = 0;
    auto down = [](double d) {
        float f = (float)d;
        return (double)f > d ? nextafterf(f, -INFINITY) : f;
    };
    auto up = [](double d) {
        float f = (float)d;
        return (double)f < d ? nextafterf(f, INFINITY) : f;
    };
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
        for (size_t pi = 0; pi < pts.size(); pi++) {
            const auto& p = pts[pi];
            const bool want = pip::locate_in_ring(pv.data(), (uint32_t)m + 1, p.first, p.second) == pip::LOC_INTERIOR;
            const bool ex = ringwalk::ring_interior_exact((const double*)v.data(), (uint32_t)m + 1, p.first, p.second);
            const bool bf = ringwalk::ring_interior((const double*)v.data(), (uint32_t)m + 1, p.first, p.second);
            // the f32 walk in the tile join's chip frame (tile_images.h: outward-rounded f32
            // envelope, vertices float(v - fmin)); only for points inside the f32 envelope, as there
            double bx0 = v[0].x, by0 = v[0].y, bx1 = v[0].x, by1 = v[0].y;
            for (const auto& q : v) {
                bx0 = fmin(bx0, q.x);
                by0 = fmin(by0, q.y);
                bx1 = fmax(bx1, q.x);
                by1 = fmax(by1, q.y);
            }
            const float fb[4] = {down(bx0), down(by0), up(bx1), up(by1)};
            const float fx = (float)p.first, fy = (float)p.second;
            if (fx >= fb[0] && fy >= fb[1] && fx <= fb[2] && fy <= fb[3]) {
                std::vector<float> rv;
                for (const auto& q : v) {
                    rv.push_back((float)(q.x - (double)fb[0]));
                    rv.push_back((float)(q.y - (double)fb[1]));
                }
                const ringwalk::F32Frame fr = ringwalk::f32_frame(fb[0], fb[1], fb[2], fb[3], p.first, p.second);
                const int r32 = ringwalk::ring_interior_f32(rv.data(), (uint32_t)m + 1, fr);
                f32_cases++;
                f32_random += pi < 24;
                if (r32 == 2) {
                    f32_undecided++;
                    f32_random_undecided += pi < 24;
                } else {
                    bad += (r32 == 1) != want;
                }
            }
            cases++;
            bad += (ex != want) + (bf != want);
        }
    }
    printf("%ld %ld %ld %ld %ld %ld\n", cases, bad, f32_cases, f32_undecided, f32_random, f32_random_undecided);
    return 0;
}
