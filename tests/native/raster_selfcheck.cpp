// Test-only: builds the ray-parity rasters of mosaic_amd/csrc/raster.h on the host for a set of
// rings and compares raster::cell_contains with the full-ring JTS locate (pip_device.h
// locate_in_ring, itself pinned against the oracle) on uniform and adversarial points: vertices,
// points on segments, points 1-3 ulp off segments and vertices, points on and next to the raster
// cell lines, points level with vertices.
// Input file: uint32 n_rings, then per ring uint32 n and n (x, y) doubles (closed ring).
// Usage: raster_selfcheck <rings.bin> <dims> <points_per_ring> <seed>
//   -> prints "mismatches points uniform_points uniform_pure mixed_records"
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

#include "../../mosaic_amd/csrc/raster.h"

using namespace mosaic;

int main(int argc, char** argv) {
    if (argc < 5) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    int dims = atoi(argv[2]);
    long per = atol(argv[3]);
    std::mt19937_64 rng(atoi(argv[4]));
    std::uniform_real_distribution<double> u(0.0, 1.0);
    uint32_t nr = 0;
    if (fread(&nr, 4, 1, f) != 1) return 2;
    long bad = 0, total = 0, uni = 0, uni_pure = 0, mixed_records = 0;
    for (uint32_t r = 0; r < nr; r++) {
        uint32_t n = 0;
        if (fread(&n, 4, 1, f) != 1) return 2;
        std::vector<pip::Vec2> v(n);
        if (fread(v.data(), 16, n, f) != n) return 2;
        raster::Builder b;
        raster::ChipHdr h;
        h.box = pip::Box{INFINITY, INFINITY, -INFINITY, -INFINITY};
        for (auto& p : v) {
            h.box.minx = fmin(h.box.minx, p.x);
            h.box.miny = fmin(h.box.miny, p.y);
            h.box.maxx = fmax(h.box.maxx, p.x);
            h.box.maxy = fmax(h.box.maxy, p.y);
        }
        b.add_ring(h, v.data(), n, dims);
        if (h.cell_base == raster::kNoRaster) continue;
        const double W = h.box.maxx - h.box.minx, H = h.box.maxy - h.box.miny;
        auto check = [&](double x, double y, bool uniform) {
            if (pip::box_excludes(h.box, x, y)) return;
            const raster::CellRec& rec = b.cells[raster::cell_index(h, x, y)];
            bool got = raster::cell_contains(rec, b.edges.data(), x, y);
            bool want = pip::locate_in_ring(v.data(), n, x, y) == pip::LOC_INTERIOR;
            total++;
            if (got != want) {
                if (bad < 5)
                    fprintf(stderr, "ring %u point (%.17g, %.17g): raster %d ring %d (m=%u)\n", r, x, y, got, want,
                            rec.m);
                bad++;
            }
            if (uniform) {
                uni++;
                if (rec.m == 0) uni_pure++;
                mixed_records += rec.m;
            }
        };
        auto nudge = [&](double a, int k) {
            for (int i = 0; i < abs(k); i++) a = nextafter(a, k > 0 ? INFINITY : -INFINITY);
            return a;
        };
        for (long i = 0; i < per; i++) {
            int mode = (int)(i % 8);
            double x, y;
            if (mode < 3) {
                check(h.box.minx + W * u(rng), h.box.miny + H * u(rng), true);
                continue;
            }
            uint32_t k = 1 + (uint32_t)(u(rng) * (n - 1));
            if (k >= n) k = n - 1;
            const pip::Vec2 p1 = v[k], p2 = v[k - 1];
            int dx = (int)(u(rng) * 7) - 3, dy = (int)(u(rng) * 7) - 3;
            if (mode == 3) {  // vertex, exactly or a few ulp off
                x = p1.x;
                y = p1.y;
                check(x, y, false);
                check(nudge(x, dx), nudge(y, dy), false);
            } else if (mode == 4) {  // on / next to a segment
                double t = u(rng);
                x = p1.x + t * (p2.x - p1.x);
                y = p1.y + t * (p2.y - p1.y);
                check(x, y, false);
                check(nudge(x, dx), nudge(y, dy), false);
            } else if (mode == 5) {  // on / next to a raster cell line
                int c = (int)(u(rng) * (h.cols + 1)), rr = (int)(u(rng) * (h.rows + 1));
                x = h.box.minx + W * c / (h.cols ? h.cols : 1);
                y = h.box.miny + H * u(rng);
                check(nudge(x, dx), y, false);
                x = h.box.minx + W * u(rng);
                y = h.box.miny + H * rr / (h.rows ? h.rows : 1);
                check(x, nudge(y, dy), false);
            } else if (mode == 6) {  // level with a vertex (the ray passes through it)
                check(h.box.minx + W * u(rng), p1.y, false);
                check(h.box.minx + W * u(rng), nudge(p1.y, dy), false);
            } else {  // level with a vertex, just left of it
                check(nudge(p1.x, -1 - (int)(u(rng) * 3)), p1.y, false);
                check(p1.x, h.box.miny + H * u(rng), false);
            }
        }
    }
    fclose(f);
    printf("%ld %ld %ld %ld %ld\n", bad, total, uni, uni_pure, mixed_records);
    return 0;
}
