// CPU-only check of the tile directory's closed-form bounds (tiles.h TileCurv, rect_tol, poly_tol):
// on random tiles at several resolutions and latitudes, finite-difference derivatives of the
// lon / lat -> face-plane map F must stay under jac / kax / kdir, and every sampled point of a
// random sub-rectangle must lie within rect_tol of the quadrilateral of its corner images.
// Prints: tiles checked, violations, and the largest observed / bound ratios (jac, kax, kdir, rect).
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>

#include "../../mosaic_amd/csrc/geom_build.h"
#include "../../mosaic_amd/csrc/tiles_build.cpp"

using namespace mosaic;

struct V2 {
    double x, y;
};

static V2 image(int face, int res, double lon, double lat) {
    double px, py, pz, vx, vy, b;
    h3::fast_unit(lat, lon, &px, &py, &pz);
    h3::fast_plane(px, py, pz, face, res, &vx, &vy, &b);
    return V2{vx, vy};
}

// distance from p to the quadrilateral q[4] (0 inside; q counter-clockwise or clockwise)
static double quad_dist(const V2* q, V2 p) {
    double sgn = 0.0, dmin = INFINITY;
    bool inside = true;
    for (int k = 0; k < 4; k++) {
        const V2 a = q[k], b = q[(k + 1) & 3];
        const double cr = (b.x - a.x) * (p.y - a.y) - (b.y - a.y) * (p.x - a.x);
        if (cr != 0.0) {
            if (sgn == 0.0) sgn = cr > 0 ? 1.0 : -1.0;
            else if (cr * sgn < 0) inside = false;
        }
        const double ex = b.x - a.x, ey = b.y - a.y, l2 = ex * ex + ey * ey;
        double t = l2 > 0 ? ((p.x - a.x) * ex + (p.y - a.y) * ey) / l2 : 0.0;
        t = std::min(1.0, std::max(0.0, t));
        dmin = std::min(dmin, hypot(p.x - a.x - t * ex, p.y - a.y - t * ey));
    }
    return inside ? 0.0 : dmin;
}

int main(int argc, char** argv) {
    const int n_tiles = argc > 1 ? atoi(argv[1]) : 2000;
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    const int resl[] = {3, 6, 9, 11, 13, 15};
    int checked = 0, bad = 0;
    double r_jac = 0, r_ax = 0, r_dir = 0, r_rect = 0;
    for (int it = 0; it < n_tiles; it++) {
        const int res = resl[it % 6];
        const double lat = -75.0 + 150.0 * U(rng), lon = -180.0 + 360.0 * U(rng);
        // tile size as the builder picks it (~4 hex units, at most 0.25 degrees)
        tiles::Builder::Samples s0;
        if (!tiles::Builder::sample(lon, lat, 1e-4, 1e-4, res, &s0)) continue;
        const double sc = h3::kH3FastScale[res] * 3.141592653589793 / 180.0;  // ~ hex units per degree
        const double tw = std::min(0.25, 4.0 / sc / std::max(0.2, cos(lat * 3.141592653589793 / 180.0)));
        const double th = std::min(0.25, 4.0 / sc);
        tiles::Builder::Samples s;
        if (!tiles::Builder::sample(lon, lat, tw, th, res, &s)) continue;
        tiles::TileCurv cv;
        if (!tiles::Builder::tile_curv(s.face, lon, lat, tw, th, res, &cv)) continue;
        checked++;
        const int f = s.face;
        for (int q = 0; q < 40; q++) {
            const double x = lon + tw * (0.1 + 0.8 * U(rng)), y = lat + th * (0.1 + 0.8 * U(rng));
            const double h = 0.05 * std::min(tw, th);
            const double ang = 6.283185307179586 * U(rng);
            const double dirs[3][2] = {{1, 0}, {0, 1}, {cos(ang), sin(ang)}};
            for (int d = 0; d < 3; d++) {
                const double dx = dirs[d][0] * h, dy = dirs[d][1] * h;
                const V2 m = image(f, res, x - dx, y - dy), c = image(f, res, x, y), p = image(f, res, x + dx, y + dy);
                const double d1 = hypot(p.x - m.x, p.y - m.y) / (2 * h);
                const double d2 = hypot(p.x - 2 * c.x + m.x, p.y - 2 * c.y + m.y) / (h * h);
                r_jac = std::max(r_jac, d1 / cv.jac);
                if (d1 > cv.jac) bad++;
                const double k2 = d < 2 ? cv.kax : cv.kdir;
                if (d < 2) r_ax = std::max(r_ax, d2 / cv.kax);
                else r_dir = std::max(r_dir, d2 / cv.kdir);
                if (d2 > k2) bad++;
            }
        }
        // a random sub-rectangle: sampled images within rect_tol of its corner quadrilateral
        const double w = tw * (0.02 + 0.98 * U(rng)), hh = th * (0.02 + 0.98 * U(rng));
        const double x0 = lon + (tw - w) * U(rng), y0 = lat + (th - hh) * U(rng);
        const V2 q[4] = {image(f, res, x0, y0), image(f, res, x0 + w, y0), image(f, res, x0 + w, y0 + hh),
                         image(f, res, x0, y0 + hh)};
        const double tol = tiles::rect_tol(cv, w, hh, 0.0) - 1e-7;
        for (int k = 0; k < 64; k++) {
            const double u = (k < 16) ? (k % 4) / 3.0 : U(rng), v = (k < 16) ? (k / 4) / 3.0 : U(rng);
            const double dd = quad_dist(q, image(f, res, x0 + u * w, y0 + v * hh));
            r_rect = std::max(r_rect, dd / tol);
            if (dd > tol + 1e-7) bad++;
        }
    }
    printf("%d %d %.6g %.6g %.6g %.6g\n", checked, bad, r_jac, r_ax, r_dir, r_rect);
    return 0;
}
