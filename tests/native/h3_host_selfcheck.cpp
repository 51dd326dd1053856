// Test-only: compiles the device H3 code (mosaic_amd/csrc/h3_device.h) for the host and compares
// h3_exact / h3_fast against the C oracle (glibc libm on both sides, so h3_exact must match
// bit-for-bit; h3_fast must match whenever it does not report "ambiguous").
// Usage: h3_host_selfcheck <n_points> <seed>   -> prints "mismatch_exact mismatch_fast ambiguous"
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <stdint.h>
#include <random>
#include "../../mosaic_amd/csrc/h3_device.h"
extern "C" {
int64_t oracle_h3_geo_to_h3(double lat_rad, double lng_rad, int res);
double oracle_to_radians(double deg, int jdk);
}
int main(int argc, char** argv) {
    long n = argc > 1 ? atol(argv[1]) : 100000;
    int seed = argc > 2 ? atoi(argv[2]) : 1;
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> u(0.0, 1.0);
    long bad_exact = 0, bad_fast = 0, amb = 0;
    for (long i = 0; i < n; i++) {
        double lon, lat;
        int mode = i % 4;
        if (mode == 0) {  // global uniform on the sphere, longitudes also beyond +-180 (valid input)
            lon = (i & 8) ? -200.0 + 400.0 * u(rng) : -180.0 + 360.0 * u(rng);
            lat = asin(2.0 * u(rng) - 1.0) * 57.29577951308232;
        } else if (mode == 1) {  // NYC bbox
            lon = -74.25559136315209 + 0.5556 * u(rng);
            lat = 40.496115395170364 + 0.4194 * u(rng);
        } else if (mode == 2) {  // rounded to 1e-6 like taxi GPS
            lon = round((-74.3 + 0.6 * u(rng)) * 1e6) / 1e6;
            lat = round((40.4 + 0.6 * u(rng)) * 1e6) / 1e6;
        } else {  // adversarial: points within ~1e-9 hex units of cell edges / vertices / face centres
            int f = (int)(u(rng) * 20) % 20;
            int r = (int)((i / 4) % 16);
            const double* b = mosaic::h3::kH3FastBasis[f];
            const double* ei = b + ((r & 1) ? 9 : 3);
            const double* ep = b + ((r & 1) ? 12 : 6);
            double S = mosaic::h3::kH3FastScale[r];
            double span = 0.6 * S;  // stay within the face
            int ci = (int)((u(rng) - 0.5) * span), cj = (int)((u(rng) - 0.5) * span);
            double cx = ci - 0.5 * cj, cy = cj * 0.8660254037844386;
            double kind = u(rng);
            double hx, hy;
            if (kind < 0.4) {  // edge between (ci,cj) and a neighbour
                double ang = (int)(u(rng) * 6) * 1.0471975511965976;
                double t = u(rng) - 0.5;
                hx = cx + 0.5 * cos(ang) - t * 0.57735 * sin(ang);
                hy = cy + 0.5 * sin(ang) + t * 0.57735 * cos(ang);
            } else if (kind < 0.8) {  // vertex
                double ang = (int)(u(rng) * 6) * 1.0471975511965976 + 0.5235987755982988;
                hx = cx + 0.5773502691896258 * cos(ang);
                hy = cy + 0.5773502691896258 * sin(ang);
            } else if (kind < 0.9) {  // near the face centre
                hx = (u(rng) - 0.5) * 1e-6;
                hy = (u(rng) - 0.5) * 1e-6;
            } else {  // on the axes (fold lines)
                hx = (u(rng) < 0.5) ? 0.0 : cx;
                hy = (hx == 0.0) ? cy : 0.0;
            }
            double eps = (u(rng) - 0.5) * 2e-9 * (1.0 + fabs(hx) + fabs(hy)) * (u(rng) < 0.5 ? 1.0 : 0.0);
            hx += eps;
            hy -= eps;
            double px = b[0] + (hx * ei[0] + hy * ep[0]) / S;
            double py = b[1] + (hx * ei[1] + hy * ep[1]) / S;
            double pz = b[2] + (hx * ei[2] + hy * ep[2]) / S;
            double nn = sqrt(px * px + py * py + pz * pz);
            lat = asin(pz / nn) * 57.29577951308232;
            lon = atan2(py, px) * 57.29577951308232;
        }
        int res = (int)(i % 16);
        if (mode == 3) {
            // same resolution as used for construction is unknown here; sweep all
            res = (int)((i / 4) % 16);
        }
        int jdk = (i & 1) ? 8 : 11;
        double la = oracle_to_radians(lat, jdk), lo = oracle_to_radians(lon, jdk);
        int64_t want = oracle_h3_geo_to_h3(la, lo, res);
        int64_t ex = (int64_t)mosaic::h3::h3_exact(la, lo, res);
        if (ex != want) {
            if (bad_exact < 5) fprintf(stderr, "exact mismatch lat %.17g lon %.17g res %d: %llx vs %llx\n", lat, lon, res,
                                       (unsigned long long)ex, (unsigned long long)want);
            bad_exact++;
        }
        bool a = false;
        int64_t fa = (int64_t)mosaic::h3::h3_fast(lat, lon, res, &a);
        {
            // the two-point form (k_cell_h3): this point beside the previous one, both as h3_fast
            static double plat = 40.7, plon = -74.0;
            const double la2[2] = {plat, lat}, lo2[2] = {plon, lon};
            uint64_t c2[2];
            bool a2[2], r2[2];
            if ((i >> 6) & 1)
                mosaic::h3::h3_fast2(la2, lo2, res, c2, a2, r2);
            else  // the four-level digit form (k_cell_h3's)
                mosaic::h3::h3_fast2_quad(la2, lo2, res, c2, a2, r2);
            for (int k = 0; k < 2; k++)
                if (r2[k]) c2[k] = mosaic::h3::h3_fast(la2[k], lo2[k], res, &a2[k]);  // (the caller's rare path)
            bool ap = false;
            const uint64_t cp = mosaic::h3::h3_fast(plat, plon, res, &ap);
            if (c2[1] != (uint64_t)fa || a2[1] != a || c2[0] != cp || a2[0] != ap) {
                if (bad_fast < 5) fprintf(stderr, "fast2 mismatch lat %.17g lon %.17g res %d\n", lat, lon, res);
                bad_fast++;
            }
            plat = lat;
            plon = lon;
        }
        if (a) {
            amb++;
        } else if (fa != want) {
            if (bad_fast < 5) fprintf(stderr, "fast mismatch lat %.17g lon %.17g res %d: %llx vs %llx\n", lat, lon, res,
                                      (unsigned long long)fa, (unsigned long long)want);
            bad_fast++;
        }
    }
    printf("%ld %ld %ld\n", bad_exact, bad_fast, amb);
    return 0;
}
