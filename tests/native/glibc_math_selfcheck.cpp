// Test-only: mosaic_amd/csrc/glibc_math.h compiled for the host must equal this image's libm
// (glibc 2.35: generic sincos, FMA-build tan / acos / atan2 selected by ifunc) bit for bit.
// Usage: glibc_math_selfcheck <n_per_family> <seed>
//   prints "<function> <checked> <mismatches>" lines; exit status 1 on any mismatch.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>

#include "../../mosaic_amd/csrc/glibc_math.h"

namespace g = mosaic::glibc;

static uint64_t bits_of(double v) {
    uint64_t b;
    memcpy(&b, &v, 8);
    return b;
}
// NaN results compare equal regardless of payload
static bool same(double a, double b) { return (isnan(a) && isnan(b)) || bits_of(a) == bits_of(b); }

struct Tally {
    const char* name;
    long n = 0, bad = 0;
    void check(bool ok, double a, double b, double got, double want) {
        n++;
        if (!ok) {
            if (bad < 5)
                fprintf(stderr, "%s(%a, %a): got %a want %a\n", name, a, b, got, want);
            bad++;
        }
    }
};

int main(int argc, char** argv) {
    long n = argc > 1 ? atol(argv[1]) : 1000000;
    uint64_t seed = argc > 2 ? strtoull(argv[2], 0, 10) : 1;
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> u01(0.0, 1.0);
    auto logu = [&](double lo, double hi) { return exp(log(lo) + (log(hi) - log(lo)) * u01(rng)); };
    auto sgn = [&]() { return (rng() & 1) ? 1.0 : -1.0; };
    auto rbits = [&]() {  // random finite double
        for (;;) {
            uint64_t b = rng();
            double v;
            memcpy(&v, &b, 8);
            if (isfinite(v)) return v;
        }
    };

    Tally ts{"sin"}, tc{"cos"}, tt{"tan"}, ta{"acos"}, t2{"atan2"}, tat{"atan"}, tas{"asin"};
    const double thresholds[] = {0.126, 0.855469, 2.426265, 105414350.0, 0x1p-27, 0x1p-26};
    for (long i = 0; i < n; i++) {
        // ---- sincos ----
        double x;
        switch (i % 8) {
            case 0: x = (u01(rng) - 0.5) * 2.0 * M_PI; break;               // H3 lat / lon / theta range
            case 1: x = (u01(rng) - 0.5) * 20.0; break;
            case 2: x = sgn() * logu(1e-12, 1e9); break;
            case 3: x = sgn() * logu(1e8, 1e300); break;                     // __branred
            case 4: x = (double)((long)(u01(rng) * 200) - 100) * (M_PI / 2) + (u01(rng) - 0.5) * 1e-6; break;
            case 5: x = sgn() * thresholds[rng() % 6] * (1.0 + (u01(rng) - 0.5) * 1e-9); break;
            case 6: x = rbits(); break;
            default: x = sgn() * (u01(rng) * 0.126); break;
        }
        double s0, c0, s1, c1;
        ::sincos(x, &s0, &c0);
        g::sincos(x, &s1, &c1);
        ts.check(same(s0, s1), x, 0, s1, s0);
        tc.check(same(c0, c1), x, 0, c1, c0);

        // ---- tan, |x| <= 0.787 ----
        double tx;
        switch (i % 4) {
            case 0: tx = u01(rng) * 0.6525; break;  // H3: r in [0, 0.6524]
            case 1: tx = sgn() * logu(1e-12, 0.787); break;
            case 2: tx = sgn() * 0.0608 * (1.0 + (u01(rng) - 0.5) * 1e-6); break;
            default: tx = sgn() * u01(rng) * 0.787; break;
        }
        if (fabs(tx) <= 0x1.92f1ap-1) {
            double w0 = ::tan(tx), w1 = g::tan(tx);
            tt.check(same(w0, w1), tx, 0, w1, w0);
        }

        // ---- acos ----
        double ax;
        switch (i % 6) {
            case 0: ax = 1.0 - u01(rng) * 0.2054; break;                   // H3: 1 - sqd / 2
            case 1: ax = (u01(rng) - 0.5) * 2.0; break;
            case 2: ax = sgn() * (1.0 - logu(1e-17, 0.04)); break;         // the 1/sqrt branch
            case 3: ax = sgn() * logu(1e-20, 0.5); break;
            case 4: ax = sgn() * (0.5 + u01(rng) * 0.5); break;
            default: ax = (rng() % 64 == 0) ? rbits() : sgn() * u01(rng); break;
        }
        double a0 = ::acos(ax), a1 = g::acos(ax);
        ta.check(same(a0, a1), ax, 0, a1, a0);

        // ---- atan2 ----
        double y, xx;
        switch (i % 6) {
            case 0: y = (u01(rng) - 0.5) * 2.0; xx = (u01(rng) - 0.5) * 2.0; break;  // H3 azimuth range
            case 1: y = sgn() * logu(1e-300, 1e300); xx = sgn() * logu(1e-300, 1e300); break;
            case 2: y = sgn() * logu(1e-3, 1.0); xx = y * (1.0 + (u01(rng) - 0.5) * 1e-3); break;  // |y| ~ |x|
            case 3: y = sgn() * u01(rng) * 0.07; xx = sgn(); break;                                  // small u
            case 4: {
                const double sp[] = {0.0, -0.0, INFINITY, -INFINITY, 1.0, -1.0, 1e-310, -1e-310};
                y = (rng() & 1) ? sp[rng() % 8] : (u01(rng) - 0.5);
                xx = (rng() & 1) ? sp[rng() % 8] : (u01(rng) - 0.5);
                break;
            }
            default: y = rbits(); xx = rbits(); break;
        }
        double b0 = ::atan2(y, xx), b1 = g::atan2(y, xx);
        t2.check(same(b0, b1), y, xx, b1, b0);

        // ---- atan (h3ToGeo / h3ToGeoBoundary: atan of the gnomonic radius) ----
        double at;
        switch (i % 7) {
            case 0: at = u01(rng) * 0.76; break;  // H3: r RES0_U_GNOMONIC over a face
            case 1: at = sgn() * logu(1e-300, 1e300); break;
            case 2: at = sgn() * u01(rng); break;
            case 3: at = sgn() * (1.0 + u01(rng) * 15.0); break;
            case 4: {
                const double th[] = {0x1.bb67ap-27, 0.0625, 1.0, 16.0, 0x1.49ff2p+53, 0x1p-1022};
                at = sgn() * th[rng() % 6] * (1.0 + (u01(rng) - 0.5) * 1e-12);
                break;
            }
            case 5: {
                const double sp[] = {0.0, -0.0, INFINITY, -INFINITY, NAN, 5e-324};
                at = sp[rng() % 6];
                break;
            }
            default: at = rbits(); break;
        }
        double q0 = ::atan(at), q1 = g::atan(at);
        tat.check(same(q0, q1), at, 0, q1, q0);

        // ---- asin (_geoAzDistanceRads: asin of the destination's sin(lat)) ----
        double as;
        switch (i % 6) {
            case 0: as = (u01(rng) - 0.5) * 2.0; break;
            case 1: as = sgn() * (1.0 - logu(1e-17, 0.04)); break;  // the sqrt branch
            case 2: as = sgn() * logu(1e-300, 0.5); break;
            case 3: {
                const double th[] = {0x1p-26, 0.125, 0.25, 0.5, 0.75, 0.921875, 0.953125, 0.96875, 1.0};
                as = sgn() * th[rng() % 9] * (1.0 + (u01(rng) - 0.5) * 1e-12);
                break;
            }
            case 4: {
                const double sp[] = {0.0, -0.0, 1.0, -1.0, INFINITY, NAN, 1.5, 5e-324};
                as = sp[rng() % 8];
                break;
            }
            default: as = (rng() % 16 == 0) ? rbits() : sgn() * u01(rng); break;
        }
        double e0 = ::asin(as), e1 = g::asin(as);
        tas.check(same(e0, e1), as, 0, e1, e0);
    }
    long bad = 0;
    for (Tally* t : {&ts, &tc, &tt, &ta, &t2, &tat, &tas}) {
        printf("%s %ld %ld\n", t->name, t->n, t->bad);
        bad += t->bad;
    }
    return bad ? 1 : 0;
}
