// glibc 2.35 x86-64 libm, restated bit for bit, as the reference's H3 C calls it.
//
// Why: the reference indexes points with H3 C v3.7 (h3-java 3.7.0 -> geoToH3, called at
// H3IndexSystem.scala:140-142), linked against the host glibc.  On points within an ulp of a cell
// boundary the cell depends on the last bit of libm, and glibc's results are not correctly
// rounded, so a correctly rounded (or OCML) libm disagrees with the reference on rare inputs.
// H3's _geoToHex2d / _geoToVec3d / _geoAzimuthRads, compiled by gcc -O2 on x86-64, reach libm as:
//   * sincos  -- gcc fuses every sin(v) / cos(v) pair of one argument into one sincos(v) call
//                (verified in the oracle's object code: five sincos calls, no sin / cos);
//                glibc 2.35 has a single generic sincos (s_sincos.c, SSE2, no FMA contraction);
//   * tan, acos, atan2 -- glibc's ifunc picks the FMA builds (s_tan-fma.c, e_asin-fma.c,
//                e_atan2-fma.c, i.e. the same sources compiled with -mfma -mavx2, where gcc
//                contracts a*b+c into one fused multiply-add) on every AVX2+FMA host.
// Each function below restates the glibc 2.35 source *and* the contractions gcc made in the
// shipped object (read from /lib/x86_64-linux-gnu/libm-2.35.a): fma() exactly where the shipped
// code has a vfmadd / vfmsub / vfnmadd, plain IEEE operations everywhere else.  This file must be
// compiled with -ffp-contract=off (Makefile), on the device and in host self-checks alike.
// Tables (glibc_math_tables.h) are glibc's own data, extracted by tools/glibc_tables.py.
//
// Domains: sincos and atan2 are restated for every input (incl. huge arguments via __branred,
// zeros, infinities, NaN); acos for every input; tan for |x| <= 0.787 (glibc's cases I-III),
// which covers H3's only call, tan(r) with r = the angular distance from the point to its face
// centre <= 0.6524 (the icosahedron's face circumradius); tan returns NaN beyond that.
//
// Verified bit for bit against this image's libm on ~10^8 arguments per function
// (tests/native/glibc_math_selfcheck.cpp, tests/test_native_selfcheck.py) and on the GPU
// (tests/test_gpu_parity.py::test_glibc_math_device).
#pragma once
#include <math.h>
#include <stdint.h>

#if !defined(MOSAIC_HD)
#if defined(__HIPCC__)
#define MOSAIC_HD __host__ __device__ inline
#else
#define MOSAIC_HD inline
#endif
#endif

namespace mosaic {
namespace glibc {

#if defined(__HIPCC__)
#define GLIBC_TABLE static __device__ const
#else
#define GLIBC_TABLE static const
#endif
#include "glibc_math_tables.h"
#undef GLIBC_TABLE

MOSAIC_HD uint64_t bits(double x) { return __builtin_bit_cast(uint64_t, x); }
MOSAIC_HD double from_bits(uint64_t b) { return __builtin_bit_cast(double, b); }
MOSAIC_HD int32_t hi32(double x) { return (int32_t)(bits(x) >> 32); }
MOSAIC_HD uint32_t lo32(double x) { return (uint32_t)bits(x); }

// ---- s_sin.c / usncs.h constants (shared by sincos and branred's callers) ----
static constexpr double kSn3 = -0x1.5555555555515p-3, kSn5 = 0x1.11110e829872fp-7;
static constexpr double kCs2 = 0.5, kCs4 = -0x1.5555555555535p-5, kCs6 = 0x1.6c16bedd9e239p-10;
static constexpr double kS1 = -0x1.5555555555555p-3, kS2 = 0x1.1111111110ecep-7, kS3 = -0x1.a01a019db08b8p-13,
                        kS4 = 0x1.71de27b9a7ed9p-19, kS5 = -0x1.addffc2fcdf59p-26;
static constexpr double kBig = 0x1.8p+45;  // 52776558133248: |x| + big rounds |x| to a multiple of 1/128
static constexpr double kHp0 = 0x1.921fb54442d18p+0, kHp1 = 0x1.1a62633145c07p-54;  // pi/2 = hp0 + hp1
static constexpr double kHpInv = 0x1.45f306dc9c883p-1, kToInt = 0x1.8p+52;
static constexpr double kMp1 = 0x1.921fb58p+0, kMp2 = -0x1.dde973cp-27;
static constexpr double kPp3 = -0x1.cb3b398p-55, kPp4 = -0x1.d747f23e32ed7p-83;

// ---- sincos: s_sincos.c with the inlined do_sin / do_cos / reduce_sincos of s_sin.c (generic
// build, no contraction) ----

// TAYLOR_SIN(xx, a, da)
MOSAIC_HD double taylor_sin(double xx, double a, double da) {
    double poly = ((((kS5 * xx + kS4) * xx + kS3) * xx + kS2) * xx) + kS1;
    double t = ((poly * a - 0.5 * da) * xx + da);
    return a + t;
}

// SINCOS_TABLE_LOOKUP: u = big + |x|, k = low word of u << 2
MOSAIC_HD void sincos_lookup(double u, double* sn, double* ssn, double* cs, double* ccs) {
    int k = (int)(lo32(u) << 2);
    *sn = kSinCosTab[k];
    *ssn = kSinCosTab[k + 1];
    *cs = kSinCosTab[k + 2];
    *ccs = kSinCosTab[k + 3];
}

MOSAIC_HD double do_sin(double x, double dx) {
    double xold = x;
    if (fabs(x) < 0.126) return taylor_sin(x * x, x, dx);
    if (x <= 0) dx = -dx;
    double u = kBig + fabs(x);
    x = fabs(x) - (u - kBig);
    double xx = x * x;
    double s = x + (dx + x * xx * (kSn3 + xx * kSn5));
    double c = x * dx + xx * (kCs2 + xx * (kCs4 + xx * kCs6));
    double sn, ssn, cs, ccs;
    sincos_lookup(u, &sn, &ssn, &cs, &ccs);
    double cor = (ssn + s * ccs - sn * c) + cs * s;
    return copysign(sn + cor, xold);
}

MOSAIC_HD double do_cos(double x, double dx) {
    if (x < 0) dx = -dx;
    double u = kBig + fabs(x);
    x = fabs(x) - (u - kBig) + dx;
    double xx = x * x;
    double s = x + x * xx * (kSn3 + xx * kSn5);
    double c = xx * (kCs2 + xx * (kCs4 + xx * kCs6));
    double sn, ssn, cs, ccs;
    sincos_lookup(u, &sn, &ssn, &cs, &ccs);
    double cor = (ccs - s * ssn - cs * c) - sn * s;
    return cs + cor;
}

// reduce_sincos: x - n pi/2 as a + da, |x| < 105414350
MOSAIC_HD int reduce_sincos(double x, double* a, double* da) {
    double t = (x * kHpInv + kToInt);
    double xn = t - kToInt;
    int n = (int)(lo32(t) & 3);
    double y = (x - xn * kMp1) - xn * kMp2;
    double t1 = xn * kPp3;
    double t2 = y - t1;
    double db = (y - t2) - t1;
    t1 = xn * kPp4;
    double b = t2 - t1;
    db += (t2 - b) - t1;
    *a = b;
    *da = db;
    return n;
}

// branred.c __branred: x mod pi/2 for |x| >= 105414350 (Payne-Hanek with 24-bit chunks of 2/pi)
MOSAIC_HD int branred(double x, double* a, double* aa) {
    const double tm600 = 0x1p-600, split = 0x1.0000002p+27, tm24 = 0x1p-24;
    const double big = 0x1.8p+52, big1 = 0x1.8p+54;
    const double hp0 = kHp0, hp1 = kHp1, mp1 = 0x1.921fb58p+0, mp2 = -0x1.dde974p-27;
    double r[6], s, t, sum, b, bb, sum1, sum2, b1, bb1, b2, bb2, x1, x2, t1, t2;
    x *= tm600;
    t = x * split;
    x1 = t - (t - x);
    x2 = x - x1;
    double parts[2] = {x1, x2};
    double bo[2], bbo[2], so[2];
    for (int h = 0; h < 2; h++) {
        double xp = parts[h];
        sum = 0;
        int k = (int)((bits(xp) >> 52) & 2047);
        k = (k - 450) / 24;
        if (k < 0) k = 0;
        double gor = from_bits((uint64_t)(0x63f00000u - (uint32_t)((k * 24) << 20)) << 32);
        for (int i = 0; i < 6; i++) {
            r[i] = xp * kToverp[k + i] * gor;
            gor *= tm24;
        }
        for (int i = 0; i < 3; i++) {
            s = (r[i] + big) - big;
            sum += s;
            r[i] -= s;
        }
        t = 0;
        for (int i = 0; i < 6; i++) t += r[5 - i];
        bb = (((((r[0] - t) + r[1]) + r[2]) + r[3]) + r[4]) + r[5];
        s = (t + big) - big;
        sum += s;
        t -= s;
        b = t + bb;
        bb = (t - b) + bb;
        s = (sum + big1) - big1;
        sum -= s;
        bo[h] = b;
        bbo[h] = bb;
        so[h] = sum;
    }
    b1 = bo[0];
    bb1 = bbo[0];
    sum1 = so[0];
    b2 = bo[1];
    bb2 = bbo[1];
    sum2 = so[1];
    sum = sum1 + sum2;
    b = b1 + b2;
    bb = (fabs(b1) > fabs(b2)) ? (b1 - b) + b2 : (b2 - b) + b1;
    if (b > 0.5) {
        b -= 1.0;
        sum += 1.0;
    } else if (b < -0.5) {
        b += 1.0;
        sum -= 1.0;
    }
    s = b + (bb + bb1 + bb2);
    t = ((b - s) + bb) + (bb1 + bb2);
    b = s * split;
    t1 = b - (b - s);
    t2 = s - t1;
    b = s * hp0;
    bb = (((t1 * mp1 - b) + t1 * mp2) + t2 * mp1) + (t2 * mp2 + s * hp1 + t * hp0);
    s = b + bb;
    t = (b - s) + bb;
    *a = s;
    *aa = t;
    return ((int)sum) & 3;
}

MOSAIC_HD void sincos(double x, double* sinx, double* cosx) {
    int32_t k = hi32(x) & 0x7fffffff;
    if (k < 0x400368fd) {
        if (k < 0x3e400000) {
            *sinx = x;
            *cosx = 1.0;
            return;
        }
        if (k < 0x3feb6000) {
            *sinx = do_sin(x, 0);
            *cosx = do_cos(x, 0);
            return;
        }
        double y = kHp0 - fabs(x);
        double a = y + kHp1;
        double da = (y - a) + kHp1;
        *sinx = copysign(do_cos(a, da), x);
        *cosx = do_sin(a, da);
        return;
    }
    if (k < 0x7ff00000) {
        double a, da;
        int n = (k < 0x419921FB) ? reduce_sincos(x, &a, &da) : branred(x, &a, &da);
        if (n == 1 || n == 2) {
            a = -a;
            da = -da;
        }
        double sv = do_sin(a, da), cv = do_cos(a, da);
        if (n & 2) cv = -cv;
        if (n & 1) {
            *sinx = cv;
            *cosx = sv;
        } else {
            *sinx = sv;
            *cosx = cv;
        }
        return;
    }
    *sinx = *cosx = x / x;
}

// ---- tan: s_tan.c (FMA build), cases |x| <= 0.787 ----
MOSAIC_HD double tan(double x) {
    const double g1 = 0x1.b096cp-27, g2 = 0x1.f212dp-5, g3 = 0x1.92f1ap-1;
    const double d3 = 0x1.5555555555555p-2, d5 = 0x1.11111111107c6p-3, d7 = 0x1.ba1ba1cdb8745p-5,
                 d9 = 0x1.664ed49cfc666p-6, d11 = 0x1.2385a3cf2e4eap-7;
    const double e0 = 0x1.5555555554dbdp-2, e1 = 0x1.11112e0a6b45fp-3;
    if ((hi32(x) & 0x7ff00000) == 0x7ff00000) return x - x;
    double w = (x < 0.0) ? -x : x;
    if (w <= g1) return x;  // (I)
    if (w <= g2) {          // (II)
        double x2 = x * x;
        double t2 = fma(fma(fma(fma(d11, x2, d9), x2, d7), x2, d5), x2, d3);
        return fma(x * x2, t2, x);
    }
    if (w <= g3) {  // (III)
        int i = (int)fma(256.0, w, -15.5);
        double z = w - kTanXfg[4 * i];
        double z2 = z * z;
        double s = (x < 0.0) ? -1.0 : 1.0;
        double pz = fma(z * z2, fma(z2, e1, e0), z);
        double fi = kTanXfg[4 * i + 1], gi = kTanXfg[4 * i + 2];
        double t2 = pz * (gi + fi) / (gi - pz);
        double y = fi + t2;
        return s * y;
    }
    return __builtin_nan("");  // outside the restated domain (see header)
}

// ---- acos: e_asin.c __ieee754_acos (FMA build) ----
MOSAIC_HD double acos(double x) {
    const double hp0 = kHp0, hp1 = kHp1;
    const double d1 = 0x1.55555555554f9p-3, d2 = 0x1.333333336127dp-4, d3 = 0x1.6db6dae42c0e4p-5,
                 d4 = 0x1.f1c7e04f4ad99p-6, d5 = 0x1.6e442c822d419p-6, d6 = 0x1.292d80f453c72p-6;
    const double rt0 = 0x1.fffffffecc1ddp-1, rt1 = 0x1.fffffff757304p-2, rt2 = 0x1.800496769c91ap-2,
                 rt3 = 0x1.4006318d1dab9p-2;
    const double t27 = 0x1p+27;
    int32_t m = hi32(x);
    int32_t k = m & 0x7fffffff;
    if (k < 0x3c880000) return hp0;
    if (k < 0x3fc00000) {  // |x| < 0.125
        double x2 = x * x;
        double p = fma(fma(fma(fma(fma(d6, x2, d5), x2, d4), x2, d3), x2, d2), x2, d1);
        double r = hp0 - x;
        double cor = ((hp0 - r) - x) + hp1;
        return r + fma(-(x * x2), p, cor);
    }
    if (k < 0x3fef0000) {  // 0.125 <= |x| < 0.96875: per-interval polynomial in |x| - x0
        int n, top;
        if (k < 0x3fd00000) {
            n = 11 * ((k >> 15) & 0x1f);
            top = 6;
        } else if (k < 0x3fe00000) {
            n = 352 + 11 * ((k >> 14) & 0x3f);
            top = 6;
        } else if (k < 0x3fe80000) {
            n = 1056 + 12 * ((k >> 13) & 0x7f);
            top = 7;
        } else if (k < 0x3fed8000) {
            n = 992 + 13 * ((k >> 13) & 0x7f);
            top = 8;
        } else if (k < 0x3fee8000) {
            n = 884 + 14 * ((k >> 13) & 0x7f);
            top = 9;
        } else {
            n = 768 + 15 * ((k >> 13) & 0x7f);
            top = 10;
        }
        const double* T = kAsnCs + n;
        double ax = (m > 0) ? x : -x;
        double xx = ax - T[0];
        double xx2 = xx * xx;
        double p = T[top];
        for (int j = top - 1; j >= 2; j--) p = fma(xx, p, T[j]);
        p = fma(xx2, p, T[top + 1]);
        double t = fma(xx, T[1], p);
        double res0 = T[top + 2];
        if (m > 0) return (hp1 - t) + (hp0 - res0);
        return (t + hp1) + (res0 + hp0);
    }
    if (k < 0x3ff00000) {  // 0.96875 <= |x| < 1: 2 asin(sqrt((1 - |x|) / 2)) from a table 1/sqrt
        double z = ((m > 0) ? (1.0 - x) : (x + 1.0)) * 0.5;
        int64_t zb = (int64_t)bits(z);
        int i0 = (int)((zb >> 46) & 0x7f);
        int e = 0x1ff - (int)(zb >> 53);
        double y = kInRoot[i0] * kPowTwo[e];
        double r = fma(-(y * y), z, 1.0);
        y = fma(fma(fma(rt3, r, rt2), r, rt1), r, rt0) * y;
        double c = z * y;
        double t = fma(-(y * 0.5), c, 1.5);
        double hx = fma(-t27, c, fma(c, t27, c));
        double den = fma(t, c, hx);
        double cc = fma(-hx, hx, z) / den;
        double p = fma(fma(fma(fma(fma(d6, z, d5), z, d4), z, d3), z, d2), z, d1);
        double P = (p * z) * (hx + cc);
        if (m >= 0) {
            double v = (cc + P) + hx;
            return v + v;
        }
        double v = ((hp1 - cc) - P) + (hp0 - hx);
        return v + v;
    }
    if (k == 0x3ff00000 && lo32(x) == 0) return (m > 0) ? 0.0 : 2.0 * hp0;
    if (k > 0x7ff00000 || (k == 0x7ff00000 && lo32(x) != 0)) return x + x;
    double zz = x - x;
    return zz / zz;
}

// ---- atan2: e_atan2.c __ieee754_atan2 (FMA build) ----
MOSAIC_HD double atan2_poly(double z2) {  // odd series d1..d11 of atan for |u| < 1/16
    const double d1 = -0x1.5555555555555p-2, d3 = 0x1.99999999997fdp-3, d5 = -0x1.24924923f7603p-3,
                 d7 = 0x1.c71c6e5129a3bp-4, d9 = -0x1.7458022b13c25p-4, d11 = 0x1.375f08b31cbcep-4;
    return fma(fma(fma(fma(fma(d11, z2, d9), z2, d7), z2, d5), z2, d3), z2, d1);
}
MOSAIC_HD const double* atan2_row(double u) {
    const double two52 = 0x1p+52;
    int i = (int)(fma(u, 256.0, two52) - two52) - 16;
    return kAtan2Cij + 7 * i;
}
MOSAIC_HD double atan2_tpoly(const double* c, double t) {
    return fma(fma(fma(fma(c[6], t, c[5]), t, c[4]), t, c[3]), t, c[2]);
}

MOSAIC_HD double atan2(double y, double x) {
    const double hp0 = kHp0, hp1 = kHp1, pi = 0x1.921fb54442d18p+1, pi_lo = 0x1.1a62633145c07p-53;
    const double pi4 = 0x1.921fb54442d18p-1, pi34 = 0x1.2d97c7f3321d2p+1;
    const double two500 = 0x1p+500, twom500 = 0x1p-500;
    const uint32_t ux = (uint32_t)hi32(x), dx = lo32(x), uy = (uint32_t)hi32(y), dy = lo32(y);
    if ((ux & 0x7ff00000) == 0x7ff00000 && ((ux & 0x000fffff) | dx) != 0) return x + y;
    if ((uy & 0x7ff00000) == 0x7ff00000 && ((uy & 0x000fffff) | dy) != 0) return y + y;
    if (uy == 0 && dy == 0) return ((int32_t)ux < 0) ? pi : 0.0;                    // y = +0
    if (uy == 0x80000000u && dy == 0) return ((int32_t)ux < 0) ? -pi : -0.0;        // y = -0
    if (x == 0.0) return ((int32_t)uy < 0) ? -hp0 : hp0;                           // x = +-0
    if (ux == 0x7ff00000u && dx == 0) {                                            // x = +inf
        if (uy == 0x7ff00000u && dy == 0) return pi4;
        if (uy == 0xfff00000u && dy == 0) return -pi4;
        return ((int32_t)uy < 0) ? -0.0 : 0.0;
    }
    if (ux == 0xfff00000u && dx == 0) {                                            // x = -inf
        if (uy == 0x7ff00000u && dy == 0) return pi34;
        if (uy == 0xfff00000u && dy == 0) return -pi34;
        return ((int32_t)uy < 0) ? -pi : pi;
    }
    if (uy == 0x7ff00000u && dy == 0) return hp0;                                   // y = +inf
    if (uy == 0xfff00000u && dy == 0) return -hp0;                                  // y = -inf

    double ax = (x < 0) ? -x : x;
    double ay = (y < 0) ? -y : y;
    int32_t de = (int32_t)(uy & 0x7ff00000) - (int32_t)(ux & 0x7ff00000);
    if (de > 0x38fffff) return (y <= 0) ? -hp0 : hp0;  // |y/x| > 2^57
    if (de < -0x38fffff) {                              // |y/x| < 2^-57
        if (x > 0) return copysign(ay / ax, y);
        return (y <= 0) ? -pi : pi;
    }
    if (ax < twom500 || ay < twom500) {
        ax *= two500;
        ay *= two500;
    }
    if (ax > two500 || ay > two500) {
        ax *= twom500;
        ay *= twom500;
    }
    double u, du;
    if (ax > ay) {
        u = ay / ax;
        double v = ax * u, vv = fma(ax, u, -v);
        du = ((ay - v) - vv) / ax;
    } else {
        u = ax / ay;
        double v = ay * u, vv = fma(ay, u, -v);
        du = ((ax - v) - vv) / ay;
    }
    double r;
    if (x > 0) {
        if (ax > ay) {  // atan(u)
            if (u < 0.0625) {
                double z2 = u * u;
                r = u + fma(u * z2, atan2_poly(z2), du);
            } else {
                const double* c = atan2_row(u);
                double t = u - c[0];
                double z = du + t;
                double zz = (fabs(t) > fabs(du)) ? (t - z) + du : (du - z) + t;
                double z2 = z * z;
                double p3 = fma(fma(fma(c[6], z, c[5]), z, c[4]), z, c[3]);
                r = fma(z, c[2], fma(zz, c[2], z2 * p3)) + c[1];
            }
        } else {  // pi/2 - atan(u)
            if (u < 0.0625) {
                double z2 = u * u;
                double q = (u * z2) * atan2_poly(z2);
                double t1 = hp0 - u;
                double r1 = (hp0 > fabs(u)) ? ((hp0 - t1) - u) : (hp0 - (u + t1));
                r = (((r1 + hp1) - du) - q) + t1;
            } else {
                const double* c = atan2_row(u);
                double t = (u - c[0]) + du;
                r = (hp0 - c[1]) + fma(-t, atan2_tpoly(c, t), hp1);
            }
        }
    } else {
        if (ay <= ax) {  // pi - atan(u)
            if (u < 0.0625) {
                double z2 = u * u;
                double q = (z2 * u) * atan2_poly(z2);
                double t1 = pi - u;
                double r1 = (pi > fabs(u)) ? ((pi - t1) - u) : (pi - (t1 + u));
                r = (((r1 + pi_lo) - du) - q) + t1;
            } else {
                const double* c = atan2_row(u);
                double t = (u - c[0]) + du;
                r = (pi - c[1]) + fma(-t, atan2_tpoly(c, t), pi_lo);
            }
        } else {  // pi/2 + atan(u)
            if (u < 0.0625) {
                double z2 = u * u;
                double t1 = u + hp0;
                double q = (z2 * u) * atan2_poly(z2);
                double r1 = (hp0 > fabs(u)) ? ((hp0 - t1) + u) : ((u - t1) + hp0);
                r = (((r1 + hp1) + du) + q) + t1;
            } else {
                const double* c = atan2_row(u);
                double t = (u - c[0]) + du;
                r = (hp0 + c[1]) + fma(t, atan2_tpoly(c, t), hp1);
            }
        }
    }
    return copysign(r, y);
}

// ---- atan: s_atan.c __atan (FMA build, s_atan-fma.o), table cij shared with atan2 ----
// Thresholds A = 0x1.bb67ap-27 (.LC6), B = 1/16, C = 1, D = 16, E = 0x1.49ff2p+53; the shipped
// object contracts TWO52 + TWO8 u, the EMULV products and the Horner steps into fused ops.
MOSAIC_HD double atan(double x) {
    const double hp0 = kHp0, hp1 = kHp1;
    const uint32_t ux = (uint32_t)hi32(x), dx = lo32(x);
    if ((ux & 0x7ff00000) == 0x7ff00000 && ((ux & 0x000fffff) | dx) != 0) return x + x;
    const double u = (x < 0) ? -x : x;
    const double A = 0x1.bb67ap-27, E = 0x1.49ff2p+53;
    if (u < 1.0) {
        if (u < 0.0625) {
            if (u < A) return x;
            const double v = x * x;
            return fma(x * v, atan2_poly(v), x);
        }
        const double* c = atan2_row(u);
        const double z = u - c[0];
        const double yy = fma(fma(fma(fma(c[6], z, c[5]), z, c[4]), z, c[3]), z, c[2]);
        return copysign(fma(yy, z, c[1]), x);
    }
    if (u < 16.0) {
        const double w = 1.0 / u;
        const double t1 = u * w, t2 = fma(u, w, -t1);
        const double* c = atan2_row(w);
        const double z = fma((1.0 - t1) - t2, w, w - c[0]);
        const double yy = fma(-z, atan2_tpoly(c, z), hp1);
        return copysign((hp0 - c[1]) + yy, x);
    }
    if (u < E) {
        const double w = 1.0 / u;
        const double v = w * w, t1 = u * w;
        const double yy = (w * v) * atan2_poly(v);
        const double t2 = fma(u, w, -t1);
        const double ww = ((1.0 - t1) - t2) * w;
        const double t3 = hp0 - w;
        const double cor = (hp0 > fabs(w)) ? (hp0 - t3) - w : hp0 - (w + t3);
        return copysign(((((cor + hp1) - ww) - yy) + t3), x);
    }
    return (x < 0) ? -hp0 : hp0;
}

// ---- asin: e_asin.c __ieee754_asin (FMA build, e_asin-fma.o), tables asncs / inroot / powtwo ----
MOSAIC_HD double asin(double x) {
    const double hp0 = kHp0, hp1 = kHp1;
    const double f1 = 0x1.55555555554f9p-3, f2 = 0x1.333333336127dp-4, f3 = 0x1.6db6dae42c0e4p-5,
                 f4 = 0x1.f1c7e04f4ad99p-6, f5 = 0x1.6e442c822d419p-6, f6 = 0x1.292d80f453c72p-6;
    const double rt0 = 0x1.fffffffecc1ddp-1, rt1 = 0x1.fffffff757304p-2, rt2 = 0x1.800496769c91ap-2,
                 rt3 = 0x1.4006318d1dab9p-2;
    const double t24 = 0x1p+24;
    const int32_t m = hi32(x);
    const int32_t k = m & 0x7fffffff;
    if (k < 0x3e500000) return x;
    if (k < 0x3fc00000) {  // |x| < 0.125
        const double x2 = x * x;
        const double p = fma(fma(fma(fma(fma(f6, x2, f5), x2, f4), x2, f3), x2, f2), x2, f1);
        return fma(x * x2, p, x);
    }
    if (k < 0x3fef0000) {  // 0.125 <= |x| < 0.96875: per-interval polynomial in |x| - x0
        int n, top;
        if (k < 0x3fd00000) {
            n = 11 * ((k >> 15) & 0x1f);
            top = 6;
        } else if (k < 0x3fe00000) {
            n = 352 + 11 * ((k >> 14) & 0x3f);
            top = 6;
        } else if (k < 0x3fe80000) {
            n = 1056 + 12 * ((k >> 13) & 0x7f);
            top = 7;
        } else if (k < 0x3fed8000) {
            n = 992 + 13 * ((k >> 13) & 0x7f);
            top = 8;
        } else if (k < 0x3fee8000) {
            n = 884 + 14 * ((k >> 13) & 0x7f);
            top = 9;
        } else {
            n = 768 + 15 * ((k >> 13) & 0x7f);
            top = 10;
        }
        const double* T = kAsnCs + n;
        const double xx = ((m > 0) ? x : -x) - T[0];
        const double xx2 = xx * xx;
        double p = T[top];
        for (int j = top - 1; j >= 2; j--) p = fma(xx, p, T[j]);
        p = fma(xx2, p, T[top + 1]);
        const double res = fma(xx, T[1], p) + T[top + 2];
        return (m > 0) ? res : -res;
    }
    if (k < 0x3ff00000) {  // 0.96875 <= |x| < 1: pi/2 - 2 asin(sqrt((1 - |x|) / 2))
        const double z = ((m > 0) ? (1.0 - x) : (x + 1.0)) * 0.5;
        const int64_t zb = (int64_t)bits(z);
        double t = kInRoot[(int)((zb >> 46) & 0x7f)] * kPowTwo[0x1ff - (int)(zb >> 53)];
        const double r = fma(-(t * t), z, 1.0);
        t = fma(fma(fma(rt3, r, rt2), r, rt1), r, rt0) * t;
        const double c = z * t;
        const double y = (c + t24) - t24;
        const double den = fma(fma(-c, t * 0.5, 1.5), c, y);
        const double cc = fma(-y, y, z) / den;
        const double p = fma(fma(fma(fma(fma(f6, z, f5), z, f4), z, f3), z, f2), z, f1) * z;
        const double cor = fma(-((y + cc) + (y + cc)), p, fma(-2.0, cc, hp1));
        const double res = cor + fma(-2.0, y, hp0);
        return (m > 0) ? res : -res;
    }
    if (k == 0x3ff00000 && lo32(x) == 0) return (m > 0) ? hp0 : -hp0;
    if (k > 0x7ff00000 || (k == 0x7ff00000 && lo32(x) != 0)) return x + x;
    const double zz = x - x;
    return zz / zz;
}

}  // namespace glibc
}  // namespace mosaic
