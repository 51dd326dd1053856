// H3 v3.7 geoToH3 for gfx950 (and the host, for self-checks): the point -> cell step of
// grid_pointascellid / grid_longlatascellid (reference H3IndexSystem.pointToIndex,
// src/main/scala/com/databricks/labs/mosaic/core/index/H3IndexSystem.scala:140-142, which calls
// h3-java geoToH3(lat, lon, res) -> H3 C geoToH3).
//
// Two paths, one answer:
//  * h3_fast():  the acos/azimuth/tan/sin/cos chain of H3's _geoToHex2d is mathematically the
//    gnomonic (projective) map  x = S (EI.p)/(FC.p), y = S (EP.p)/(FC.p)  of the unit vector p.
//    That costs two sincos, 20 face dot products and one division instead of ~11 FP64
//    transcendentals.  It then checks how far the point is from every decision the integer part
//    of H3 makes (closest face, the hex-rounding thresholds of _hex2dToCoordIJK, the axis folds):
//    if every margin exceeds a bound on |fast - H3| (both errors included), H3 on the same input
//    necessarily takes the same decisions, so the cell is identical.  Otherwise it reports
//    "ambiguous" and the caller runs
//  * h3_exact(): a line-by-line restatement of H3 C with x86-64 semantics, including the
//    x87 long-double operations (x87.h), for the rare ambiguous points (~1e-8 of uniform input).
// Both share the integer stage (_hex2dToCoordIJK result -> _faceIjkToH3).
#pragma once
#include <math.h>
#include <stdint.h>

#include "glibc_math.h"
#include "x87.h"

namespace mosaic {
namespace h3 {

#if defined(__HIPCC__)
#define H3_TABLE static __constant__ const
#define H3_LUT static __device__ const
#else
#define H3_TABLE static const
#define H3_LUT static const
#endif
#include "h3_face_lut.h"
#include "h3_fast_tables.h"
#include "h3_tables.h"
#undef H3_TABLE
#undef H3_LUT

static const double kRes0UGnomonic = 0.38196601125010500003;

struct IJK {
    int i, j, k;
};

MOSAIC_HD void ijk_normalize(IJK& c) {
    if (c.i < 0) {
        c.j -= c.i;
        c.k -= c.i;
        c.i = 0;
    }
    if (c.j < 0) {
        c.i -= c.j;
        c.k -= c.j;
        c.j = 0;
    }
    if (c.k < 0) {
        c.i -= c.k;
        c.j -= c.k;
        c.k = 0;
    }
    int mn = c.i;
    if (c.j < mn) mn = c.j;
    if (c.k < mn) mn = c.k;
    if (mn > 0) {
        c.i -= mn;
        c.j -= mn;
        c.k -= mn;
    }
}

// lround(n / 7.0) for integer n: no ties are possible (7 is odd), so it is floor((n + 3) / 7).
MOSAIC_HD int round_div7(int n) {
    int t = n + 3;
    int q = t / 7;
    if ((t % 7 != 0) && (t < 0)) q -= 1;
    return q;
}

// coordijk.c _hex2dToCoordIJK, given x2 = |y| / sin60 computed by the caller (exactly as H3 does
// on the exact path, in plain double on the fast path whose margins cover the difference).
MOSAIC_HD IJK hex2d_round(double vx, double vy, double a1, double x2) {
    IJK h;
    h.k = 0;
    double x1 = a1 + x2 / 2.0;
    int m1 = (int)x1;
    int m2 = (int)x2;
    double r1 = x1 - m1;
    double r2 = x2 - m2;
    if (r1 < 0.5) {
        if (r1 < 1.0 / 3.0) {
            h.i = m1;
            h.j = (r2 < (1.0 + r1) / 2.0) ? m2 : m2 + 1;
        } else {
            h.j = (r2 < (1.0 - r1)) ? m2 : m2 + 1;
            h.i = ((1.0 - r1) <= r2 && r2 < (2.0 * r1)) ? m1 + 1 : m1;
        }
    } else {
        if (r1 < 2.0 / 3.0) {
            h.j = (r2 < (1.0 - r1)) ? m2 : m2 + 1;
            h.i = ((2.0 * r1 - 1.0) < r2 && r2 < (1.0 - r1)) ? m1 : m1 + 1;
        } else {
            h.i = m1 + 1;
            h.j = (r2 < (r1 / 2.0)) ? m2 : m2 + 1;
        }
    }
    if (vx < 0.0) {
        if ((h.j % 2) == 0) {
            long long axisi = h.j / 2;
            long long diff = h.i - axisi;
            h.i = (int)(h.i - 2.0 * diff);
        } else {
            long long axisi = (h.j + 1) / 2;
            long long diff = h.i - axisi;
            h.i = (int)(h.i - (2.0 * diff + 1));
        }
    }
    if (vy < 0.0) {
        h.i = h.i - (2 * h.j + 1) / 2;
        h.j = -1 * h.j;
    }
    ijk_normalize(h);
    return h;
}

// Distance (in x1/x2 units) from every threshold _hex2dToCoordIJK can compare against.
MOSAIC_HD double hex2d_margin(double a1, double x2) {
    double x1 = a1 + x2 / 2.0;
    double r1 = x1 - floor(x1);
    double r2 = x2 - floor(x2);
    double m = fmin(r1, 1.0 - r1);
    m = fmin(m, fmin(r2, 1.0 - r2));
    m = fmin(m, fabs(r1 - 1.0 / 3.0));
    m = fmin(m, fabs(r1 - 0.5));
    m = fmin(m, fabs(r1 - 2.0 / 3.0));
    m = fmin(m, fabs(r2 - (1.0 + r1) / 2.0));
    m = fmin(m, fabs(r2 - (1.0 - r1)));
    m = fmin(m, fabs(r2 - 2.0 * r1));
    m = fmin(m, fabs(r2 - (2.0 * r1 - 1.0)));
    m = fmin(m, fabs(r2 - r1 / 2.0));
    return m;
}

// ---- digits / base cell (h3Index.c _faceIjkToH3) ----
MOSAIC_HD int rotate60ccw(int d) {
    // 1->5, 5->4, 4->6, 6->2, 2->3, 3->1
    const int t[8] = {0, 5, 3, 1, 6, 4, 2, 7};
    return t[d];
}
MOSAIC_HD int rotate60cw(int d) {
    // 1->3, 3->2, 2->6, 6->4, 4->5, 5->1
    const int t[8] = {0, 3, 6, 2, 5, 1, 4, 7};
    return t[d];
}
MOSAIC_HD int get_digit(uint64_t h, int r) { return (int)((h >> ((15 - r) * 3)) & 7); }
MOSAIC_HD uint64_t set_digit(uint64_t h, int r, int d) {
    int s = (15 - r) * 3;
    return (h & ~((uint64_t)7 << s)) | ((uint64_t)d << s);
}
// The first nonzero digit of 1 .. res (0 if none): the most significant nonzero 3-bit group of the
// used digits.  Written without a loop exit on purpose.  Root cause of the round-4 failure (a
// compiler bug, not a source bug; tools/probes/early_exit/): with H3 C's loop-with-early-return form
// inlined into is_pentagon inside hex_range, the gfx950 code computes the exit test `d != 0` into an
// SGPR lane mask each iteration (v_cmp_ne_u32 s[0:1]) and, after the loop, reads that mask as the
// result (s_and_b64 s[2:3], s[0:1], exec) -- but a VOPC compare writes 0 for inactive lanes, so every
// lane that had left the loop in an earlier iteration read "no nonzero digit"
// (isa_old_is_pentagon.txt).  The same source gives correct code in isolation (the i1 is merged per
// lane: s_andn2 / s_and / s_or with exec each iteration), so the miscompile depends on the
// surrounding control flow; 446 of 1,476 k-ring rows near pentagons differed with the round-4
// headers, 0 with these.  Device code keeps such "bool decided inside a loop" checks loop-free where
// it can (is_valid_cell, h3_geom's digit check); the remaining loops are covered by mixed-wave GPU
// tests against the oracle.
MOSAIC_HD int leading_nonzero_digit(uint64_t h, int res) {
    const uint64_t d = (h & 0x1fffffffffffULL) >> (3 * (15 - res));  // digits 1 .. res, digit res lowest
    const int msb = d ? 63 - __builtin_clzll(d) : 0;
    return (int)((d >> (3 * (msb / 3))) & 7u);
}
MOSAIC_HD uint64_t rotate_all(uint64_t h, int res, bool ccw) {
    for (int r = 1; r <= res; r++) h = set_digit(h, r, ccw ? rotate60ccw(get_digit(h, r)) : rotate60cw(get_digit(h, r)));
    return h;
}

// rotate_all on all 15 digits at once.  A digit is the unit vector (i, j, k) = its 3 bits; a 60
// degree rotation maps a single axis to itself plus the next axis (ccw: i->ij, j->jk, k->ki) and
// a pair to its shared-next axis (ij->j, jk->k, ki->i): d | next(d) or d & next(d), with next the
// cyclic bit shift.  0 and 7 (unused digits) are fixed points, so no masking by `res` is needed.
MOSAIC_HD uint64_t rotate_all_digits(uint64_t h, bool ccw) {
    const uint64_t kDigits = 0x1fffffffffffULL, kLow = 0x1249249249249ULL;
    uint64_t d = h & kDigits;
    uint64_t K = d & kLow, J = (d >> 1) & kLow, I = (d >> 2) & kLow;
    uint64_t single = (I ^ J ^ K) & ~(I & J & K);
    uint64_t nx = ccw ? ((K << 2) | (I << 1) | J) : ((J << 2) | (K << 1) | I);
    uint64_t s3 = single * 7u;
    uint64_t nd = (s3 & (d | nx)) | (~s3 & d & nx);
    return (h & ~kDigits) | (nd & kDigits);
}
MOSAIC_HD uint64_t rotate_pent60ccw(uint64_t h, int res) {
    bool found = false;
    for (int r = 1; r <= res; r++) {
        h = set_digit(h, r, rotate60ccw(get_digit(h, r)));
        if (!found && get_digit(h, r) != 0) {
            found = true;
            if (leading_nonzero_digit(h, res) == 1) h = rotate_all(h, res, true);
        }
    }
    return h;
}

MOSAIC_HD uint64_t face_ijk_to_h3(int face, IJK ijk, int res) {
    uint64_t h = 0x00001fffffffffffULL | (1ULL << 59) | ((uint64_t)res << 52);
    if (res == 0) {
        if (ijk.i > 2 || ijk.j > 2 || ijk.k > 2) return 0;
        return h | ((uint64_t)(kH3FaceIjkBaseCells[face][ijk.i][ijk.j][ijk.k] >> 3) << 45);
    }
    for (int r = res - 1; r >= 0; r--) {
        IJK last = ijk;
        IJK c;
        int i = ijk.i - ijk.k, j = ijk.j - ijk.k;
        if ((r + 1) & 1) {  // _upAp7 then _downAp7
            ijk.i = round_div7(3 * i - j);
            ijk.j = round_div7(i + 2 * j);
            ijk.k = 0;
            ijk_normalize(ijk);
            c.i = 3 * ijk.i + ijk.j;
            c.j = 3 * ijk.j + ijk.k;
            c.k = ijk.i + 3 * ijk.k;
        } else {  // _upAp7r then _downAp7r
            ijk.i = round_div7(2 * i + j);
            ijk.j = round_div7(3 * j - i);
            ijk.k = 0;
            ijk_normalize(ijk);
            c.i = 3 * ijk.i + ijk.k;
            c.j = ijk.i + 3 * ijk.j;
            c.k = ijk.j + 3 * ijk.k;
        }
        ijk_normalize(c);
        IJK d = {last.i - c.i, last.j - c.j, last.k - c.k};
        ijk_normalize(d);
        // _unitIjkToDigit: UNIT_VECS[digit] = (digit>>2 &1, digit>>1 &1, digit&1)
        int digit = (d.i <= 1 && d.j <= 1 && d.k <= 1) ? (d.i << 2) | (d.j << 1) | d.k : 7;
        h = set_digit(h, r + 1, digit);
    }
    if (ijk.i > 2 || ijk.j > 2 || ijk.k > 2) return 0;
    int packed = kH3FaceIjkBaseCells[face][ijk.i][ijk.j][ijk.k];
    int bc = packed >> 3;
    int rots = packed & 7;
    h |= (uint64_t)bc << 45;
    if (kH3BaseCellData[bc][4]) {
        if (leading_nonzero_digit(h, res) == 1) {
            bool cw = kH3BaseCellData[bc][5] == face || kH3BaseCellData[bc][6] == face;
            h = rotate_all(h, res, !cw);
        }
        for (int i = 0; i < rots; i++) h = rotate_pent60ccw(h, res);
    } else {
        for (int i = 0; i < rots; i++) h = rotate_all(h, res, true);
    }
    return h;
}

// ---- exact path: H3 C v3.7 with x86-64 double / x87 long double semantics ----
// libm: glibc_math.h, the bit-exact restatement of the glibc 2.35 functions H3 C reaches on an
// x86-64 host (sincos for every sin / cos pair, FMA-build acos / atan2 / tan), on the device and
// in host builds alike.
MOSAIC_HD double pos_angle_rads(double rads) {
    double tmp = (rads < 0.0) ? x87::add_ld(rads, H3LD_M_2PI_M, H3LD_M_2PI_E, false) : rads;
    if (rads >= H3LD_M_2PI_DUP) tmp = x87::add_ld(tmp, H3LD_M_2PI_M, H3LD_M_2PI_E, true);
    return tmp;
}

MOSAIC_HD double sq(double v) { return v * v; }

MOSAIC_HD uint64_t h3_exact(double lat, double lon, int res) {
    if (res < 0 || res > 15) return 0;
    if (!isfinite(lat) || !isfinite(lon)) return 0;
    // vec3d.c _geoToVec3d: r = cos(lat); z = sin(lat); x = cos(lon) * r; y = sin(lon) * r
    double pz, r0, slon, clon;
    glibc::sincos(lat, &pz, &r0);
    glibc::sincos(lon, &slon, &clon);
    double px = clon * r0;
    double py = slon * r0;
    int face = 0;
    double sqd = sq(kH3FaceCenterPoint[0][0] - px) + sq(kH3FaceCenterPoint[0][1] - py) +
                 sq(kH3FaceCenterPoint[0][2] - pz);
    for (int f = 1; f < 20; f++) {
        double t = sq(kH3FaceCenterPoint[f][0] - px) + sq(kH3FaceCenterPoint[f][1] - py) +
                   sq(kH3FaceCenterPoint[f][2] - pz);
        if (t < sqd) {
            face = f;
            sqd = t;
        }
    }
    double vx, vy;
    double r = glibc::acos(1 - sqd / 2);
    if (r < H3LD_EPSILON_DUP) {
        vx = vy = 0.0;
    } else {
        // geoCoord.c _geoAzimuthRads(faceCenterGeo[face], g):
        // atan2(cos(lat2) sin(lon2 - lon1), cos(lat1) sin(lat2) - sin(lat1) cos(lat2) cos(lon2 - lon1))
        double lat1 = kH3FaceCenterGeo[face][0], lon1 = kH3FaceCenterGeo[face][1];
        double sdl, cdl, slat1, clat1;
        glibc::sincos(lon - lon1, &sdl, &cdl);
        glibc::sincos(lat1, &slat1, &clat1);
        double az = glibc::atan2(r0 * sdl, clat1 * pz - slat1 * r0 * cdl);
        double theta = pos_angle_rads(kH3FaceAxesAzRadsCII[face][0] - pos_angle_rads(az));
        if (res & 1) theta = pos_angle_rads(x87::add_ld(theta, H3LD_M_AP7_ROT_RADS_M, H3LD_M_AP7_ROT_RADS_E, true));
        r = glibc::tan(r);  // r <= 0.6524 (face circumradius): inside glibc::tan's restated domain
        r /= kRes0UGnomonic;
        for (int i = 0; i < res; i++) r = x87::mul_ld(r, H3LD_M_SQRT7_M, H3LD_M_SQRT7_E);
        double st, ct;
        glibc::sincos(theta, &st, &ct);
        vx = r * ct;
        vy = r * st;
    }
    double a1 = fabs(vx), a2 = fabs(vy);
    double x2 = x87::div_ld(a2, H3LD_M_SIN60_M, H3LD_M_SIN60_E);
    IJK ijk = hex2d_round(vx, vy, a1, x2);
    return face_ijk_to_h3(face, ijk, res);
}

// ---- fast path ----
// sin and cos of x, |x| < 201.5 / 64 (= pi + 0.0068), to ~1 ulp: x = k/64 + r (exact), |r| <= 1/128, table
// values sin/cos(k/64) correctly rounded, short Taylor polynomials for r (truncation < 1e-21).
MOSAIC_HD void fast_sincos(double x, double* s, double* c) {
    double kf = rint(x * 64.0);
    double r = x - kf * 0.015625;  // exact (Sterbenz-like: r is a multiple of ulp(x), |r| < 2^-7)
    int k = (int)kf + 201;
    k = k < 0 ? 0 : (k > 402 ? 402 : k);
    double sk = kH3SinCos64[k][0], ck = kH3SinCos64[k][1];
    double r2 = r * r;
    double sr = fma(r * r2, fma(r2, fma(r2, -1.0 / 5040.0, 1.0 / 120.0), -1.0 / 6.0), r);
    double cr = fma(r2, fma(r2, fma(r2, fma(r2, 1.0 / 40320.0, -1.0 / 720.0), 1.0 / 24.0), -0.5), 1.0);
    *s = fma(sk, cr, ck * sr);
    *c = fma(ck, cr, -(sk * sr));
}

// Closest face by full search (the 20 face dot products); sets *gap to best - second best.
MOSAIC_HD int face_search(double px, double py, double pz, double* best_out, double* gap) {
    double best = -2.0, second = -2.0;
    int face = 0;
#pragma unroll 1
    for (int f = 0; f < 20; f++) {
        const double* b = kH3FastBasis[f];
        double d = fma(b[0], px, fma(b[1], py, b[2] * pz));
        if (d > best) {
            second = best;
            best = d;
            face = f;
        } else if (d > second) {
            second = d;
        }
    }
    *best_out = best;
    *gap = best - second;
    return face;
}

// round(n / 7) for |n| < 2^27: floor((n + 3) / 7), via an unsigned division of a shifted numerator
MOSAIC_HD constexpr int div7r(int n) {
    const unsigned off = 7u << 25;
    return (int)(((unsigned)(n + 3) + off) / 7u) - (1 << 25);
}
// floor(n / 7) for |n| < 2^27
MOSAIC_HD constexpr int div7f(int n) {
    const unsigned off = 7u << 25;
    return (int)(((unsigned)n + off) / 7u) - (1 << 25);
}

// digit <- axial (i - k, j - k) offset of a child from its parent's centre; 7 = invalid.
// The 3x3 table {1, 3, 7, 5, 0, 2, 7, 4, 6} packed 3 bits per entry.
MOSAIC_HD constexpr int axial_digit(int da, int db) {
    const unsigned kPacked = 0x69d0bd9u;
    unsigned ia = (unsigned)(da + 1), ib = (unsigned)(db + 1);
    return (ia < 3 && ib < 3) ? (int)((kPacked >> (3u * (ia * 3u + ib))) & 7u) : 7;
}

// One level of _faceIjkToH3 in axial coordinates: the parent (a, b) <- child (a, b) at level r, and
// the child's digit.  Class III (r odd): _upAp7, centre _downAp7 = axial (2I + J, 3J - I); Class II:
// _upAp7r, centre _downAp7r = axial (3I - J, I + 2J).
MOSAIC_HD constexpr int axial_up(int& a, int& b, bool class3) {
    int I = 0, J = 0, da = 0, db = 0;
    if (class3) {
        I = div7r(3 * a - b);
        J = div7r(a + 2 * b);
        da = a - (2 * I + J);
        db = b - (3 * J - I);
    } else {
        I = div7r(2 * a + b);
        J = div7r(3 * b - a);
        da = a - (3 * I - J);
        db = b - (I + 2 * J);
    }
    a = I;
    b = J;
    return axial_digit(da, db);
}

// Two levels at once.  The two steps' centre maps compose to 7 x identity -- (2I + J, 3J - I) of
// (3I - J, I + 2J) is (7I, 7J), in either order -- and each step's rounding commutes with
// translations by its parent lattice, so with (a, b) = 7 (qa, qb) + (ra, rb), 0 <= ra, rb < 7, the two
// digits depend on (ra, rb) alone and the grandparent is (qa, qb) + a small offset from (ra, rb).
// Table [first level is Class III][7 ra + rb]: bits 0-2 the first (finer) level's digit, 3-5 the
// second's, 6-8 / 9-11 the grandparent offset + 2.  Built at compile time from axial_up itself.
struct AxialPairTab {
    uint16_t v[2][49];
};
MOSAIC_HD constexpr AxialPairTab make_axial_pair_tab() {
    AxialPairTab t{};
    for (int c3 = 0; c3 < 2; c3++)
        for (int ra = 0; ra < 7; ra++)
            for (int rb = 0; rb < 7; rb++) {
                int a = ra, b = rb;
                const int d1 = axial_up(a, b, c3 != 0);
                const int d2 = axial_up(a, b, c3 == 0);
                t.v[c3][7 * ra + rb] = (uint16_t)(d1 | d2 << 3 | (a + 2) << 6 | (b + 2) << 9);
            }
    return t;
}
#if defined(__HIPCC__)
static __constant__ const AxialPairTab kAxialPairs = make_axial_pair_tab();
#else
static const AxialPairTab kAxialPairs = make_axial_pair_tab();
#endif

// Four levels at once, by the same argument twice: the two pair steps compose to 49 x identity, so
// with (a, b) = 49 (qa, qb) + (ra, rb), 0 <= ra, rb < 49, the four digits depend on (ra, rb) alone and
// the level-4 ancestor is (qa, qb) + an offset in [-3, 3].  Table [first level is Class III][49 ra + rb]:
// bits 0-11 the four digits (finest lowest), 12-14 / 15-17 the ancestor offset + 3.  Built at compile
// time from the pair table (tests/native/h3_pairs_check.cpp: identical to the one-level form).
struct AxialQuadTab {
    uint32_t v[2][2401];
};
MOSAIC_HD constexpr AxialQuadTab make_axial_quad_tab() {
    AxialQuadTab t{};
    const AxialPairTab P = make_axial_pair_tab();
    for (int c3 = 0; c3 < 2; c3++)
        for (int ra = 0; ra < 49; ra++)
            for (int rb = 0; rb < 49; rb++) {
                const unsigned e1 = P.v[c3][7 * (ra % 7) + rb % 7];
                const int a1 = ra / 7 + (int)((e1 >> 6) & 7u) - 2, b1 = rb / 7 + (int)((e1 >> 9) & 7u) - 2;
                const int qa = div7f(a1), qb = div7f(b1);
                const unsigned e2 = P.v[c3][7 * (a1 - 7 * qa) + (b1 - 7 * qb)];
                const int a2 = qa + (int)((e2 >> 6) & 7u) - 2, b2 = qb + (int)((e2 >> 9) & 7u) - 2;
                t.v[c3][49 * ra + rb] = (e1 & 63u) | (e2 & 63u) << 6 | (unsigned)(a2 + 3) << 12 | (unsigned)(b2 + 3) << 15;
            }
    return t;
}
#if defined(__HIPCC__)
static __constant__ const AxialQuadTab kAxialQuads = make_axial_quad_tab();
#else
static const AxialQuadTab kAxialQuads = make_axial_quad_tab();
#endif
// floor(n / 49) for |n| < 2^27
MOSAIC_HD constexpr int div49f(int n) {
    const unsigned off = 49u << 22;
    return (int)(((unsigned)n + off) / 49u) - (1 << 22);
}

// _faceIjkToH3 in axial coordinates (a, b) = (i - k, j - k) of the res-`res` cell on `face`.
// Same arithmetic as face_ijk_to_h3 (the axial pair is invariant under _ijkNormalize, and
// _downAp7 / _downAp7r are linear), with the three normalisations per level removed and the levels
// taken two at a time (kAxialPairs: two floor divisions by 7 and one table read per pair instead of
// four rounding divisions and two digit decodings); face_axial_to_h3_levels is the one-level form,
// kept for the self-check (tests/native/h3_pairs_check.cpp: identical on every input).
MOSAIC_HD uint64_t axial_base_to_h3(int face, int a, int b, int res, uint64_t digits) {
    uint64_t h = digits | (1ULL << 59) | ((uint64_t)res << 52);
    IJK ijk = {a, b, 0};
    ijk_normalize(ijk);
    if (ijk.i > 2 || ijk.j > 2 || ijk.k > 2) return 0;
    int packed = kH3FaceIjkBaseCells[face][ijk.i][ijk.j][ijk.k];
    int bc = packed >> 3;
    int rots = packed & 7;
    h |= (uint64_t)bc << 45;
    if (kH3BaseCellData[bc][4]) {  // pentagon: the reference rotation sequence
        if (leading_nonzero_digit(h, res) == 1) {
            bool cw = kH3BaseCellData[bc][5] == face || kH3BaseCellData[bc][6] == face;
            h = rotate_all(h, res, !cw);
        }
        for (int i = 0; i < rots; i++) h = rotate_pent60ccw(h, res);
    } else if (rots) {
        for (int i = 0; i < rots; i++) h = rotate_all_digits(h, true);
    }
    return h;
}
MOSAIC_HD uint64_t face_axial_to_h3_levels(int face, int a, int b, int res) {
    uint64_t h = 0x00001fffffffffffULL;
    for (int r = res; r >= 1; r--) {
        const int s = (15 - r) * 3;
        h = (h & ~((uint64_t)7 << s)) | ((uint64_t)axial_up(a, b, (r & 1) != 0) << s);
    }
    return axial_base_to_h3(face, a, b, res, h);
}
MOSAIC_HD uint64_t face_axial_to_h3(int face, int a, int b, int res) {
    // digits of levels res .. 1 gathered with level res lowest, placed above the unused 7s at the end
    uint64_t d = 0;
    int sh = 0, r = res;
    const int c3 = res & 1;  // every pair starts on a level of res's parity
    for (; r >= 2; r -= 2, sh += 6) {
        const int qa = div7f(a), qb = div7f(b);
        const unsigned e = kAxialPairs.v[c3][7 * (a - 7 * qa) + (b - 7 * qb)];
        d |= (uint64_t)(e & 63u) << sh;
        a = qa + (int)((e >> 6) & 7u) - 2;
        b = qb + (int)((e >> 9) & 7u) - 2;
    }
    if (r == 1) d |= (uint64_t)axial_up(a, b, true) << sh;
    const int low = 3 * (15 - res);
    const uint64_t digits = (d << low) | ((1ULL << low) - 1ULL);
    return axial_base_to_h3(face, a, b, res, digits);
}
// face_axial_to_h3 with the levels four at a time (kAxialQuads), then at most one pair and one level.
MOSAIC_HD uint64_t face_axial_to_h3_quad(int face, int a, int b, int res, const uint32_t* Q) {
    uint64_t d = 0;
    int sh = 0, r = res;
    const int c3 = res & 1;
    for (; r >= 4; r -= 4, sh += 12) {
        const int qa = div49f(a), qb = div49f(b);
        const unsigned e = Q[49 * (a - 49 * qa) + (b - 49 * qb)];
        d |= (uint64_t)(e & 4095u) << sh;
        a = qa + (int)((e >> 12) & 7u) - 3;
        b = qb + (int)((e >> 15) & 7u) - 3;
    }
    if (r >= 2) {
        const int qa = div7f(a), qb = div7f(b);
        const unsigned e = kAxialPairs.v[c3][7 * (a - 7 * qa) + (b - 7 * qb)];
        d |= (uint64_t)(e & 63u) << sh;
        a = qa + (int)((e >> 6) & 7u) - 2;
        b = qb + (int)((e >> 9) & 7u) - 2;
        r -= 2, sh += 6;
    }
    if (r == 1) d |= (uint64_t)axial_up(a, b, true) << sh;
    const int low = 3 * (15 - res);
    return axial_base_to_h3(face, a, b, res, (d << low) | ((1ULL << low) - 1ULL));
}

// The unit vector of (lat_deg, lon_deg) for the fast path: radians by one multiply (within 2 ulp of
// Java's toRadians, covered by the error bound) and the table sine / cosine.  Finite inputs only.
MOSAIC_HD void fast_unit(double lat_deg, double lon_deg, double* px, double* py, double* pz) {
    const double d2r = 0.017453292519943295;
    double lat = lat_deg * d2r, lon = lon_deg * d2r;
    double slat, clat, slon, clon;
    // fast_sincos's table spans k / 64 for |k| <= 201, i.e. |x| < 201.5 / 64 = 3.1484375 (180.39 deg)
    if (fabs(lon) < 3.1484375 && fabs(lat) < 3.1484375) {
        fast_sincos(lat, &slat, &clat);
        fast_sincos(lon, &slon, &clon);
    } else {  // |lon| beyond 180.39 deg (or |lat| beyond): glibc's sincos, < 0.55 ulp on host and device
        glibc::sincos(lat, &slat, &clat);
        glibc::sincos(lon, &slon, &clon);
    }
    *px = clon * clat;
    *py = slon * clat;
    *pz = slat;
}

// Face-plane coordinates (res-`res` hex units, Class III rotation included) of the unit vector p on
// `face`, and best = FC(face) . p.
MOSAIC_HD void fast_plane(double px, double py, double pz, int face, int res, double* vx, double* vy,
                          double* best) {
    const double* fb = kH3FastBasis[face];
    const double* ei = fb + ((res & 1) ? 9 : 3);
    const double* ep = fb + ((res & 1) ? 12 : 6);
    double b = fma(fb[0], px, fma(fb[1], py, fb[2] * pz));
    double s = kH3FastScale[res] / b;
    *vx = s * fma(ei[0], px, fma(ei[1], py, ei[2] * pz));
    *vy = s * fma(ep[0], px, fma(ep[1], py, ep[2] * pz));
    *best = b;
}

// The certified integer part of the fast path on a known face: the res-`res` hexagon (axial
// (ba, bb) = (i - k, j - k)) of face-plane point (vx, vy), or false when a decision is too close to
// call (the caller then runs h3_exact).
MOSAIC_HD bool fast_hex(double vx, double vy, int res, int* ba_out, int* bb_out) {
    const double S = kH3FastScale[res];
    double a1 = fabs(vx), a2 = fabs(vy);
    // bound on |fast - H3| per hex2d coordinate ("H3 fast path"): relative rounding of
    // both computations, the acos(1 - sqd/2) ill-conditioning near the face centre, and the
    // 2-ulp radians difference.
    // The bound is delta = 64 eps rh + 32 eps S^2 / rh + 8 eps S; every comparison against it is
    // made multiplied by rh > 0 (drh = delta * rh, widened by 1e-12 for its own rounding), so no
    // division is needed.  rh == 0 compares 0 < positive: ambiguous, as it must be.
    const double eps = 1.1102230246251565e-16;
    double rh = a1 + a2;
    double drh = (64.0 * eps * rh * rh + 32.0 * eps * S * S + 8.0 * eps * S * rh) * (1.0 + 1e-12);
    if (a1 * rh < 8.0 * drh || a2 * rh < 8.0 * drh) return false;  // axis folds, r < EPSILON centre
    // nearest lattice centre (H3's _hex2dToCoordIJK is exact hexagon rounding) and the distance
    // from the point to that hexagon's boundary
    // Centres are a e1 + b e2 with e1 = (1, 0), e2 = (-1/2, sin60).  Cube rounding in the 60-degree
    // basis (e1, e1 + e2): u = a - b, w = b, t = -u - w; round all three, recompute the one that
    // moved most.  The margin test below re-derives the distance to the chosen hexagon's boundary,
    // so a wrong centre could only ever make the point "ambiguous", never wrong.
    const double s60 = 0.86602540378443864676, inv_s60 = 1.1547005383792515;
    double wq = vy * inv_s60;
    double uq = vx - 0.5 * wq;
    double tq = -uq - wq;
    double ru = rint(uq), rw = rint(wq), rt = rint(tq);
    double du = fabs(ru - uq), dw = fabs(rw - wq), dt = fabs(rt - tq);
    if (du > dw && du > dt) ru = -rw - rt;
    else if (dw > dt) rw = -ru - rt;
    int ba = (int)(ru + rw), bb = (int)rw;
    double dx = vx - ((double)ba - 0.5 * (double)bb);
    double dy = vy - (double)bb * s60;
    double m = 0.5 - fmax(fabs(dx), fmax(fabs(0.5 * dx + s60 * dy), fabs(0.5 * dx - s60 * dy)));
    if (m * rh < 4.0 * drh) return false;
    *ba_out = ba;
    *bb_out = bb;
    return true;
}

// Closest face of unit vector p: the 1-degree lookup cell is wholly inside one face's region
// (gap > 3e-3), or the full search with a gap check.  Returns -1 when too close to call.
MOSAIC_HD int fast_face(double lat_deg, double lon_deg, double px, double py, double pz) {
    int li = (int)floor(lat_deg + 90.0), lj = (int)floor(lon_deg + 180.0);
    int face = (li >= 0 && li < 180 && lj >= 0 && lj < 360) ? (int)kH3FaceLut[li][lj] : 255;
    if (face != 255) return face;
    double best, gap;
    face = face_search(px, py, pz, &best, &gap);
    return gap < 1e-12 ? -1 : face;
}

// Returns the cell of (lat_deg, lon_deg) -- the cell H3 C computes from Math.toRadians of the same
// degrees -- or sets *ambiguous and returns 0 when a decision is too close to call.
MOSAIC_HD uint64_t h3_fast(double lat_deg, double lon_deg, int res, bool* ambiguous) {
    *ambiguous = false;
    if (res < 0 || res > 15) return 0;
    if (!isfinite(lat_deg) || !isfinite(lon_deg)) return 0;
    double px, py, pz;
    fast_unit(lat_deg, lon_deg, &px, &py, &pz);
    int face = fast_face(lat_deg, lon_deg, px, py, pz);
    if (face < 0) {
        *ambiguous = true;
        return 0;
    }
    double vx, vy, best;
    fast_plane(px, py, pz, face, res, &vx, &vy, &best);
    int ba, bb;
    if (!fast_hex(vx, vy, res, &ba, &bb)) {
        *ambiguous = true;
        return 0;
    }
    return face_axial_to_h3(face, ba, bb, res);
}

// h3_fast for two points at once (the cell kernel's two rows per lane): the same arithmetic stage by
// stage for both, so the two independent chains interleave in one instruction stream.  Points off the
// common path (non-finite, beyond the table sine's range, outside the face lookup table's cells) are
// reported in rare[] (out 0) for the caller to run h3_fast on -- out of this instruction stream: its
// glibc sincos and 20-face search, inlined here, cost the common path registers.  Otherwise out /
// amb exactly as h3_fast's (host self-check: tests/native/h3_host_selfcheck.cpp).
// The digit tables are parameters (a kernel passes its LDS copies, referenced directly so that the
// reads compile to LDS loads -- a pointer chosen at run time between LDS and the constant table is a
// flat pointer, and the loads go through the vector memory path); Q = the four-level table of res's
// parity (kAxialQuads.v[res & 1] or a copy), used when kQuad.
template <int K, bool kQuad>
MOSAIC_HD void h3_fastk_tab(const double lat[K], const double lon[K], int res, uint64_t out[K], bool amb[K], bool rare[K],
                            const AxialPairTab& P, const uint32_t* Q) {
    if (res < 0 || res > 15) {
        for (int k = 0; k < K; k++) out[k] = 0, amb[k] = rare[k] = false;
        return;
    }
    bool common[K], ok[K];
    int face[K], a[K], b[K];
    double px[K], py[K], pz[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        const double d2r = 0.017453292519943295;
        const double la = lat[k] * d2r, lo = lon[k] * d2r;
        common[k] = fabs(lo) < 3.1484375 && fabs(la) < 3.1484375;  // (false for NaN and infinities)
        double slat, clat, slon, clon;
        fast_sincos(common[k] ? la : 0.0, &slat, &clat);
        fast_sincos(common[k] ? lo : 0.0, &slon, &clon);
        px[k] = clon * clat, py[k] = slon * clat, pz[k] = slat;
        const int li = common[k] ? (int)floor(lat[k] + 90.0) : -1, lj = common[k] ? (int)floor(lon[k] + 180.0) : -1;
        const int f = (li >= 0 && li < 180 && lj >= 0 && lj < 360) ? (int)kH3FaceLut[li][lj] : 255;
        common[k] = f != 255;
        face[k] = common[k] ? f : 0;
    }
    double vx[K], vy[K];
#if defined(__HIP_DEVICE_COMPILE__)
    // a wave whose points all lie on one face (nearly every wave of a regional batch) reads that face's
    // basis with scalar loads into SGPRs instead of 15 vector gathers per point
    const int f0 = __builtin_amdgcn_readfirstlane(face[0]);
    bool other = false;
#pragma unroll
    for (int k = 0; k < K; k++) other = other || face[k] != f0;
    if (__ballot(other) == 0) {
        const double* fb = kH3FastBasis[f0];
        const double* ei = fb + ((res & 1) ? 9 : 3);
        const double* ep = fb + ((res & 1) ? 12 : 6);
#pragma unroll
        for (int k = 0; k < K; k++) {
            const double bb = fma(fb[0], px[k], fma(fb[1], py[k], fb[2] * pz[k]));
            const double sc = kH3FastScale[res] / bb;
            vx[k] = sc * fma(ei[0], px[k], fma(ei[1], py[k], ei[2] * pz[k]));
            vy[k] = sc * fma(ep[0], px[k], fma(ep[1], py[k], ep[2] * pz[k]));
        }
    } else
#endif
    {
#pragma unroll
        for (int k = 0; k < K; k++) {
            double best;
            fast_plane(px[k], py[k], pz[k], face[k], res, &vx[k], &vy[k], &best);
        }
    }
#pragma unroll
    for (int k = 0; k < K; k++) {
        a[k] = b[k] = 0;
        ok[k] = fast_hex(vx[k], vy[k], res, &a[k], &b[k]);
        if (!ok[k]) a[k] = b[k] = 0;
    }
    uint64_t d[K];
#pragma unroll
    for (int k = 0; k < K; k++) d[k] = 0;
    int sh = 0, r = res;
    const int c3 = res & 1;
    if (kQuad) {
        for (; r >= 4; r -= 4, sh += 12) {
#pragma unroll
            for (int k = 0; k < K; k++) {
                const int qa = div49f(a[k]), qb = div49f(b[k]);
                const unsigned e = Q[49 * (a[k] - 49 * qa) + (b[k] - 49 * qb)];
                d[k] |= (uint64_t)(e & 4095u) << sh;
                a[k] = qa + (int)((e >> 12) & 7u) - 3;
                b[k] = qb + (int)((e >> 15) & 7u) - 3;
            }
        }
    }
    for (; r >= 2; r -= 2, sh += 6) {
#pragma unroll
        for (int k = 0; k < K; k++) {
            const int qa = div7f(a[k]), qb = div7f(b[k]);
            const unsigned e = P.v[c3][7 * (a[k] - 7 * qa) + (b[k] - 7 * qb)];
            d[k] |= (uint64_t)(e & 63u) << sh;
            a[k] = qa + (int)((e >> 6) & 7u) - 2;
            b[k] = qb + (int)((e >> 9) & 7u) - 2;
        }
    }
    const int low = 3 * (15 - res);
#pragma unroll
    for (int k = 0; k < K; k++) {
        if (r == 1) d[k] |= (uint64_t)axial_up(a[k], b[k], true) << sh;
        const uint64_t h = axial_base_to_h3(face[k], a[k], b[k], res, (d[k] << low) | ((1ULL << low) - 1ULL));
        out[k] = ok[k] && common[k] ? h : 0;
        amb[k] = !ok[k] && common[k];
        rare[k] = !common[k];
    }
}
template <int K>
MOSAIC_HD void h3_fastk(const double lat[K], const double lon[K], int res, uint64_t out[K], bool amb[K], bool rare[K]) {
    h3_fastk_tab<K, false>(lat, lon, res, out, amb, rare, kAxialPairs, nullptr);
}
MOSAIC_HD void h3_fast2(const double lat[2], const double lon[2], int res, uint64_t out[2], bool amb[2], bool rare[2]) {
    h3_fastk<2>(lat, lon, res, out, amb, rare);
}
MOSAIC_HD void h3_fast2_quad(const double lat[2], const double lon[2], int res, uint64_t out[2], bool amb[2], bool rare[2]) {
    h3_fastk_tab<2, true>(lat, lon, res, out, amb, rare, kAxialPairs, res >= 0 && res <= 15 ? kAxialQuads.v[res & 1] : nullptr);
}

// java.lang.Math.toRadians (h3-java converts degrees in Java before calling H3 C)
MOSAIC_HD double to_radians(double deg, int jdk) {
    if (jdk <= 8) return deg / 180.0 * 3.141592653589793;
    return deg * 0.017453292519943295;
}

}  // namespace h3
}  // namespace mosaic
