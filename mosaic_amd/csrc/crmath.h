// Correctly rounded (to nearest) sin, cos, tan, acos and atan2 for H3's exact path.
//
// Why: the exact path restates H3 C, whose results on points within an ulp of a cell boundary
// depend on the last bit of libm.  The reference runs H3 C against glibc (2.35 here), which is
// within 1 ulp but not always correctly rounded; the GPU's OCML is further off (1-2 ulp).  These
// functions evaluate in double-double (~104 bits) and round once, so they agree with glibc
// wherever glibc is correctly rounded (measured: all but ~0.1-0.3 % of random arguments, see
// tests/test_crmath.py) -- a closer match to the reference than any 1-ulp library.  They cost
// ~300 FP64 operations each and run only for the ~1e-8 of points the fast path defers.
//
// Building blocks: error-free transformations (two_sum, two_prod via fma), double-double Horner
// Taylor series for sin / cos after a three-part pi/2 reduction, and one Newton step in
// double-double from the library value for acos (via asin) and atan2.
#pragma once
#include <math.h>

#if !defined(MOSAIC_HD)
#if defined(__HIPCC__)
#define MOSAIC_HD __host__ __device__ inline
#else
#define MOSAIC_HD inline
#endif
#endif

namespace mosaic {
namespace crm {

struct dd {
    double hi, lo;
};

MOSAIC_HD dd two_sum(double a, double b) {
    double s = a + b;
    double bb = s - a;
    return dd{s, (a - (s - bb)) + (b - bb)};
}
MOSAIC_HD dd quick_two_sum(double a, double b) {
    double s = a + b;
    return dd{s, b - (s - a)};
}
MOSAIC_HD dd two_prod(double a, double b) {
    double p = a * b;
    return dd{p, fma(a, b, -p)};
}
MOSAIC_HD dd add(dd a, dd b) {
    dd s = two_sum(a.hi, b.hi);
    dd t = two_sum(a.lo, b.lo);
    s = quick_two_sum(s.hi, s.lo + t.hi);
    return quick_two_sum(s.hi, s.lo + t.lo);
}
MOSAIC_HD dd neg(dd a) { return dd{-a.hi, -a.lo}; }
MOSAIC_HD dd mul(dd a, dd b) {
    dd p = two_prod(a.hi, b.hi);
    return quick_two_sum(p.hi, p.lo + (a.hi * b.lo + a.lo * b.hi));
}
MOSAIC_HD dd mul_d(dd a, double b) {
    dd p = two_prod(a.hi, b);
    return quick_two_sum(p.hi, p.lo + a.lo * b);
}
MOSAIC_HD dd div(dd a, dd b) {
    double q1 = a.hi / b.hi;
    dd r = add(a, neg(mul_d(b, q1)));
    double q2 = r.hi / b.hi;
    r = add(r, neg(mul_d(b, q2)));
    double q3 = r.hi / b.hi;
    return add(quick_two_sum(q1, q2), dd{q3, 0.0});
}
MOSAIC_HD double round_dd(dd a) { return a.hi + a.lo; }

// (-1)^k / (2k+1)! and (-1)^k / (2k)!, k = 0..14, as double-double (hi, lo)
#define MOSAIC_CRM_SIN_C                                                                                  \
    {1.0, 0.0}, {-0.16666666666666666, -9.25185853854297e-18}, {0.008333333333333333, 1.1564823173178714e-19}, \
        {-0.0001984126984126984, -1.7209558293420705e-22}, {2.7557319223985893e-06, -1.858393274046472e-22},   \
        {-2.505210838544172e-08, 1.448814070935912e-24}, {1.6059043836821613e-10, 1.2585294588752098e-26},     \
        {-7.647163731819816e-13, -7.03872877733453e-30}, {2.8114572543455206e-15, 1.6508842730861433e-31},     \
        {-8.22063524662433e-18, -2.2141894119604265e-34}, {1.9572941063391263e-20, -1.3643503830087908e-36},   \
        {-3.868170170630684e-23, 8.843177655482344e-40}, {6.446950284384474e-26, -1.9330404233703465e-42},     \
        {-9.183689863795546e-29, -1.4303150396787322e-45}, {1.1309962886447716e-31, 1.0498015412959506e-47}
#define MOSAIC_CRM_COS_C                                                                                  \
    {1.0, 0.0}, {-0.5, 0.0}, {0.041666666666666664, 2.3129646346357427e-18},                                    \
        {-0.001388888888888889, 5.300543954373577e-20}, {2.48015873015873e-05, 2.1511947866775882e-23},       \
        {-2.755731922398589e-07, -2.3767714622250297e-23}, {2.08767569878681e-09, -1.20734505911326e-25},      \
        {-1.1470745597729725e-11, -2.0655512752830745e-28}, {4.779477332387385e-14, 4.399205485834081e-31},    \
        {-1.5619206968586225e-16, -1.1910679660273754e-32}, {4.110317623312165e-19, 1.4412973378659527e-36},   \
        {-8.896791392450574e-22, 7.911402614872376e-38}, {1.6117375710961184e-24, -3.6846573564509766e-41},    \
        {-2.4795962632247976e-27, 1.2953730964765229e-43}, {3.279889237069838e-30, 1.5117542744029879e-46}

// sin and cos of x (|x| < 1e5) as double-double
MOSAIC_HD void sincos_dd(double x, dd* s, dd* c) {
    const dd SC[15] = {MOSAIC_CRM_SIN_C};
    const dd CC[15] = {MOSAIC_CRM_COS_C};
    const double P1 = 1.5707963267948966, P2 = 6.123233995736766e-17, P3 = -1.4973849048591698e-33;
    double kf = rint(x * 0.6366197723675814);
    dd r = add(dd{x, 0.0}, neg(two_prod(kf, P1)));
    r = add(r, neg(two_prod(kf, P2)));
    r = add(r, dd{-kf * P3, 0.0});
    dd z = mul(r, r);
    dd ps = SC[14], pc = CC[14];
    for (int k = 13; k >= 0; k--) {
        ps = add(mul(ps, z), SC[k]);
        pc = add(mul(pc, z), CC[k]);
    }
    ps = mul(ps, r);
    int q = ((int)kf) & 3;
    dd so = q == 0 ? ps : (q == 1 ? pc : (q == 2 ? neg(ps) : neg(pc)));
    dd co = q == 0 ? pc : (q == 1 ? neg(ps) : (q == 2 ? neg(pc) : ps));
    *s = so;
    *c = co;
}

MOSAIC_HD double sin_cr(double x) {
    if (!(fabs(x) < 1e5)) return sin(x);
    if (x == 0.0) return x;
    dd s, c;
    sincos_dd(x, &s, &c);
    return round_dd(s);
}
MOSAIC_HD double cos_cr(double x) {
    if (!(fabs(x) < 1e5)) return cos(x);
    dd s, c;
    sincos_dd(x, &s, &c);
    return round_dd(c);
}
MOSAIC_HD double tan_cr(double x) {
    if (!(fabs(x) < 1e5)) return tan(x);
    if (x == 0.0) return x;
    dd s, c;
    sincos_dd(x, &s, &c);
    return round_dd(div(s, c));
}

// asin of a double-double v, |v| <= 0.71: one Newton step on sin(psi) = v from the library value
MOSAIC_HD dd asin_dd(dd v) {
    double p0 = asin(v.hi);
    dd s, c;
    sincos_dd(p0, &s, &c);
    return add(dd{p0, 0.0}, div(add(v, neg(s)), c));
}

MOSAIC_HD double acos_cr(double x) {
    if (!(fabs(x) <= 1.0)) return acos(x);
    if (x == 1.0) return 0.0;
    const dd PI = {3.141592653589793, 1.2246467991473532e-16};
    const dd PIO2 = {1.5707963267948966, 6.123233995736766e-17};
    if (fabs(x) >= 0.5) {
        // acos(x) = 2 asin(sqrt((1 - x) / 2)) (x >= 1/2), pi - 2 asin(sqrt((1 + x) / 2)) (x <= -1/2);
        // 1 -+ x is exact here (Sterbenz) and so is the halving
        double a = (x > 0 ? 1.0 - x : 1.0 + x) * 0.5;
        double s0 = sqrt(a);
        dd v = quick_two_sum(s0, fma(-s0, s0, a) / (2.0 * s0));
        dd t = asin_dd(v);
        t = dd{2.0 * t.hi, 2.0 * t.lo};
        return round_dd(x > 0 ? t : add(PI, neg(t)));
    }
    return round_dd(add(PIO2, neg(asin_dd(dd{x, 0.0}))));
}

MOSAIC_HD double atan2_cr(double y, double x) {
    if (x == 0.0 || y == 0.0 || !isfinite(x) || !isfinite(y)) return atan2(y, x);
    double t0 = atan2(y, x);
    dd s, c;
    sincos_dd(t0, &s, &c);
    dd num = add(mul_d(c, y), neg(mul_d(s, x)));
    dd den = add(mul_d(c, x), mul_d(s, y));
    return round_dd(add(dd{t0, 0.0}, div(num, den)));
}

}  // namespace crm
}  // namespace mosaic
