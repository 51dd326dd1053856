// Exact emulation of the x86-64 `long double` (x87 double-extended, 64-bit significand) operations
// that H3 v3.7 performs where it uses L-suffixed constants: double (op) LDconst, rounded to the
// 64-bit significand (round-to-nearest-even), then rounded again to double on assignment.
//
// Integer-only (unsigned __int128), so device and host give identical bits.  Used only by the
// exact ("slow") H3 path, which runs for the rare points whose cell the fast projective path cannot
// decide with certainty (h3_device.h).  Operands are finite normal doubles in the ranges H3 uses.
#pragma once
#include <stdint.h>

#include "h3_ld_constants.h"

#if defined(__HIPCC__)
#define MOSAIC_HD __host__ __device__ inline
#else
#define MOSAIC_HD inline
#endif

namespace mosaic {
namespace x87 {

typedef unsigned __int128 u128;

struct Ext {  // value = (neg ? -1 : 1) * m * 2^e, m has bit 63 set (or m == 0 for zero)
    uint64_t m;
    int e;
    bool neg;
};

MOSAIC_HD int clz64(uint64_t x) { return x ? __builtin_clzll(x) : 64; }
MOSAIC_HD int clz128(u128 x) {
    uint64_t hi = (uint64_t)(x >> 64);
    return hi ? clz64(hi) : 64 + clz64((uint64_t)x);
}

MOSAIC_HD Ext from_double(double d) {
    Ext r;
    union {
        double d;
        uint64_t u;
    } c;
    c.d = d;
    r.neg = (c.u >> 63) != 0;
    int be = (int)((c.u >> 52) & 0x7ff);
    uint64_t frac = c.u & 0xfffffffffffffULL;
    if (be == 0 && frac == 0) {
        r.m = 0;
        r.e = 0;
        return r;
    }
    uint64_t m53 = be ? (frac | (1ULL << 52)) : frac;
    int e = (be ? be : 1) - 1075;  // value = m53 * 2^e
    int s = clz64(m53);
    r.m = m53 << s;
    r.e = e - s;
    return r;
}

// Round a 128-bit magnitude (value = x * 2^e) to 64 significant bits (RNE); sticky folded in LSB.
MOSAIC_HD Ext round64(u128 x, int e, bool neg) {
    Ext r;
    r.neg = neg;
    if (x == 0) {
        r.m = 0;
        r.e = 0;
        return r;
    }
    int lz = clz128(x);
    x <<= lz;  // bit 127 set
    e -= lz;
    uint64_t hi = (uint64_t)(x >> 64);
    uint64_t lo = (uint64_t)x;
    const uint64_t half = 1ULL << 63;
    if (lo > half || (lo == half && (hi & 1))) {
        hi += 1;
        if (hi == 0) {
            hi = 1ULL << 63;
            e += 1;
        }
    }
    r.m = hi;
    r.e = e + 64;
    return r;
}

// Round an Ext to double (RNE): the implicit conversion on assignment to a `double`.
MOSAIC_HD double to_double(Ext v) {
    if (v.m == 0) return v.neg ? -0.0 : 0.0;
    uint64_t m = v.m >> 11;
    uint64_t rem = v.m & 0x7ff;
    int e = v.e + 11;
    if (rem > 0x400 || (rem == 0x400 && (m & 1))) {
        m += 1;
        if (m == (1ULL << 53)) {
            m >>= 1;
            e += 1;
        }
    }
    // m < 2^53, exact scaling (results stay normal in H3's ranges)
    double d = (double)m;
    // multiply by 2^e exactly
    union {
        double d;
        uint64_t u;
    } c;
    c.u = (uint64_t)(e + 1023) << 52;  // 2^e for -1022 <= e <= 1023
    double r = d * c.d;
    return v.neg ? -r : r;
}

MOSAIC_HD Ext add(Ext a, Ext b) {  // exact a + b rounded to 64 bits
    if (a.m == 0) return b;
    if (b.m == 0) return a;
    if (a.e < b.e || (a.e == b.e && a.m < b.m)) {
        Ext t = a;
        a = b;
        b = t;
    }
    // |a| >= |b|; put significands in the top of 128-bit fields
    u128 xa = (u128)a.m << 63;  // leave one bit of headroom for carries
    int d = a.e - b.e;
    u128 xb;
    if (d >= 127) {
        xb = 1;  // pure sticky
    } else {
        u128 full = (u128)b.m << 63;
        xb = full >> d;
        if ((xb << d) != full) xb |= 1;  // sticky
    }
    int e = a.e - 63;
    if (a.neg == b.neg) return round64(xa + xb, e, a.neg);
    return round64(xa - xb, e, a.neg);
}

MOSAIC_HD Ext mul(Ext a, Ext b) {
    u128 p = (u128)a.m * (u128)b.m;
    return round64(p, a.e + b.e, a.neg != b.neg);
}

MOSAIC_HD Ext div(Ext a, Ext b) {  // a / b, b != 0
    if (a.m == 0) return a;
    // long division producing 128 quotient bits of a.m / b.m, plus a sticky bit
    u128 r = a.m;
    u128 q = 0;
    if (r >= b.m) {  // both normalized to bit 63: at most one subtraction
        q = 1;
        r -= b.m;
    }
    for (int i = 0; i < 126; i++) {
        r <<= 1;
        q <<= 1;
        if (r >= b.m) {
            r -= b.m;
            q |= 1;
        }
    }
    if (r) q |= 1;
    // value = q * 2^(a.e - b.e - 126)
    return round64(q, a.e - b.e - 126, a.neg != b.neg);
}

MOSAIC_HD Ext make(uint64_t m, int e, bool neg = false) {
    Ext r;
    r.m = m;
    r.e = e;
    r.neg = neg;
    return r;
}

// double (op) long-double-constant, evaluated in x87 precision and assigned back to double
MOSAIC_HD double add_ld(double a, uint64_t cm, int ce, bool cneg) {
    return to_double(add(from_double(a), make(cm, ce, cneg)));
}
MOSAIC_HD double mul_ld(double a, uint64_t cm, int ce) { return to_double(mul(from_double(a), make(cm, ce))); }
MOSAIC_HD double div_ld(double a, uint64_t cm, int ce) { return to_double(div(from_double(a), make(cm, ce))); }

}  // namespace x87
}  // namespace mosaic
