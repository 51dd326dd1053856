// Point geometry column -> coordinates, for grid_pointascellid over a geometry column
// (PointIndexGeom.nullSafeEval, PointIndexGeom.scala:32-40: GeometryAPI.geometry(input, dataType)
// GeometryAPI.scala:64-72 -> MosaicGeometryJTS.fromWKB / fromWKT / fromHEX (MosaicGeometryJTS.scala:
// 164, 195-198, 200) -> getCentroid (:49-53) -> getX / getY, MosaicPointJTS.scala:23-25).  The
// centroid of a non-empty Point is the point itself (JTS Centroid: one point, sum / 1), so a row
// decodes to its first two ordinates.  Device and host (tests) code.
//
// Contract: a row decodes (kOk) only when JTS 1.19 [3P] certainly reads it as a non-empty Point
// with exactly these x / y.  Every other row -- another geometry type (whose centroid the
// reference computes), POINT EMPTY (getX throws), malformed input (ParseException), grammar this
// decoder does not follow -- is reported as "row path" and left to the reference's own row-wise
// evaluation, so being stricter than JTS never changes a result.
//
// WKB (JTS WKBReader, non-strict): byte order byte 1 = little endian, anything else big endian;
// type word: (t & 0xffff) % 1000 is the geometry type, Z if bit 31 or (t & 0xffff) / 1000 in {1, 3},
// M if bit 30 or / 1000 in {2, 3}, SRID (4 bytes) if bit 29; x, y, then any z / m.  A Point with x or
// y NaN reads as the empty point.  Bytes after the point are ignored, as by WKBReader.
// HEX (WKBReader.hexToBytes): pairs of hex digits (either case), a trailing odd digit ignored.
// WKT (JTS WKTReader over java.io.StreamTokenizer: whitespace = bytes 0..32, words = runs of
// [A-Za-z0-9+-.] and bytes >= 160): "POINT[Z|M|ZM] [Z|M|ZM] ( x y [z] [m] )" with the keywords in
// any case; ordinates: x y (+ one more, the old JTS syntax) without a modifier, x y z / x y m /
// x y z m with one; a number is "NaN" (any case, JTS) or what Double.parseDouble accepts in
// decimal form ([+-] digits [. digits] [(e|E) [+-] digits] [f F d D], [+-] "Infinity" / "NaN").
// Decimal strings are converted with correct rounding (ties to even) like Double.parseDouble:
// Clinger's exact fast path where it applies, else an approximation corrected against exact
// big-integer comparisons with the neighbouring halfway points (Clinger's algorithm R).  Digits
// beyond the first kMaxDigits only set a sticky bit: a halfway point between doubles has at most
// 767 significant digits, so comparing 800 digits plus the sticky bit is exact for any length.
// Row path instead: hexadecimal literals, '#' comments, rows longer than kMaxText bytes.
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#if !defined(MOSAIC_HD)
#if defined(__HIPCC__)
#define MOSAIC_HD __host__ __device__ inline
#else
#define MOSAIC_HD inline
#endif
#endif

namespace mosaic {
namespace decode {

enum : int {
    kOk = 0,
    kBadWkb = 1,     // truncated WKB, unknown type, bad hex digit
    kBadWkt = 2,     // not the POINT grammar above, or a malformed number
    kNotPoint = 3,   // a geometry type other than Point
    kEmpty = 4,      // POINT EMPTY (getX on an empty point throws)
    kTooLong = 5,    // beyond kMaxText bytes
};
enum : int { kFormatWkb = 0, kFormatWkt = 1, kFormatHex = 2 };
static const int kMaxDigits = 800;
static const int64_t kMaxText = 4096;

// ---- exact decimal -> double ----
// Unsigned big integer, 32-bit limbs, little endian; large enough for the comparisons below
// (< 2800 bits for kMaxDigits digits and values within the double range).
static const int kLimbs = 100;
struct Big {
    uint32_t w[kLimbs];
    int n;  // limbs in use (w[n..] are zero)
};
MOSAIC_HD void big_set(Big& b, uint64_t v) {
    for (int k = 0; k < kLimbs; k++) b.w[k] = 0;
    b.w[0] = (uint32_t)v;
    b.w[1] = (uint32_t)(v >> 32);
    b.n = b.w[1] ? 2 : (b.w[0] ? 1 : 0);
}
// b = b * m + add; false on overflow
MOSAIC_HD bool big_muladd(Big& b, uint32_t m, uint32_t add) {
    uint64_t carry = add;
    for (int k = 0; k < b.n; k++) {
        const uint64_t t = (uint64_t)b.w[k] * m + carry;
        b.w[k] = (uint32_t)t;
        carry = t >> 32;
    }
    if (carry) {
        if (b.n >= kLimbs) return false;
        b.w[b.n++] = (uint32_t)carry;
    }
    return true;
}
MOSAIC_HD bool big_mul_pow5(Big& b, int e) {
    while (e >= 13) {
        if (!big_muladd(b, 1220703125u, 0)) return false;  // 5^13
        e -= 13;
    }
    uint32_t m = 1;
    for (int k = 0; k < e; k++) m *= 5u;
    return big_muladd(b, m, 0);
}
MOSAIC_HD bool big_shl(Big& b, int s) {
    if (b.n == 0 || s == 0) return true;
    const int ls = s >> 5, bs = s & 31;
    if (b.n + ls + 1 > kLimbs) return false;
    for (int k = b.n - 1 + ls + 1; k >= 0; k--) {
        const int src = k - ls;
        uint32_t hi = (src >= 0 && src < b.n) ? b.w[src] : 0u;
        uint32_t lo = (src - 1 >= 0 && src - 1 < b.n) ? b.w[src - 1] : 0u;
        b.w[k] = bs ? ((hi << bs) | (lo >> (32 - bs))) : hi;
    }
    b.n = b.n + ls + 1;
    while (b.n > 0 && b.w[b.n - 1] == 0) b.n--;
    return true;
}
MOSAIC_HD int big_cmp(const Big& a, const Big& b) {
    if (a.n != b.n) return a.n < b.n ? -1 : 1;
    for (int k = a.n - 1; k >= 0; k--)
        if (a.w[k] != b.w[k]) return a.w[k] < b.w[k] ? -1 : 1;
    return 0;
}

// sign of (D + sticky) * 10^q - A * 2^f (D given by its digit string, sticky: nonzero digits
// follow), or 2 if a big integer overflowed
MOSAIC_HD int cmp_decimal(const char* digits, int nd, bool sticky, int q, uint64_t A, int f) {
    Big L, R;
    big_set(L, 0);
    for (int k = 0; k < nd; k++)
        if (!big_muladd(L, 10u, (uint32_t)(digits[k] - '0'))) return 2;
    big_set(R, A);
    // D 5^q 2^q vs A 2^f  (q >= 0)   or   D vs A 5^-q 2^(f - q)  (q < 0)
    int e2l = 0, e2r = f;
    if (q >= 0) {
        if (!big_mul_pow5(L, q)) return 2;
        e2l = q;
    } else {
        if (!big_mul_pow5(R, -q)) return 2;
        e2r = f - q;
    }
    if (e2l >= e2r) {
        if (!big_shl(L, e2l - e2r)) return 2;
    } else {
        if (!big_shl(R, e2r - e2l)) return 2;
    }
    const int c = big_cmp(L, R);
    return (c == 0 && sticky) ? 1 : c;
}

MOSAIC_HD double pow10_exact(int k) {  // 10^k for 0 <= k <= 22: exact doubles
    double p = 1.0;
    for (int i = 0; i < k; i++) p *= 10.0;
    return p;
}

// Correctly rounded value of D * 10^q, D = the significant digits d[0..nd) (first and last
// nonzero, nd <= kMaxDigits) followed by nonzero digits if sticky; false if the comparisons
// overflowed (not expected within the limits).
MOSAIC_HD bool decimal_round(const char* d, int nd, bool sticky, int q, double z, double* out) {
    if (!(z > 0.0)) z = 4.9406564584124654e-324;
    if (isinf(z)) z = 1.7976931348623157e308;
    for (int it = 0; it < 64; it++) {
        // z = m 2^e, m < 2^53, e >= -1074
        int e;
        double fr = frexp(z, &e);  // z = fr 2^e, fr in [0.5, 1)
        uint64_t m;
        if (e - 53 >= -1074) {
            m = (uint64_t)ldexp(fr, 53);
            e -= 53;
        } else {
            m = (uint64_t)ldexp(z, 1074);
            e = -1074;
        }
        // upper halfway (2m + 1) 2^(e - 1)
        const int cu = cmp_decimal(d, nd, sticky, q, 2 * m + 1, e - 1);
        if (cu == 2) return false;
        if (cu > 0 || (cu == 0 && (m & 1u))) {
            const double nz = nextafter(z, INFINITY);
            if (cu == 0 || isinf(nz)) {
                *out = nz;  // tie to the even neighbour, or overflow
                return true;
            }
            z = nz;
            continue;
        }
        if (cu == 0) {  // tie, m even
            *out = z;
            return true;
        }
        // lower halfway: (2m - 1) 2^(e - 1), or (4m - 1) 2^(e - 2) at a binade boundary
        const bool boundary = m == ((uint64_t)1 << 52) && e > -1074;
        const int cl = boundary ? cmp_decimal(d, nd, sticky, q, 4 * m - 1, e - 2)
                                : cmp_decimal(d, nd, sticky, q, 2 * m - 1, e - 1);
        if (cl == 2) return false;
        if (cl < 0 || (cl == 0 && (m & 1u))) {
            const double pz = nextafter(z, 0.0);
            if (cl == 0 || pz == 0.0) {
                *out = pz;
                return true;
            }
            z = pz;
            continue;
        }
        *out = z;
        return true;
    }
    return false;
}

MOSAIC_HD bool is_space(uint8_t c) { return c <= 32; }  // StreamTokenizer.whitespaceChars(0, ' ')
MOSAIC_HD bool is_word(uint8_t c) {
    return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '+' || c == '-' || c == '.' ||
           c >= 160;
}
MOSAIC_HD uint8_t lower(uint8_t c) { return (c >= 'A' && c <= 'Z') ? (uint8_t)(c + 32) : c; }

// w 10^q (w < 10^19 exact, |q| <= 22) correctly rounded when a double-double evaluation decides
// it: the product / quotient of the exact double-double w and the exact double 10^|q| carries a
// relative error below 2^-100, so S + E (S = round(S + E)) rounds like the exact value unless the
// exact value may lie beyond a midpoint next to S.  false: undecided (take the big-integer path).
MOSAIC_HD bool dd_round(uint64_t w, int q, double* out) {
    const double hi = (double)w;
    const double lo = (double)(int64_t)(w - (uint64_t)hi);  // exact: |w - hi| <= 2^10
    const double p = pow10_exact(q >= 0 ? q : -q);
    double S, E;
    if (q >= 0) {
        const double ph = hi * p;
        const double pl = fma(lo, p, fma(hi, p, -ph));
        S = ph + pl;
        E = pl - (S - ph);
    } else {
        const double q1 = hi / p;
        const double r = fma(-q1, p, hi) + lo;
        const double q2 = r / p;
        S = q1 + q2;
        E = q2 - (S - q1);
    }
    if (!(S > 0.0) || isinf(S)) return false;
    int ex;
    frexp(S, &ex);                            // S in [2^(ex-1), 2^ex)
    const double ulp = ldexp(1.0, ex - 53);   // normal range only (|q| <= 22)
    const double tol = ldexp(S, -98);         // >> the evaluation error
    const bool pow2 = S == ldexp(1.0, ex - 1);
    const double half = (pow2 && E < 0.0) ? 0.25 * ulp : 0.5 * ulp;
    if (fabs(E) + tol >= half) return false;
    *out = S;
    return true;
}

// Number token s[p..e) (Double.parseDouble's decimal grammar, JTS's NaN) -> *out
MOSAIC_HD int parse_number(const uint8_t* s, int64_t p, int64_t e, double* out) {
    bool neg = false, sign = false;
    if (p < e && (s[p] == '+' || s[p] == '-')) {
        neg = s[p] == '-';
        sign = true;
        p++;
    }
    // JTS: the whole token equalsIgnoreCase("NaN"); Double.parseDouble: [+-]"NaN" exactly
    if (e - p == 3 && (sign ? (s[p] == 'N' && s[p + 1] == 'a' && s[p + 2] == 'N')
                            : (lower(s[p]) == 'n' && lower(s[p + 1]) == 'a' && lower(s[p + 2]) == 'n'))) {
        *out = NAN;
        return kOk;
    }
    if (e - p == 8) {
        const char* inf = "Infinity";
        bool ok = true;
        for (int k = 0; k < 8; k++) ok = ok && s[p + k] == (uint8_t)inf[k];
        if (ok) {
            *out = neg ? -INFINITY : INFINITY;
            return kOk;
        }
    }
    if (e > p && (s[e - 1] == 'd' || s[e - 1] == 'D' || s[e - 1] == 'f' || s[e - 1] == 'F')) e--;
    // pass 1: digits d1..dn from the first to the last nonzero digit, value = D 10^(E - n + exp)
    // with E the position of d1 relative to the point; w = the first min(n, 19) digits
    const int64_t m0 = p;
    int64_t nsig = 0, n = 0, E = 0, nmant = 0;
    uint64_t w = 0, w_at_n = 0;
    bool dot = false, seen = false;
    for (; p < e; p++) {
        const uint8_t c = s[p];
        if (c == '.') {
            if (dot) return kBadWkt;
            dot = true;
            continue;
        }
        if (c < '0' || c > '9') break;
        nmant++;
        if (!seen) {
            if (c == '0') {
                if (dot) E--;
                continue;
            }
            seen = true;
        }
        if (!dot) E++;
        nsig++;
        if (nsig <= 19) w = w * 10u + (uint64_t)(c - '0');
        if (c != '0') {
            n = nsig;
            w_at_n = w;
        }
    }
    if (nmant == 0) return kBadWkt;
    const int64_t m1 = p;
    int64_t ex = 0;
    if (p < e) {
        if (s[p] != 'e' && s[p] != 'E') return kBadWkt;
        p++;
        bool eneg = false;
        if (p < e && (s[p] == '+' || s[p] == '-')) {
            eneg = s[p] == '-';
            p++;
        }
        if (p >= e) return kBadWkt;
        for (; p < e; p++) {
            if (s[p] < '0' || s[p] > '9') return kBadWkt;
            if (ex < 100000) ex = ex * 10 + (s[p] - '0');
        }
        if (eneg) ex = -ex;
    }
    if (n == 0) {
        *out = neg ? -0.0 : 0.0;
        return kOk;
    }
    const int64_t mag = E + ex;  // value in [10^(mag - 1), 10^mag)
    double v;
    if (mag > 310) {
        v = INFINITY;
    } else if (mag < -324) {  // below 1e-325 < 2^-1075: rounds to zero
        v = 0.0;
    } else {
        const int q = (int)(mag - n);  // value = D 10^q
        if (n <= 19) w = w_at_n;  // else w holds the first 19 digits
        if (n <= 15 && q >= -22 && q <= 22) {
            // Clinger's fast path: w and 10^|q| exact doubles, one correctly rounded operation
            v = q >= 0 ? (double)w * pow10_exact(q) : (double)w / pow10_exact(-q);
        } else if (!(n <= 19 && q >= -22 && q <= 22 && dd_round(w, q, &v))) {
            // approximation (a few ulps off), then exact correction on the digit string
            int qa = q + (int)(n > 19 ? n - 19 : 0);
            double z = (double)w;
            while (qa > 22) {
                z *= 1e22;
                qa -= 22;
            }
            while (qa < -22) {
                z /= 1e22;
                qa += 22;
            }
            z = qa >= 0 ? z * pow10_exact(qa) : z / pow10_exact(-qa);
            char dig[kMaxDigits];
            int nd = 0;
            bool sticky = false;
            bool started = false;
            for (int64_t k = m0; k < m1; k++) {
                const uint8_t c = s[k];
                if (c == '.') continue;
                if (!started && c == '0') continue;
                started = true;
                if (nd < kMaxDigits && nd < n) dig[nd++] = (char)c;
                else if (c != '0') sticky = true;
            }
            const int qd = q + (int)(n - nd);
            if (!decimal_round(dig, nd, sticky, qd, z, &v)) return kTooLong;
        }
    }
    *out = neg ? -v : v;
    return kOk;
}

// Ordinate modifier word s[w..w+l): 0 none, 1 Z, 2 M, 3 ZM, -1 other
MOSAIC_HD int ord_modifier(const uint8_t* s, int64_t w, int64_t l) {
    if (l == 1 && lower(s[w]) == 'z') return 1;
    if (l == 1 && lower(s[w]) == 'm') return 2;
    if (l == 2 && lower(s[w]) == 'z' && lower(s[w + 1]) == 'm') return 3;
    return -1;
}
MOSAIC_HD bool word_is(const uint8_t* s, int64_t w, int64_t l, const char* lit, int n) {
    if (l != n) return false;
    for (int k = 0; k < n; k++)
        if (lower(s[w + k]) != (uint8_t)lit[k]) return false;
    return true;
}
// next token: a word [t0, t1) or one ordinary character (t1 = t0 + 1); false at the end
MOSAIC_HD bool next_token(const uint8_t* s, int64_t len, int64_t& p, int64_t& t0, int64_t& t1) {
    while (p < len && is_space(s[p])) p++;
    if (p >= len) return false;
    t0 = p;
    if (is_word(s[p])) {
        while (p < len && is_word(s[p])) p++;
    } else {
        p++;
    }
    t1 = p;
    return true;
}

// One WKT row s[0..len) -> (x, y) (WKTReader.readGeometryTaggedText -> readPointText -> getCoordinate)
MOSAIC_HD int wkt_point(const uint8_t* s, int64_t len, double* x, double* y) {
    if (len > kMaxText) return kTooLong;
    int64_t p = 0, t0, t1;
    if (!next_token(s, len, p, t0, t1) || !is_word(s[t0])) return kBadWkt;
    // geometry keyword with an optional modifier suffix (POINTZ, pointzm, ...)
    int64_t kl = t1 - t0;
    if (kl < 5 || !word_is(s, t0, 5, "point", 5)) {
        // another geometry type (or none): JTS reads it, or throws, on the row path
        return kNotPoint;
    }
    int mods = 0;
    if (kl > 5) {
        mods = ord_modifier(s, t0 + 5, kl - 5);
        if (mods < 0) return kBadWkt;
    }
    if (!next_token(s, len, p, t0, t1)) return kBadWkt;
    // getNextOrdinateFlags (only without a suffix), then getNextEmptyOrOpener's own Z / M / ZM
    if (mods == 0 && is_word(s[t0])) {
        const int m = ord_modifier(s, t0, t1 - t0);
        if (m > 0) {
            mods = m;
            if (!next_token(s, len, p, t0, t1)) return kBadWkt;
        }
    }
    if (is_word(s[t0]) && ord_modifier(s, t0, t1 - t0) > 0) {
        if (!next_token(s, len, p, t0, t1)) return kBadWkt;
    }
    if (is_word(s[t0]) && word_is(s, t0, t1 - t0, "empty", 5)) return kEmpty;
    if (s[t0] != '(' ) return kBadWkt;
    // ordinates: x y, z if Z, m if M; without modifiers one optional extra number (old syntax)
    const int need = 2 + ((mods & 1) ? 1 : 0) + ((mods & 2) ? 1 : 0);
    double ord[4];
    int got = 0;
    while (true) {
        if (!next_token(s, len, p, t0, t1)) return kBadWkt;
        if (!is_word(s[t0])) break;
        if (got == need + (mods == 0 ? 1 : 0)) return kBadWkt;
        const int rc = parse_number(s, t0, t1, &ord[got]);
        if (rc != kOk) return rc;
        got++;
    }
    if (s[t0] != ')' || got < need) return kBadWkt;
    // JTS ignores what follows the geometry; the row path is taken for anything but whitespace
    if (next_token(s, len, p, t0, t1)) return kBadWkt;
    *x = ord[0];
    *y = ord[1];
    return kOk;
}

MOSAIC_HD uint32_t rd_u32(const uint8_t* b, bool le) {
    return le ? ((uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24))
              : ((uint32_t)b[3] | ((uint32_t)b[2] << 8) | ((uint32_t)b[1] << 16) | ((uint32_t)b[0] << 24));
}
MOSAIC_HD double rd_f64(const uint8_t* b, bool le) {
    uint64_t v = 0;
    for (int k = 0; k < 8; k++) v |= (uint64_t)b[le ? k : 7 - k] << (8 * k);
    double d;
    memcpy(&d, &v, 8);
    return d;
}

// One WKB row b[0..len) -> (x, y) (WKBReader.readGeometry -> readPoint)
MOSAIC_HD int wkb_point(const uint8_t* b, int64_t len, double* x, double* y) {
    if (len < 5) return kBadWkb;
    const bool le = b[0] == 1;  // non-strict reader: any other byte keeps big endian
    const uint32_t t = rd_u32(b + 1, le);
    int64_t p = 5;
    if (t & 0x20000000u) p += 4;  // EWKB SRID
    const uint32_t base = t & 0xffffu;
    const uint32_t kind = base % 1000u, iso = base / 1000u;
    if (kind != 1) return (kind >= 2 && kind <= 7) ? kNotPoint : kBadWkb;
    const int nord = 2 + (((t & 0x80000000u) || iso == 1 || iso == 3) ? 1 : 0) +
                     (((t & 0x40000000u) || iso == 2 || iso == 3) ? 1 : 0);
    if (len < p + 8 * nord) return kBadWkb;
    const double px = rd_f64(b + p, le), py = rd_f64(b + p + 8, le);
    if (isnan(px) || isnan(py)) return kEmpty;  // readPoint: NaN x or y -> createPoint()
    *x = px;
    *y = py;
    return kOk;
}

MOSAIC_HD int hex_digit(uint8_t c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}
// One hex-WKB row (WKBReader.hexToBytes: every pair must be hex digits) -> (x, y)
MOSAIC_HD int hex_point(const uint8_t* s, int64_t len, double* x, double* y) {
    if (len > kMaxText) return kTooLong;
    const int64_t nb = len / 2;
    uint8_t buf[48];
    const int64_t keep = nb < 48 ? nb : 48;  // a Point needs at most 1 + 4 + 4 + 32 = 41 bytes
    for (int64_t k = 0; k < nb; k++) {
        const int hi = hex_digit(s[2 * k]), lo = hex_digit(s[2 * k + 1]);
        if (hi < 0 || lo < 0) return kBadWkb;
        if (k < keep) buf[k] = (uint8_t)(hi * 16 + lo);
    }
    return wkb_point(buf, keep, x, y);
}

MOSAIC_HD int decode_row(int format, const uint8_t* s, int64_t len, double* x, double* y) {
    if (format == kFormatWkb) return wkb_point(s, len, x, y);
    if (format == kFormatWkt) return wkt_point(s, len, x, y);
    return hex_point(s, len, x, y);
}

}  // namespace decode
}  // namespace mosaic
