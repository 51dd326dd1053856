// BNG (British National Grid) point -> cell id for gfx950 and the host.
// Restates reference src/main/scala/com/databricks/labs/mosaic/core/index/BNGIndexSystem.scala
//   pointToIndex :277-291, getQuadrant :309-327, encode :528-541
// with JVM semantics (Double.toInt / toLong truncate and saturate, Int `/` and `%` truncate toward
// zero, Int `*` wraps, math.pow(10, n) exact).  Every operation is an exactly specified IEEE or
// integer operation, so the device result is bit-identical to the JVM's.
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
namespace bng {

MOSAIC_HD int32_t jvm_d2i(double d) {
#if defined(__HIP_DEVICE_COMPILE__)
    // v_cvt_i32_f64 is Double.toInt: truncation toward zero, NaN -> 0, saturation at Int bounds
    int32_t r;
    __asm__("v_cvt_i32_f64 %0, %1" : "=v"(r) : "v"(d));
    return r;
#else
    if (d != d) return 0;
    if (d >= 2147483647.0) return 2147483647;
    if (d <= -2147483648.0) return (-2147483647 - 1);
    return (int32_t)d;
#endif
}
MOSAIC_HD int64_t jvm_d2l(double d) {
    if (d != d) return 0;
    if (d >= 9223372036854775807.0) return INT64_MAX;
    if (d <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)d;
}
MOSAIC_HD double pow10i(int n) {
    double r = 1.0;
    // exact for 0 <= n <= 22 (every intermediate is an exactly representable power of ten)
    for (int i = 0; i < n; i++) r *= 10.0;
    return r;
}
MOSAIC_HD bool valid_resolution(int res) { return res != 0 && res >= -6 && res <= 6; }

// Returns false for NaN input (the reference throws IllegalStateException).
MOSAIC_HD bool point_to_index(double eastings, double northings, int res, int64_t* out) {
    if (eastings != eastings || northings != northings) return false;
    int32_t eI = jvm_d2i(eastings);
    int32_t nI = jvm_d2i(northings);
    int32_t eLetter = jvm_d2i(floor((double)(eI / 100000)));
    int32_t nLetter = jvm_d2i(floor((double)(nI / 100000)));
    int ares = res < 0 ? -res : res;
    double divisor = res < 0 ? pow10i(6 - ares + 1) : pow10i(6 - res);
    int32_t quadrant = 0;
    if (res < -1) {
        double eQ = (double)eI / divisor;
        double nQ = (double)nI / divisor;
        double eD = eQ - floor(eQ);
        double nD = nQ - floor(nQ);
        if (eD < 0.5 && nD < 0.5)
            quadrant = 1;
        else if (eD < 0.5)
            quadrant = 2;
        else if (nD < 0.5)
            quadrant = 4;
        else
            quadrant = 3;
    }
    int32_t nPositions = res >= -1 ? ares : ares - 1;
    int32_t eBin = jvm_d2i(floor((double)(eI % 100000) / divisor));
    int32_t nBin = jvm_d2i(floor((double)(nI % 100000) / divisor));
    double idPlaceholder = pow10i(5 + 2 * nPositions - 2);
    double eLetterShift = pow10i(3 + 2 * nPositions - 2);
    double nLetterShift = pow10i(1 + 2 * nPositions - 2);
    double eShift = pow10i(nPositions);
    double id;
    if (res == -1) {
        id = (idPlaceholder + (double)eLetter * eLetterShift) / 100 + (double)quadrant;
    } else {
        int32_t nb10 = (int32_t)((uint32_t)nBin * 10u);
        id = idPlaceholder + (double)eLetter * eLetterShift + (double)nLetter * nLetterShift + (double)eBin * eShift +
             (double)nb10 + (double)quadrant;
    }
    *out = jvm_d2l(id);
    return true;
}


// ---- BNGIndexSystem.parse (BNGIndexSystem.scala:391-413) + encode (:528-541): a string id (the
// StringType cell ids BNG chips carry by default, BNGIndexSystem.scala:28) -> the long id.
// letterMap (:84-99, row 10 repeats "SZ": find() takes the first row, row 0) and quadrants (:36).
MOSAIC_HD int letter_code(char a, char b) {
    // letterMap as a table of the two characters; returns row * 8 + column of the first match
    const char* rows = "SVSWSXSYSZTVTW" "SQSRSSSTSUTQTR" "SLSMSNSOSPTLTM" "SFSGSHSJSKTFTG" "SASBSCSDSETATB"
                       "NVNWNXNYNZOVOW" "NQNRNSNTNUOQOR" "NLNMNNNONPOLOM" "NFNGNHNJNKOFOG" "NANBNCNDNEOAOB"
                       "HVHWHXHYSZJVJW" "HQHRHSHTHUJQJR" "HLHMHNHOHPJLJM";
    for (int r = 0; r < 13; r++)
        for (int c = 0; c < 7; c++)
            if (rows[r * 14 + 2 * c] == a && rows[r * 14 + 2 * c + 1] == b) return r * 8 + c;
    return -1;
}
// Integer.parseInt over s[0 .. n): optional sign, then at least one ASCII digit, within Int range
// (Java also accepts non-ASCII Unicode digits, which this does not: such ids are rejected)
MOSAIC_HD bool java_parse_int(const char* s, int n, int32_t* out) {
    if (n <= 0) return false;
    int i = 0;
    bool neg = false;
    if (s[0] == '-' || s[0] == '+') {
        neg = s[0] == '-';
        i = 1;
        if (n == 1) return false;
    }
    int64_t v = 0;
    for (; i < n; i++) {
        if (s[i] < '0' || s[i] > '9') return false;
        v = v * 10 + (s[i] - '0');
        if (v > 2147483648LL) return false;
    }
    if (!neg && v > 2147483647LL) return false;
    *out = (int32_t)(neg ? -v : v);
    return true;
}
MOSAIC_HD int64_t encode(int eLetter, int nLetter, int32_t eBin, int32_t nBin, int quadrant, int nPositions, int res) {
    const double idP = pow10i(5 + 2 * nPositions - 2), eLS = pow10i(3 + 2 * nPositions - 2),
                 nLS = pow10i(1 + 2 * nPositions - 2), eS = pow10i(nPositions);
    const int32_t nb10 = (int32_t)((uint32_t)nBin * 10u);  // Int * Int wraps
    const double id = res == -1 ? (idP + (double)eLetter * eLS) / 100 + (double)quadrant
                                : idP + (double)eLetter * eLS + (double)nLetter * nLS + (double)eBin * eS + (double)nb10 +
                                      (double)quadrant;
    return jvm_d2l(id);
}
// Returns false where the reference throws (no letter pair, non-numeric bins, Int overflow).
MOSAIC_HD bool parse(const char* s, int n, int64_t* out) {
    const int lc = n >= 2 ? letter_code(s[0], s[1]) : (n == 1 ? letter_code(s[0], 'V') : -1);
    if (lc < 0) return false;
    const int eLetter = lc & 7, nLetter = lc >> 3;
    if (n == 1) {
        *out = encode(eLetter, 0, 0, 0, 0, 1, -1);
        return true;
    }
    // suffix = the last two characters; quadrants = ("", "SW", "NW", "NE", "SE")
    const char a = s[n - 2], b = s[n - 1];
    int quadrant = 0;
    if (b == 'W' && (a == 'S' || a == 'N')) quadrant = a == 'S' ? 1 : 2;
    else if (b == 'E' && (a == 'N' || a == 'S')) quadrant = a == 'N' ? 3 : 4;
    // binDigits = drop(2) (then dropRight(2) with a quadrant); may be empty or, for "SW"-like ids of
    // length 2 or 3, start past its end
    const int d0 = 2, d1 = quadrant > 0 ? n - 2 : n;
    const int L = d1 > d0 ? d1 - d0 : 0;
    if (L == 0) {
        *out = encode(eLetter, nLetter, 0, 0, quadrant, 1, -2);
        return true;
    }
    int32_t eBin, nBin;
    if (!java_parse_int(s + d0, L - L / 2, &eBin) || !java_parse_int(s + d0 + L / 2, L - L / 2, &nBin)) return false;
    const int nPositions = L / 2 + 1;
    const int res = quadrant == 0 ? nPositions + 1 : -nPositions;
    *out = encode(eLetter, nLetter, eBin, nBin, quadrant, nPositions, res);
    return true;
}

// ---- k-loops / k-rings: BNGIndexSystem.kLoop / kRing (BNGIndexSystem.scala:216-246) with the
// cell decoding they use: indexDigits (index.toString digits), getResolution(digits), getEdgeSize
// (sizeMap), getX / getY, isValid (BNGIndexSystem.scala:248-263).  Int arithmetic as in Scala.

// decimal digits of a positive id, most significant first; returns their count (0 for id <= 0,
// whose toString the reference would not decode)
MOSAIC_HD int index_digits(int64_t id, int* d) {
    if (id <= 0) return 0;
    // 64-bit division only to split off 9-digit groups; the digits come from 32-bit arithmetic
    int t[20], n = 0;
    uint64_t u = (uint64_t)id;
    while (u >= 1000000000ull) {
        uint32_t lo = (uint32_t)(u % 1000000000ull);
        u /= 1000000000ull;
        for (int i = 0; i < 9; i++) {
            t[n++] = (int)(lo % 10u);
            lo /= 10u;
        }
    }
    uint32_t hi = (uint32_t)u;
    while (hi > 0) {
        t[n++] = (int)(hi % 10u);
        hi /= 10u;
    }
    for (int i = 0; i < n; i++) d[i] = t[n - 1 - i];
    return n;
}
MOSAIC_HD int digits_resolution(const int* d, int n) {
    if (n < 6) return -1;  // 500km
    const int k = (n - 6) / 2;
    return d[n - 1] > 0 ? -(k + 2) : k + 1;
}
// sizeMap(getResolutionStr(res)); 0 where the reference's map lookup throws
MOSAIC_HD int32_t edge_size(int res) {
    switch (res) {
        case -1: return 500000;
        case 1: return 100000;
        case -2: return 50000;
        case 2: return 10000;
        case -3: return 5000;
        case 3: return 1000;
        case -4: return 500;
        case 4: return 100;
        case -5: return 50;
        case 5: return 10;
        case -6: return 5;
        case 6: return 1;
        default: return 0;
    }
}
// getX (y = 0) / getY (y = 1): the letter digits then k coordinate digits, as one Int, times the
// (quadrant-adjusted) edge size, plus the quadrant's offset
MOSAIC_HD int32_t digits_coord(const int* d, int n, int32_t edge, int y) {
    const int k = (n - 6) / 2;  // JVM Int division: truncates toward zero (0 for n = 5)
    const int a = y ? 3 : 1, b = y ? 5 + k : 5;
    int32_t v = 0;
    for (int i = a; i < a + 2 && i < n; i++) v = v * 10 + d[i];  // at most 2 + 6 digits: no overflow
    for (int i = b; i < b + k && i < n; i++) v = v * 10 + d[i];
    const int q = d[n - 1];
    const int32_t adj = q > 0 ? 2 * edge : edge;
    const int32_t off = y ? ((q == 2 || q == 3) ? edge : 0) : ((q == 3 || q == 4) ? edge : 0);
    return (int32_t)((uint32_t)v * (uint32_t)adj + (uint32_t)off);  // Int * and + wrap
}
// cell -> (resolution, edge size, x, y); false if the reference could not decode it
MOSAIC_HD bool cell_origin(int64_t id, int* res, int32_t* edge, int32_t* x, int32_t* y) {
    int d[20];
    const int n = index_digits(id, d);
    if (n < 4) return false;  // the reference's digit slices would be empty (NumberFormatException)
    *res = digits_resolution(d, n);
    *edge = edge_size(*res);
    if (*edge == 0) return false;
    *x = digits_coord(d, n, *edge, 0);
    *y = digits_coord(d, n, *edge, 1);
    return true;
}
MOSAIC_HD bool is_valid(int64_t id) {
    int res;
    int32_t e, x, y;
    if (!cell_origin(id, &res, &e, &x, &y)) return false;
    return x >= 0 && x <= 700000 && y >= 0 && y <= 1300000;
}
// kLoop(id, k): the 8k cells of the square loop at distance k, bottom, right, top, left, each
// side from its first corner, keeping the isValid ones (order kept).  Returns the count, or -1 if
// the id cannot be decoded.
MOSAIC_HD int kloop(int64_t id, int k, int64_t* out) {
    int res;
    int32_t e, x, y;
    if (!cell_origin(id, &res, &e, &x, &y)) return -1;
    int m = 0;
    for (int side = 0; side < 4; side++)
        for (int c = 0; c < 2 * k; c++) {
            // Int arithmetic, wrapping as the JVM's does (exact in int64 for |k| < 2^20, then
            // truncated to 32 bits)
            const int64_t X = x, Y = y, E = e, K = k, C = c;
            int64_t qx, qy;
            if (side == 0) {
                qx = X + (C - K) * E;
                qy = Y - K * E;
            } else if (side == 1) {
                qx = X + K * E;
                qy = Y + (C - K) * E;
            } else if (side == 2) {
                qx = X + (K - C) * E;
                qy = Y + K * E;
            } else {
                qx = X - K * E;
                qy = Y + (K - C) * E;
            }
            const int32_t px = (int32_t)(uint32_t)(uint64_t)qx, py = (int32_t)(uint32_t)(uint64_t)qy;
            int64_t cell = 0;
            point_to_index((double)px, (double)py, res, &cell);
            if (is_valid(cell)) out[m++] = cell;
        }
    return m;
}
// kRing(id, n) = id, then kLoop(id, 1 .. n)
MOSAIC_HD int kring(int64_t id, int n, int64_t* out) {
    int res;
    int32_t e, x, y;
    if (!cell_origin(id, &res, &e, &x, &y)) return -1;
    int m = 0;
    out[m++] = id;
    for (int k = 1; k <= n; k++) m += kloop(id, k, out + m);
    return m;
}


// ---- BNGIndexSystem.format (BNGIndexSystem.scala:114-129) for one id, device and host: the two
// letters of letterMap(nLetter digits)(eLetter digits) (row 10 col 4 is "SZ" as in the reference,
// :96), then the k easting and k northing digits and the quadrant's name.  Writes at most 16 chars
// to out (may be null: length only); returns the length, or -1 for an id the reference cannot format.
MOSAIC_HD int format_id(int64_t id, char* out) {
    const char* const kLetters =
        "SVSWSXSYSZTVTWSQSRSSSTSUTQTRSLSMSNSOSPTLTMSFSGSHSJSKTFTGSASBSCSDSETATBNVNWNXNYNZOVOW"
        "NQNRNSNTNUOQORNLNMNNNONPOLOMNFNGNHNJNKOFOGNANBNCNDNEOAOBHVHWHXHYSZJVJWHQHRHSHTHUJQJR"
        "HLHMHNHOHPJLJM";
    const char* const kQuad = "  SWNWNESE";
    int d[20];
    const int n = index_digits(id, d);
    if (n < 4) return -1;  // slice(3, 5) would be empty (NumberFormatException)
    const int col = d[1] * 10 + d[2], row = n == 4 ? d[3] : d[3] * 10 + d[4];
    if (row > 12 || col > 6) return -1;
    const char* lt = kLetters + 2 * (row * 7 + col);
    if (n < 6) {
        if (out) out[0] = lt[0];
        return 1;
    }
    const int q = d[n - 1];
    if (q > 4) return -1;
    const int k = (n - 6) / 2;
    int m = 0;
    if (out) {
        out[0] = lt[0];
        out[1] = lt[1];
    }
    m = 2;
    for (int i = 5; i < 5 + 2 * k; i++, m++)
        if (out) out[m] = (char)('0' + d[i]);
    if (q > 0) {
        if (out) {
            out[m] = kQuad[2 * q];
            out[m + 1] = kQuad[2 * q + 1];
        }
        m += 2;
    }
    return m;
}


// ---- BNGIndexSystem.indexToGeometry (BNGIndexSystem.scala:420-431 area: the cell square
// (x, y) (x + e, y) (x + e, y + e) (x, y + e) (x, y) in Int arithmetic) as JTS WKBWriter writes it
// for grid_boundaryaswkb: big-endian, 2D Polygon, one ring of 5 points = 93 bytes.
static const int kCellWkbBytes = 93;
MOSAIC_HD void put_be_u32(uint8_t* o, uint32_t v) {
    o[0] = (uint8_t)(v >> 24);
    o[1] = (uint8_t)(v >> 16);
    o[2] = (uint8_t)(v >> 8);
    o[3] = (uint8_t)v;
}
MOSAIC_HD void put_be_f64(uint8_t* o, double d) {
    uint64_t u;
    memcpy(&u, &d, 8);
    for (int i = 0; i < 8; i++) o[i] = (uint8_t)(u >> (56 - 8 * i));
}
MOSAIC_HD bool cell_wkb(int64_t id, uint8_t* o) {
    int res;
    int32_t e, x, y;
    if (!cell_origin(id, &res, &e, &x, &y)) return false;
    const int32_t x1 = (int32_t)((uint32_t)x + (uint32_t)e), y1 = (int32_t)((uint32_t)y + (uint32_t)e);
    const int32_t px[5] = {x, x1, x1, x, x}, py[5] = {y, y, y1, y1, y};
    o[0] = 0;  // big-endian
    put_be_u32(o + 1, 3);
    put_be_u32(o + 5, 1);
    put_be_u32(o + 9, 5);
    for (int i = 0; i < 5; i++) {
        put_be_f64(o + 13 + 16 * i, (double)px[i]);
        put_be_f64(o + 21 + 16 * i, (double)py[i]);
    }
    return true;
}

}  // namespace bng
}  // namespace mosaic
