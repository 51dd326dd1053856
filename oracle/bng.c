/*
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  CPU restatement of BNGIndexSystem point indexing.
 *
 * Follows src/main/scala/com/databricks/labs/mosaic/core/index/BNGIndexSystem.scala with JVM
 * semantics:
 *   pointToIndex  :277-291  (Double.toInt truncation/saturation, Int division and remainder)
 *   getQuadrant   :309-327
 *   encode        :528-541  (id assembled in f64 from math.pow(10, n) then Double.toLong)
 *   format        :114-129  (letterMap :84-99, quadrants :36)
 * Pinned by the reference's golden vectors TestBNGIndexSystem.scala:10-90 (tests/test_oracle_bng.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

/* JVM d2i: NaN -> 0, saturate to [INT_MIN, INT_MAX], truncate toward zero */
static int32_t jvm_d2i(double d) {
    if (d != d) return 0;
    if (d >= 2147483647.0) return 2147483647;
    if (d <= -2147483648.0) return (-2147483647 - 1);
    return (int32_t)d;
}
/* JVM d2l */
static int64_t jvm_d2l(double d) {
    if (d != d) return 0;
    if (d >= 9223372036854775807.0) return INT64_MAX;
    if (d <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)d;
}
/* java.lang.Math.pow(10, n) is exact for the integer exponents used here (JLS: exact when
 * representable); n ranges over 0..15. */
static double pow10i(int n) {
    static const double t[] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7,
                               1e8, 1e9, 1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                               1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
    if (n >= 0 && n <= 22) return t[n];
    return pow(10.0, (double)n);
}
/* JVM Int arithmetic wraps */
static int32_t imul32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }

/* BNGIndexSystem.scala:309-327 */
static int get_quadrant(int res, double e, double n, double divisor) {
    if (res < -1) {
        double eQ = e / divisor;
        double nQ = n / divisor;
        double eD = eQ - floor(eQ);
        double nD = nQ - floor(nQ);
        if (eD < 0.5 && nD < 0.5) return 1; /* SW */
        if (eD < 0.5) return 2;             /* NW */
        if (nD < 0.5) return 4;             /* SE */
        return 3;                           /* NE */
    }
    return 0;
}

/* BNGIndexSystem.scala:528-541 */
static int64_t encode(int32_t eLetter, int32_t nLetter, int32_t eBin, int32_t nBin, int32_t quadrant,
                      int32_t nPositions, int32_t res) {
    double idPlaceholder = pow10i(5 + 2 * nPositions - 2);
    double eLetterShift = pow10i(3 + 2 * nPositions - 2);
    double nLetterShift = pow10i(1 + 2 * nPositions - 2);
    double eShift = pow10i(nPositions);
    int32_t nShift = 10;
    double id;
    if (res == -1) {
        id = (idPlaceholder + (double)eLetter * eLetterShift) / 100 + (double)quadrant;
    } else {
        id = idPlaceholder + (double)eLetter * eLetterShift + (double)nLetter * nLetterShift +
             (double)eBin * eShift + (double)imul32(nBin, nShift) + (double)quadrant;
    }
    return jvm_d2l(id);
}

static int valid_res(int res) { return res != 0 && res >= -6 && res <= 6; }

/* BNGIndexSystem.scala:277-291 */
int64_t oracle_bng_point_to_index(double eastings, double northings, int res, int* err) {
    *err = 0;
    if (eastings != eastings || northings != northings) {
        *err = 1; /* IllegalStateException("NaN coordinates are not supported.") */
        return 0;
    }
    if (!valid_res(res)) {
        *err = 2; /* IllegalStateException("BNG resolution not supported; found ...") */
        return 0;
    }
    int32_t eI = jvm_d2i(eastings);
    int32_t nI = jvm_d2i(northings);
    int32_t eLetter = jvm_d2i(floor((double)(eI / 100000)));
    int32_t nLetter = jvm_d2i(floor((double)(nI / 100000)));
    int ares = res < 0 ? -res : res;
    double divisor = res < 0 ? pow10i(6 - ares + 1) : pow10i(6 - res);
    int32_t quadrant = get_quadrant(res, (double)eI, (double)nI, divisor);
    int32_t nPositions = res >= -1 ? ares : ares - 1;
    int32_t eBin = jvm_d2i(floor((double)(eI % 100000) / divisor));
    int32_t nBin = jvm_d2i(floor((double)(nI % 100000) / divisor));
    return encode(eLetter, nLetter, eBin, nBin, quadrant, nPositions, res);
}

void oracle_bng_point_to_index_batch(const double* e, const double* n, int64_t count, int res,
                                     int64_t* out, uint8_t* err) {
    for (int64_t i = 0; i < count; i++) {
        int er;
        out[i] = oracle_bng_point_to_index(e[i], n[i], res, &er);
        err[i] = (uint8_t)er;
    }
}

/* BNGIndexSystem.scala:84-99 */
static const char* kLetterMap[13][7] = {
    {"SV", "SW", "SX", "SY", "SZ", "TV", "TW"}, {"SQ", "SR", "SS", "ST", "SU", "TQ", "TR"},
    {"SL", "SM", "SN", "SO", "SP", "TL", "TM"}, {"SF", "SG", "SH", "SJ", "SK", "TF", "TG"},
    {"SA", "SB", "SC", "SD", "SE", "TA", "TB"}, {"NV", "NW", "NX", "NY", "NZ", "OV", "OW"},
    {"NQ", "NR", "NS", "NT", "NU", "OQ", "OR"}, {"NL", "NM", "NN", "NO", "NP", "OL", "OM"},
    {"NF", "NG", "NH", "NJ", "NK", "OF", "OG"}, {"NA", "NB", "NC", "ND", "NE", "OA", "OB"},
    {"HV", "HW", "HX", "HY", "SZ", "JV", "JW"}, {"HQ", "HR", "HS", "HT", "HU", "JQ", "JR"},
    {"HL", "HM", "HN", "HO", "HP", "JL", "JM"}};
static const char* kQuadrants[5] = {"", "SW", "NW", "NE", "SE"};

static int digits_to_int(const char* d, int from, int to, int len) {
    /* Seq.slice(from, to).mkString.toInt */
    int v = 0;
    if (from >= len) return -1;
    if (to > len) to = len;
    for (int i = from; i < to; i++) v = v * 10 + (d[i] - '0');
    return v;
}

/* BNGIndexSystem.scala:114-129 */
int oracle_bng_format(int64_t id, char* buf, int cap) {
    char d[32];
    if (id <= 0) return -1;
    int len = snprintf(d, sizeof d, "%lld", (long long)id);
    int row = digits_to_int(d, 3, 5, len);
    int col = digits_to_int(d, 1, 3, len);
    if (row < 0 || col < 0 || row > 12 || col > 6) return -1;
    const char* prefix = kLetterMap[row][col];
    char out[64];
    int o = 0;
    if (len < 6) {
        out[o++] = prefix[0];
    } else {
        int quadrant = d[len - 1] - '0';
        if (quadrant > 4) return -1;
        out[o++] = prefix[0];
        out[o++] = prefix[1];
        int clen = len - 6; /* digits.drop(5).dropRight(1) */
        int k = clen / 2;
        for (int i = 0; i < k; i++) out[o++] = d[5 + i];
        for (int i = 0; i < k; i++) out[o++] = d[5 + k + i];
        const char* q = kQuadrants[quadrant];
        for (int i = 0; q[i]; i++) out[o++] = q[i];
    }
    out[o] = 0;
    if (o + 1 > cap) return -1;
    memcpy(buf, out, o + 1);
    return o;
}

/* ---- BNGIndexSystem.parse (BNGIndexSystem.scala:391-413) + encode (:528-541) ----
 * letterMap.find(_.contains(prefix)).get: the first row holding the pair (row 0 for "SZ"), its
 * first column; Integer.parseInt for the bins (sign, ASCII digits, Int range; Java's non-ASCII
 * Unicode digits are not restated).  Returns 1 and the id, or 0 where the reference throws. */
static int java_parse_int(const char* s, int n, int32_t* out) {
    if (n <= 0) return 0;
    int i = 0, neg = 0;
    if (s[0] == '-' || s[0] == '+') {
        neg = s[0] == '-';
        i = 1;
        if (n == 1) return 0;
    }
    long long v = 0;
    for (; i < n; i++) {
        if (s[i] < '0' || s[i] > '9') return 0;
        v = v * 10 + (s[i] - '0');
        if (v > 2147483648LL) return 0;
    }
    if (!neg && v > 2147483647LL) return 0;
    *out = (int32_t)(neg ? -v : v);
    return 1;
}

static int64_t bng_encode(int eL, int nL, int32_t eBin, int32_t nBin, int q, int nPos, int res) {
    double idP = pow(10.0, 5 + 2 * nPos - 2), eLS = pow(10.0, 3 + 2 * nPos - 2), nLS = pow(10.0, 1 + 2 * nPos - 2);
    double eS = pow(10.0, nPos);
    int32_t nb10 = (int32_t)((uint32_t)nBin * 10u);
    double id = res == -1 ? (idP + eL * eLS) / 100 + q : idP + eL * eLS + nL * nLS + eBin * eS + nb10 + q;
    return jvm_d2l(id);
}

int oracle_bng_parse(const char* s, int n, int64_t* out) {
    char prefix[3] = {0, 0, 0};
    if (n >= 2) {
        prefix[0] = s[0];
        prefix[1] = s[1];
    } else if (n == 1) {
        prefix[0] = s[0];
        prefix[1] = 'V';
    } else {
        return 0;
    }
    int eL = -1, nL = -1;
    for (int r = 0; r < 13 && eL < 0; r++)
        for (int c = 0; c < 7; c++)
            if (strcmp(kLetterMap[r][c], prefix) == 0) {
                eL = c;
                nL = r;
                break;
            }
    if (eL < 0) return 0;
    if (n == 1) {
        *out = bng_encode(eL, 0, 0, 0, 0, 1, -1);
        return 1;
    }
    char suffix[3] = {s[n - 2], s[n - 1], 0};
    int q = 0;
    for (int i = 1; i < 5; i++)
        if (strcmp(kQuadrants[i], suffix) == 0) q = i;
    /* drop(2), then dropRight(2) with a quadrant */
    int from = 2, to = q > 0 ? n - 2 : n;
    int L = to > from ? to - from : 0;
    if (L == 0) {
        *out = bng_encode(eL, nL, 0, 0, q, 1, -2);
        return 1;
    }
    int32_t eBin, nBin;
    int half = L / 2;
    if (!java_parse_int(s + from, L - half, &eBin)) return 0;  /* dropRight(half) */
    if (!java_parse_int(s + from + half, L - half, &nBin)) return 0;  /* drop(half) */
    int nPos = half + 1;
    int res = q == 0 ? nPos + 1 : -nPos;
    *out = bng_encode(eL, nL, eBin, nBin, q, nPos, res);
    return 1;
}

/* ---- BNGIndexSystem.kLoop / kRing / isValid (BNGIndexSystem.scala:216-263) ----
 * The id's decimal string (indexDigits), getResolution(digits), sizeMap, getX / getY (Int
 * arithmetic, wrapping), then pointToIndex of the loop's cell origins filtered by isValid. */
static int bng_digits(int64_t id, int* d) {
    char buf[32];
    if (id <= 0) return 0;
    int n = snprintf(buf, sizeof buf, "%lld", (long long)id);
    for (int i = 0; i < n; i++) d[i] = buf[i] - '0';
    return n;
}

/* (slice(a0, a1) ++ slice(b0, b1)).mkString.toInt of the digit sequence (at most 8 digits here) */
static int32_t bng_slices_int(const int* d, int n, int a0, int a1, int b0, int b1) {
    char s[40];
    int m = 0;
    for (int i = a0; i < a1 && i < n; i++) s[m++] = (char)('0' + d[i]);
    for (int i = b0; i < b1 && i < n; i++) s[m++] = (char)('0' + d[i]);
    s[m] = 0;
    return (int32_t)strtol(s, NULL, 10);
}

/* 0 if the reference cannot decode the id */
static int bng_origin(int64_t id, int* res, int32_t* edge, int32_t* x, int32_t* y) {
    static const int sizes_pos[7] = {0, 100000, 10000, 1000, 100, 10, 1};
    static const int sizes_neg[7] = {0, 500000, 50000, 5000, 500, 50, 5};
    int d[32];
    int n = bng_digits(id, d);
    if (n < 4) return 0;
    int q = d[n - 1];
    int k = (n - 6) / 2; /* C and JVM Int division both truncate toward zero */
    *res = n < 6 ? -1 : (q > 0 ? -(k + 2) : k + 1);
    if (*res < -6 || *res > 6 || *res == 0) return 0;
    *edge = *res > 0 ? sizes_pos[*res] : sizes_neg[-*res];
    uint32_t adj = (uint32_t)(q > 0 ? 2 * *edge : *edge);
    int32_t xd = bng_slices_int(d, n, 1, 3, 5, 5 + k), yd = bng_slices_int(d, n, 3, 5, 5 + k, 5 + 2 * k);
    *x = (int32_t)((uint32_t)xd * adj + (uint32_t)((q == 3 || q == 4) ? *edge : 0));
    *y = (int32_t)((uint32_t)yd * adj + (uint32_t)((q == 2 || q == 3) ? *edge : 0));
    return 1;
}

int oracle_bng_is_valid(int64_t id) {
    int res;
    int32_t e, x, y;
    if (!bng_origin(id, &res, &e, &x, &y)) return 0;
    return x >= 0 && x <= 700000 && y >= 0 && y <= 1300000;
}

int oracle_bng_kloop(int64_t id, int k, int64_t* out) {
    int res;
    int32_t e, x, y;
    if (!bng_origin(id, &res, &e, &x, &y)) return -1;
    int m = 0;
    /* bottom, right, top, left (BNGIndexSystem.scala:238-241) */
    for (int side = 0; side < 4; side++) {
        for (int c = 0; c < 2 * k; c++) {
            uint32_t ux = (uint32_t)x, uy = (uint32_t)y, ue = (uint32_t)e, uk = (uint32_t)k, uc = (uint32_t)c;
            uint32_t qx, qy;
            switch (side) {
                case 0: qx = ux + (uc - uk) * ue; qy = uy - uk * ue; break;
                case 1: qx = ux + uk * ue; qy = uy + (uc - uk) * ue; break;
                case 2: qx = ux + (uk - uc) * ue; qy = uy + uk * ue; break;
                default: qx = ux - uk * ue; qy = uy + (uk - uc) * ue; break;
            }
            int err = 0;
            int64_t cell = oracle_bng_point_to_index((double)(int32_t)qx, (double)(int32_t)qy, res, &err);
            if (oracle_bng_is_valid(cell)) out[m++] = cell;
        }
    }
    return m;
}

int oracle_bng_kring(int64_t id, int n, int64_t* out) {
    int res;
    int32_t e, x, y;
    if (!bng_origin(id, &res, &e, &x, &y)) return -1;
    int m = 0;
    out[m++] = id;
    for (int k = 1; k <= n; k++) m += oracle_bng_kloop(id, k, out + m);
    return m;
}

/* BNGIndexSystem.indexToGeometry's square: origin (x, y) and edge of the cell (Int arithmetic as
 * getX / getY); 0 if the id cannot be decoded. */
int oracle_bng_cell_origin(int64_t id, int32_t* out4) {
    int res;
    int32_t e, x, y;
    if (!bng_origin(id, &res, &e, &x, &y)) return 0;
    out4[0] = res;
    out4[1] = e;
    out4[2] = x;
    out4[3] = y;
    return 1;
}
