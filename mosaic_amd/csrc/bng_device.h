// BNG (British National Grid) point -> cell id for gfx950 and the host.
// Restates reference src/main/scala/com/databricks/labs/mosaic/core/index/BNGIndexSystem.scala
//   pointToIndex :277-291, getQuadrant :309-327, encode :528-541
// with JVM semantics (Double.toInt / toLong truncate and saturate, Int `/` and `%` truncate toward
// zero, Int `*` wraps, math.pow(10, n) exact).  Every operation is an exactly specified IEEE or
// integer operation, so the device result is bit-identical to the JVM's.
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
namespace bng {

MOSAIC_HD int32_t jvm_d2i(double d) {
    if (d != d) return 0;
    if (d >= 2147483647.0) return 2147483647;
    if (d <= -2147483648.0) return (-2147483647 - 1);
    return (int32_t)d;
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

}  // namespace bng
}  // namespace mosaic
