// CPU probe (not a test): glibc_math.h (the glibc 2.35 dbl-64 restatement) compiled with FMA
// contraction everywhere (-mfma -ffp-contract=fast), as an aarch64 glibc build of the same sources
// would contract it; exported for the kepler ring sweep (run_fma.sh).
#include "../../../mosaic_amd/csrc/glibc_math.h"
extern "C" {
double lf_sin(double x) { double s, c; mosaic::glibc::sincos(x, &s, &c); return s; }
double lf_cos(double x) { double s, c; mosaic::glibc::sincos(x, &s, &c); return c; }
double lf_asin(double x) { return mosaic::glibc::asin(x); }
double lf_atan(double x) { return mosaic::glibc::atan(x); }
double lf_atan2(double y, double x) { return mosaic::glibc::atan2(y, x); }
}
