// Test-only: exports mosaic_amd/csrc/crmath.h (compiled for the host) over a C ABI for ctypes.
#include "../../mosaic_amd/csrc/crmath.h"
extern "C" {
void crm_eval(int fn, const double* a, const double* b, long n, double* out) {
    using namespace mosaic::crm;
    for (long i = 0; i < n; i++) {
        switch (fn) {
            case 0: out[i] = sin_cr(a[i]); break;
            case 1: out[i] = cos_cr(a[i]); break;
            case 2: out[i] = tan_cr(a[i]); break;
            case 3: out[i] = acos_cr(a[i]); break;
            default: out[i] = atan2_cr(a[i], b[i]); break;
        }
    }
}
}
