// CPU build of the H3 cell-geometry kernel code (mosaic_amd/csrc/h3_geom.h, the device code compiled
// by g++) as a small shared library, so tests/test_h3_geom.py can compare it with the oracle
// (oracle/h3.c) bit for bit without a GPU.
#include <stdint.h>

#include "h3_geom.h"

extern "C" int h3_boundary_host(int64_t cell, double* out) {
    return mosaic::h3geom::h3_to_geo_boundary((uint64_t)cell, out);
}
extern "C" int h3_center_host(int64_t cell, double* out) {
    return mosaic::h3geom::h3_to_geo((uint64_t)cell, &out[0], &out[1]) ? 1 : 0;
}
