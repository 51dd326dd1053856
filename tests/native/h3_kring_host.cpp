// CPU build of the H3 k-ring kernel code (mosaic_amd/csrc/h3_grid.h, the device code compiled by
// g++) as a small shared library, so tests/test_h3_kring.py can compare it with the oracle's
// sphere-search k-ring (oracle/h3.c) without a GPU.
#include <stdint.h>

#include "h3_grid.h"

extern "C" int h3_kring_host(int64_t cell, int k, int loop, int64_t* out) {
    return mosaic::h3grid::kring((uint64_t)cell, k, loop, out);
}
