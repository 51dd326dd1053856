// CPU build of the H3 k-ring kernel code (mosaic_amd/csrc/h3_neighbors.h, the device code compiled
// by g++) as a small shared library, so tests/test_h3_kring.py can compare it with the oracle's
// sphere-search k-ring (oracle/h3.c) without a GPU: the fast walk (hexRange / hexRing) and, where
// H3 meets a pentagon, the fallback (_kRingInternal; the reference's set difference for kLoop).
#include <stdint.h>

#include <vector>

#include "h3_neighbors.h"

// the row's cells in out; returns the count, -2 for an invalid id; *slow = 1 if the fallback ran
extern "C" int h3_kring_host(int64_t cell, int k, int loop, int64_t* out, int* slow) {
    const int n = mosaic::h3nb::kring_fast((uint64_t)cell, k, loop, out);
    *slow = n == -3;
    if (n != -3) return n;
    const int m = mosaic::h3nb::max_kring_size(k), m1 = k ? mosaic::h3nb::max_kring_size(k - 1) : 1;
    std::vector<int64_t> tab((size_t)(m + m1));
    std::vector<int32_t> dist((size_t)m);
    std::vector<uint64_t> stack((size_t)k + 1);
    return mosaic::h3nb::kring_slow((uint64_t)cell, k, loop, out, tab.data(), dist.data(), stack.data());
}

extern "C" int64_t h3_neighbor_host(int64_t cell, int dir) {
    int r = 0;
    return (int64_t)mosaic::h3nb::neighbor_rotations((uint64_t)cell, dir, &r);
}
