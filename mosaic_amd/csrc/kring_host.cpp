// H3 k-ring rows that mosaic_cell_kring answers on host threads (k > 128 near a pentagon: H3's
// _kRingInternal search, ~5 k^3 dependent visits per row).  Compiled by g++ like the other host
// builders: h3_neighbors.h's tables are host constants here (in mosaic_hip.hip's host pass they are
// __constant__ shadows, which host code must not read).
#include <stdint.h>

#include "h3_neighbors.h"

namespace mosaic {

int kring_slow_host(uint64_t origin, int k, int loop, int64_t* out, int64_t* tab, int32_t* dist, uint64_t* stack) {
    return h3nb::kring_slow(origin, k, loop, out, tab, dist, stack);
}

}  // namespace mosaic
