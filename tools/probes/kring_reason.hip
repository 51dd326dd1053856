// GPU probe: h3nb::hex_range (h3_neighbors.h) restated with a record of where it stops: per row of
// a cell list (k = 1) "row code step" -- code 0 done, 1 pentagon origin, 2 NextRing step -> 0,
// 3 NextRing step -> pentagon, 4 ring step -> 0, 5 ring step -> pentagon; and the library's own
// hex_range result.  Host build: g++ -DHOST_WALK -x c++.
#ifndef HOST_WALK
#include <hip/hip_runtime.h>
#else
#define __global__
#endif
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "../../mosaic_amd/csrc/h3_neighbors.h"
using namespace mosaic;
MOSAIC_HD int range_reason(uint64_t origin, int k, int* step, int* pent_flags) {
    int n = 0;
    *pent_flags = 0;
    if (h3nb::is_pentagon(origin)) return 1;
    int ring = 1, dir = 0, i = 0, rotations = 0;
    while (ring <= k) {
        if (dir == 0 && i == 0) {
            origin = h3nb::neighbor_rotations(origin, h3nb::kNextRing, &rotations);
            *step = n;
            if (origin == 0) return 2;
            if (h3nb::is_pentagon(origin)) return 3;
        }
        origin = h3nb::neighbor_rotations(origin, h3nb::direction(dir), &rotations);
        *step = ++n;
        if (origin == 0) return 4;
        *pent_flags |= (h3nb::base_is_pentagon(h3nb::base_cell_of(origin)) ? 1 : 0) << (2 * n);
        *pent_flags |= (h3::leading_nonzero_digit(origin, h3nb::res_of(origin)) == 0 ? 1 : 0) << (2 * n + 1);
        i++;
        if (i == ring) {
            i = 0;
            dir++;
            if (dir == 6) {
                dir = 0;
                ring++;
            }
        }
        if (h3nb::is_pentagon(origin)) return 5;
    }
    return 0;
}
__global__ void kk(const int64_t* cells, int64_t n, int* out) {
#ifndef HOST_WALK
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
#else
    for (int64_t i = 0; i < n; i++) {
#endif
        int step = -1, pf = 0;
        out[4 * i] = range_reason((uint64_t)cells[i], 1, &step, &pf);
        out[4 * i + 1] = step;
        out[4 * i + 2] = pf;
        int64_t tmp[8];
        out[4 * i + 3] = h3nb::hex_range((uint64_t)cells[i], 1, tmp) ? 1 : 0;
    }
}
int main(int argc, char** argv) {
    if (argc < 2) return 1;
    FILE* f = fopen(argv[1], "r");
    if (!f) return 1;
    std::vector<int64_t> cells;
    long long c;
    while (fscanf(f, "%lld", &c) == 1) cells.push_back(c);
    fclose(f);
    const int64_t n = (int64_t)cells.size();
    std::vector<int> out((size_t)n * 4);
#ifndef HOST_WALK
    int64_t* dc;
    int* dout;
    if (hipMalloc(&dc, n * 8) || hipMalloc(&dout, n * 16)) return 2;
    if (hipMemcpy(dc, cells.data(), n * 8, hipMemcpyHostToDevice)) return 2;
    kk<<<(unsigned)((n + 255) / 256), 256>>>(dc, n, dout);
    if (hipDeviceSynchronize() || hipMemcpy(out.data(), dout, n * 16, hipMemcpyDeviceToHost)) return 3;
#else
    kk(cells.data(), n, out.data());
#endif
    for (int64_t i = 0; i < n; i++) printf("%ld %d %d %d %d\n", (long)i, out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]);
    return 0;
}
