// GPU probe: H3 kRing fast walk (h3_neighbors.h kring_fast) over a list of cells, one lane per row as
// in k_h3_kring; prints "row count first" per row.  Host build: g++ -DHOST_WALK -x c++ kring_probe.hip
//   usage: kring_probe CELLS_FILE K
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
__global__ void kk(const int64_t* cells, int64_t n, int k, int64_t* out, int stride, int* cnt) {
#ifndef HOST_WALK
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
#else
    for (int64_t i = 0; i < n; i++)
#endif
        cnt[i] = h3nb::kring_fast((uint64_t)cells[i], k, 0, out + i * stride);
}
int main(int argc, char** argv) {
    if (argc < 3) return 1;
    FILE* f = fopen(argv[1], "r");
    if (!f) return 1;
    const int k = atoi(argv[2]), stride = 1 + 3 * k * (k + 1);
    std::vector<int64_t> cells;
    long long c;
    while (fscanf(f, "%lld", &c) == 1) cells.push_back(c);
    fclose(f);
    const int64_t n = (int64_t)cells.size();
    std::vector<int64_t> out((size_t)n * stride);
    std::vector<int> cnt((size_t)n);
#ifndef HOST_WALK
    int64_t *dc, *dout;
    int* dcnt;
    if (hipMalloc(&dc, n * 8) || hipMalloc(&dout, n * stride * 8) || hipMalloc(&dcnt, n * 4)) return 2;
    if (hipMemcpy(dc, cells.data(), n * 8, hipMemcpyHostToDevice)) return 2;
    kk<<<(unsigned)((n + 255) / 256), 256>>>(dc, n, k, dout, stride, dcnt);
    if (hipDeviceSynchronize() || hipMemcpy(out.data(), dout, n * stride * 8, hipMemcpyDeviceToHost) ||
        hipMemcpy(cnt.data(), dcnt, n * 4, hipMemcpyDeviceToHost)) return 3;
#else
    kk(cells.data(), n, k, out.data(), stride, cnt.data());
#endif
    for (int64_t i = 0; i < n; i++) printf("%ld %d %ld\n", (long)i, cnt[i], (long)(cnt[i] > 0 ? out[i * stride + 1] : 0));
    return 0;
}
