// GPU probe: the hexRange k = 1 walk (h3_neighbors.h neighbor_rotations) of every cell in a list,
// one lane per row, every step recorded (input, direction, rotations, output); host build with
// g++ -DHOST_WALK -x c++.  usage: kring_trace CELLS_FILE  -> "row step dir in rot_in out rot_out"
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
struct Step {
    unsigned long long in, out;
    int dir, rot_in, rot_out, pad;
};
static const int kSteps = 8;
MOSAIC_HD void walk1(uint64_t origin, Step* st) {
    int n = 0, dir = 0, i = 0, rotations = 0, ring = 1;
    while (ring <= 1 && n < kSteps) {
        if (dir == 0 && i == 0) {
            Step& s = st[n++];
            s.in = origin; s.dir = h3nb::kNextRing; s.rot_in = rotations;
            origin = h3nb::neighbor_rotations(origin, h3nb::kNextRing, &rotations);
            s.out = origin; s.rot_out = rotations;
            if (origin == 0) break;
        }
        Step& s = st[n++];
        s.in = origin; s.dir = h3nb::direction(dir); s.rot_in = rotations;
        origin = h3nb::neighbor_rotations(origin, h3nb::direction(dir), &rotations);
        s.out = origin; s.rot_out = rotations;
        if (origin == 0) break;
        if (++i == ring) { i = 0; if (++dir == 6) { dir = 0; ring++; } }
    }
    for (; n < kSteps; n++) st[n] = Step{0, 0, -1, 0, 0, 0};
}
__global__ void kk(const int64_t* cells, int64_t n, Step* st) {
#ifndef HOST_WALK
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
#else
    for (int64_t i = 0; i < n; i++)
#endif
        walk1((uint64_t)cells[i], st + i * kSteps);
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
    std::vector<Step> st((size_t)n * kSteps);
#ifndef HOST_WALK
    int64_t* dc;
    Step* ds;
    if (hipMalloc(&dc, n * 8) || hipMalloc(&ds, n * kSteps * sizeof(Step))) return 2;
    if (hipMemcpy(dc, cells.data(), n * 8, hipMemcpyHostToDevice)) return 2;
    kk<<<(unsigned)((n + 255) / 256), 256>>>(dc, n, ds);
    if (hipDeviceSynchronize() || hipMemcpy(st.data(), ds, n * kSteps * sizeof(Step), hipMemcpyDeviceToHost)) return 3;
#else
    kk(cells.data(), n, st.data());
#endif
    for (int64_t i = 0; i < n; i++)
        for (int k = 0; k < kSteps; k++) {
            const Step& s = st[(size_t)(i * kSteps + k)];
            printf("%ld %d %d %llu %d %llu %d\n", (long)i, k, s.dir, s.in, s.rot_in, s.out, s.rot_out);
        }
    return 0;
}
