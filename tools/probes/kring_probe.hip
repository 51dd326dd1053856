// GPU probe: H3 hexRange steps (h3_neighbors.h) for one cell, device vs host, step by step.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../mosaic_amd/csrc/h3_neighbors.h"
using namespace mosaic;
struct Step { unsigned long long in, out; int dir, rot_in, rot_out; };
__host__ __device__ int walk(uint64_t origin, int k, Step* st) {
    int n = 0, ring = 1, dir = 0, i = 0, rotations = 0;
    while (ring <= k && n < 60) {
        if (dir == 0 && i == 0) {
            Step& s = st[n++]; s.in = origin; s.dir = h3nb::kNextRing; s.rot_in = rotations;
            origin = h3nb::neighbor_rotations(origin, h3nb::kNextRing, &rotations);
            s.out = origin; s.rot_out = rotations;
        }
        Step& s = st[n++]; s.in = origin; s.dir = h3nb::direction(dir); s.rot_in = rotations;
        origin = h3nb::neighbor_rotations(origin, h3nb::direction(dir), &rotations);
        s.out = origin; s.rot_out = rotations;
        if (++i == ring) { i = 0; if (++dir == 6) { dir = 0; ring++; } }
    }
    return n;
}
__global__ void kk(uint64_t c, int k, Step* st, int* n, int64_t* fast) {
    *n = walk(c, k, st);
    fast[0] = h3nb::kring_fast(c, k, 0, fast + 1);
}
int main() {
    const uint64_t c = 632242071332407807ULL;
    Step* d; int* dn; int64_t* df;
    hipMalloc(&d, 64 * sizeof(Step)); hipMalloc(&dn, 4); hipMalloc(&df, 64 * 8);
    kk<<<1, 1>>>(c, 1, d, dn, df);
    Step hs[64], gs[64]; int gn; int64_t gf[64];
    hipMemcpy(gs, d, sizeof(gs), hipMemcpyDeviceToHost); hipMemcpy(&gn, dn, 4, hipMemcpyDeviceToHost);
    hipMemcpy(gf, df, sizeof(gf), hipMemcpyDeviceToHost);
    int hn = walk(c, 1, hs);
    printf("host steps %d gpu steps %d gpu kring_fast %ld\n", hn, gn, gf[0]);
    for (int i = 0; i < gn && i < hn; i++)
        printf("%2d dir %d in %llu rot %d -> host %llu rot %d | gpu %llu rot %d%s\n", i, hs[i].dir, hs[i].in, hs[i].rot_in,
               hs[i].out, hs[i].rot_out, gs[i].out, gs[i].rot_out, (hs[i].out != gs[i].out || hs[i].rot_out != gs[i].rot_out) ? "  <<<" : "");
    return 0;
}
