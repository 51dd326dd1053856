// Microbenchmark (GPU box): cost of random 4-byte gathers on gfx950 as a function of the share of
// lanes that gather a distinct line, and of how the others are handled (same-address dummy lane vs
// exec-masked).  Prints ms per launch and cycles per gather instruction per CU.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/gp tools/probes/gather_probe.hip && /tmp/gp
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ inline uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

// mode 0: inactive lanes read table[0] (dummy, same address); mode 1: inactive lanes exec-masked
template <int MODE>
__global__ void __launch_bounds__(256) k_gather(const uint32_t* t, uint32_t mask, int iters, uint32_t active_per_64,
                                                uint32_t* out) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t acc = 0, s = blockIdx.x * 256 + threadIdx.x;
    for (int it = 0; it < iters; it++) {
        uint32_t v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            uint32_t h = hash32(s * 4 + k + it * 0x9e3779b9u);
            bool act = ((h >> 24) & 63) < active_per_64;
            if (MODE == 0) {
                v[k] = t[act ? (h & mask) : 0];
            } else {
                v[k] = act ? t[h & mask] : 0u;
            }
        }
        acc += v[0] ^ v[1] ^ v[2] ^ v[3];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const size_t sizes[2] = {(size_t)1 << 19, (size_t)1 << 23};  // 2 MiB, 32 MiB tables
    uint32_t *t, *out;
    hipMalloc(&t, sizes[1] * 4);
    hipMemset(t, 1, sizes[1] * 4);
    hipMalloc(&out, 4);
    int cus = 256;
    const int blocks = cus * 8, iters = 256;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int si = 0; si < 2; si++) {
        for (int mode = 0; mode < 2; mode++) {
            for (uint32_t act : {64u, 32u, 16u, 4u, 0u}) {
                float best = 1e30f;
                for (int rep = 0; rep < 4; rep++) {
                    hipEventRecord(a);
                    if (mode == 0)
                        hipLaunchKernelGGL(k_gather<0>, dim3(blocks), dim3(256), 0, 0, t, (uint32_t)sizes[si] - 1, iters, act, out);
                    else
                        hipLaunchKernelGGL(k_gather<1>, dim3(blocks), dim3(256), 0, 0, t, (uint32_t)sizes[si] - 1, iters, act, out);
                    hipEventRecord(b);
                    hipEventSynchronize(b);
                    float ms;
                    hipEventElapsedTime(&ms, a, b);
                    if (rep && ms < best) best = ms;
                }
                // gather instructions per CU: waves per CU (32) * iters * 4
                double instr_per_cu = 32.0 * iters * 4;
                printf("table %4zu MiB  mode %-6s active %2u/64: %.3f ms  %.1f cyc/instr/CU (2.4 GHz)\n",
                       sizes[si] * 4 >> 20, mode ? "masked" : "dummy", act, best,
                       best * 1e-3 * 2.4e9 / instr_per_cu);
            }
        }
    }
    return 0;
}
