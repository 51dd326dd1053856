// GPU probe: the loop-with-early-return form of H3's leading-nonzero-digit that
// commit ae34561 replaced, in isolation.  Every lane of a wave gets a cell with its first nonzero
// digit at a different position (lanes exit the loop at different iterations); the device result
// is compared with the same function on the host.  Prints mismatches per wave layout.
// Build: hipcc --offload-arch=gfx950 -O3 -save-temps early_exit.hip -o early_exit
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <vector>

__host__ __device__ inline int get_digit(uint64_t h, int r) { return (int)((h >> ((15 - r) * 3)) & 7); }

// the round-3 form (H3 C v3.7 _h3LeadingNonZeroDigit restated)
__host__ __device__ __attribute__((noinline)) int lnz_loop(uint64_t h, int res) {
    for (int r = 1; r <= res; r++) {
        int d = get_digit(h, r);
        if (d) return d;
    }
    return 0;
}

__global__ void k_lnz(const uint64_t* hs, const int* res, int* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = lnz_loop(hs[i], res[i]);
}

// the same, inlined into a caller that branches on the result (as is_valid_cell / the pentagon
// rules did)
__global__ void k_lnz_inl(const uint64_t* hs, const int* res, int* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t h = hs[i];
    int v = 0;
    for (int r = 1; r <= res[i]; r++) {
        const int d = get_digit(h, r);
        if (d) {
            v = d;
            break;
        }
    }
    out[i] = v == 1 ? 100 + v : v;
}

// the pattern of the round-4 failure: a bool returned from inside a divergent loop (is_pentagon's
// "leading digit is 0" through the loop's exit test), inlined into its caller
__device__ inline bool any_nonzero_digit(uint64_t h, int res) {
    for (int r = 1; r <= res; r++)
        if (get_digit(h, r)) return true;
    return false;
}
__global__ void k_any(const uint64_t* hs, const int* res, int* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = any_nonzero_digit(hs[i], res[i]) ? 1 : 0;
}

static uint64_t cell(int res, int first, int digit) {  // digits 1..first-1 zero, digit `first`, rest 3
    uint64_t h = (1ULL << 59) | ((uint64_t)res << 52) | (4ULL << 45);
    for (int r = 1; r <= 15; r++) {
        const uint64_t d = r > res ? 7 : (r < first ? 0 : (r == first ? (uint64_t)digit : 3));
        h |= d << (3 * (15 - r));
    }
    return h;
}

int main() {
    const int n = 64 * 4096;
    std::vector<uint64_t> hs(n);
    std::vector<int> res(n), want(n), want2(n), want3(n);
    for (int i = 0; i < n; i++) {
        const int lane = i & 63, w = i >> 6;
        const int r = 1 + (w + lane) % 15;                   // resolutions vary within the wave
        const int first = 1 + (lane * 7 + w) % (r + 1);      // first nonzero digit position (r + 1: none)
        const int digit = 1 + (lane + w) % 6;
        hs[i] = cell(r, first, digit);
        res[i] = r;
        want[i] = lnz_loop(hs[i], r);
        want2[i] = want[i] == 1 ? 101 : want[i];
        want3[i] = want[i] != 0;
    }
    uint64_t* dh;
    int *dr, *dout;
    hipMalloc(&dh, n * 8);
    hipMalloc(&dr, n * 4);
    hipMalloc(&dout, n * 4);
    hipMemcpy(dh, hs.data(), n * 8, hipMemcpyHostToDevice);
    hipMemcpy(dr, res.data(), n * 4, hipMemcpyHostToDevice);
    std::vector<int> got(n);
    const char* names[3] = {"noinline, return", "inlined, break", "inlined, bool returned from the loop"};
    for (int variant = 0; variant < 3; variant++) {
        if (variant == 0) k_lnz<<<n / 256, 256>>>(dh, dr, dout, n);
        else if (variant == 1) k_lnz_inl<<<n / 256, 256>>>(dh, dr, dout, n);
        else k_any<<<n / 256, 256>>>(dh, dr, dout, n);
        if (hipDeviceSynchronize() != hipSuccess) return 3;
        hipMemcpy(got.data(), dout, n * 4, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int i = 0; i < n; i++) {
            const int w = variant == 0 ? want[i] : (variant == 1 ? want2[i] : want3[i]);
            if (got[i] != w) {
                if (bad < 5) printf("variant %d row %d res %d: device %d host %d\n", variant, i, res[i], got[i], w);
                bad++;
            }
        }
        printf("variant %d (%s): %d of %d rows differ\n", variant, names[variant], bad, n);
    }
    return 0;
}
