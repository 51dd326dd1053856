// CPU self-check: mosaic_amd/csrc/bng_device.h kring / kloop (the GPU code, compiled for the host)
// against the oracle restatement (oracle/bng.c) on 20,000 cells of every resolution, k = 0..4,
// inside and outside the grid.  Prints "<cases> <mismatches>".
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include "bng_device.h"
extern "C" {
int oracle_bng_kloop(int64_t id, int k, int64_t* out);
int oracle_bng_kring(int64_t id, int n, int64_t* out);
int64_t oracle_bng_point_to_index(double e, double n, int res, int* err);
}
int main() {
    srand(3);
    int res_list[12] = {-1, 1, -2, 2, -3, 3, -4, 4, -5, 5, -6, 6};
    long bad = 0, tot = 0;
    static int64_t a[20000], b[20000];
    for (int t = 0; t < 20000; t++) {
        int res = res_list[t % 12];
        double e = -20000 + 740000.0 * rand() / RAND_MAX, n = -20000 + 1340000.0 * rand() / RAND_MAX;
        int err = 0;
        int64_t c = oracle_bng_point_to_index(e, n, res, &err);
        for (int k = 0; k < 5; k++) {
            int m1 = mosaic::bng::kring(c, k, a), m2 = oracle_bng_kring(c, k, b);
            tot++;
            bool same = m1 == m2;
            for (int i = 0; same && i < m1; i++) same = a[i] == b[i];
            if (!same) { if (bad < 5) printf("diff id %lld k %d m %d %d\n", (long long)c, k, m1, m2); bad++; }
        }
    }
    printf("%ld %ld\n", tot, bad);
}
