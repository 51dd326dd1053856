// CPU self-check: mosaic_amd/csrc/bng_device.h format_id (the GPU formatter, compiled for the host)
// against the oracle's BNGIndexSystem.format restatement (oracle/bng.c) on ids of every resolution
// from points in and around the grid, plus short / malformed ids.  Prints "<cases> <mismatches>".
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "bng_device.h"
extern "C" {
int oracle_bng_format(int64_t id, char* buf, int cap);
int64_t oracle_bng_point_to_index(double e, double n, int res, int* err);
}
static long bad = 0, tot = 0;
static void check(int64_t id) {
    char a[64], b[64];
    int la = mosaic::bng::format_id(id, a);
    int lb = oracle_bng_format(id, b, 64);
    tot++;
    bool same = (la < 0 && lb < 0) || (la == lb && memcmp(a, b, (size_t)la) == 0);
    if (!same) {
        if (bad < 5) printf("diff id %lld: %d %d\n", (long long)id, la, lb);
        bad++;
    }
}
int main() {
    srand(7);
    int res_list[12] = {-1, 1, -2, 2, -3, 3, -4, 4, -5, 5, -6, 6};
    for (int t = 0; t < 60000; t++) {
        int res = res_list[t % 12];
        double e = -20000 + 740000.0 * rand() / RAND_MAX, n = -20000 + 1340000.0 * rand() / RAND_MAX;
        int err = 0;
        check(oracle_bng_point_to_index(e, n, res, &err));
    }
    const int64_t odd[] = {1, 12, 123, 1234, 10501, 1050138794LL, 1100438790LL, 99999999999LL, 1999, 15000};
    for (int64_t id : odd) check(id);
    printf("%ld %ld\n", tot, bad);
}
