#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
extern int g_mode, g_cr, g_dr, g_da, g_dth, g_dump;
int oracle_h3_to_geo_boundary(int64_t h3, double* out);
int main(int argc, char** argv) {
    g_mode = atoi(argv[1]); g_dump = getenv("DUMP") != 0; g_cr = argc > 2 ? atoi(argv[2]) : 0; g_dr = argc > 3 ? atoi(argv[3]) : 0; g_da = argc > 4 ? atoi(argv[4]) : 0; g_dth = argc > 5 ? atoi(argv[5]) : 0;
    long long c;
    while (scanf("%lld", &c) == 1) {
        double b[20];
        int n = oracle_h3_to_geo_boundary(c, b);
        printf("%lld %d", c, n);
        for (int i = 0; i < n; i++) printf(" %a %a", b[2*i+1], b[2*i]);
        printf("\n");
    }
}
