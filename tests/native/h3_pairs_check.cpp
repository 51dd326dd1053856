// CPU check of h3_device.h's two-level and four-level digit steps (face_axial_to_h3 with kAxialPairs,
// face_axial_to_h3_quad with kAxialQuads) against the one-level form (face_axial_to_h3_levels): every res 0..15 on every face, axial coordinates over the face's
// range (a dense block around the origin and random samples out to the res-15 face radius).  Prints
// the number of inputs and of differences.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>

#include "h3_device.h"

static int check(int face, int a, int b, int res) {
    const uint64_t want = mosaic::h3::face_axial_to_h3_levels(face, a, b, res);
    return (mosaic::h3::face_axial_to_h3(face, a, b, res) != want) +
           (mosaic::h3::face_axial_to_h3_quad(face, a, b, res, mosaic::h3::kAxialQuads.v[res & 1]) != want);
}

int main(int argc, char** argv) {
    const long n_rand = argc > 1 ? atol(argv[1]) : 1000000;
    long n = 0, bad = 0;
    std::mt19937_64 rng(7);
    for (int res = 0; res <= 15; res++) {
        // face radius in res-`res` hex units: ~ 3 x sqrt(7)^res (generous)
        double rad = 3.0;
        for (int k = 0; k < res; k++) rad *= 2.6457513110645907;
        const int lim = (int)(rad < 1e7 ? rad : 1e7);
        for (int face = 0; face < 20; face++) {
            for (int a = -60; a <= 60; a++)
                for (int b = -60; b <= 60; b++) {
                    n++;
                    bad += check(face, a, b, res);
                }
            std::uniform_int_distribution<int> u(-lim, lim);
            for (long t = 0; t < n_rand / 320; t++) {
                const int a = u(rng), b = u(rng);
                n++;
                bad += check(face, a, b, res);
            }
        }
    }
    printf("%ld %ld\n", n, bad);
    return 0;
}
