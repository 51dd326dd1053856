// Derivation probe for tools/h3gen.py (not part of the engine): the faceIjkBaseCells rotation of
// each pentagon base cell on each of the five faces around its vertex, fixed by H3's round-trip
// invariant geoToH3(h3ToGeo(h)) == h over every valid cell of the base cell at res 1-4.  h3ToGeo
// does not read that table for pentagons (home frame + overage), so it is the independent side.
// Prints, per (pentagon, face, corner), the rotations every such cell agrees with.
//   g++ -O2 -std=c++17 -ffp-contract=off -I mosaic_amd/csrc tools/probes/pent_rot_probe.cpp -o /tmp/prp
#include <stdint.h>
#include <stdio.h>

#include <map>
#include <set>
#include <vector>

#include "h3_device.h"
#include "h3_geom.h"

using namespace mosaic;
using namespace mosaic::h3;

static void geo_face_ijk(double lat, double lon, int res, int* face_out, IJK* ijk_out) {
    double pz, r0, slon, clon;
    glibc::sincos(lat, &pz, &r0);
    glibc::sincos(lon, &slon, &clon);
    double px = clon * r0, py = slon * r0;
    int face = 0;
    double sqd = sq(kH3FaceCenterPoint[0][0] - px) + sq(kH3FaceCenterPoint[0][1] - py) + sq(kH3FaceCenterPoint[0][2] - pz);
    for (int f = 1; f < 20; f++) {
        double t = sq(kH3FaceCenterPoint[f][0] - px) + sq(kH3FaceCenterPoint[f][1] - py) + sq(kH3FaceCenterPoint[f][2] - pz);
        if (t < sqd) {
            face = f;
            sqd = t;
        }
    }
    double vx, vy;
    double r = glibc::acos(1 - sqd / 2);
    if (r < H3LD_EPSILON_DUP) {
        vx = vy = 0.0;
    } else {
        double lat1 = kH3FaceCenterGeo[face][0], lon1 = kH3FaceCenterGeo[face][1];
        double sdl, cdl, slat1, clat1;
        glibc::sincos(lon - lon1, &sdl, &cdl);
        glibc::sincos(lat1, &slat1, &clat1);
        double az = glibc::atan2(r0 * sdl, clat1 * pz - slat1 * r0 * cdl);
        double theta = pos_angle_rads(kH3FaceAxesAzRadsCII[face][0] - pos_angle_rads(az));
        if (res & 1) theta = pos_angle_rads(x87::add_ld(theta, H3LD_M_AP7_ROT_RADS_M, H3LD_M_AP7_ROT_RADS_E, true));
        r = glibc::tan(r);
        r /= kRes0UGnomonic;
        for (int i = 0; i < res; i++) r = x87::mul_ld(r, H3LD_M_SQRT7_M, H3LD_M_SQRT7_E);
        double st, ct;
        glibc::sincos(theta, &st, &ct);
        vx = r * ct;
        vy = r * st;
    }
    double a1 = fabs(vx), a2 = fabs(vy);
    double x2 = x87::div_ld(a2, H3LD_M_SIN60_M, H3LD_M_SIN60_E);
    *ijk_out = hex2d_round(vx, vy, a1, x2);
    *face_out = face;
}

// face_ijk_to_h3 with the pentagon's rotation count given
static uint64_t to_h3_rot(int face, IJK ijk, int res, int rots, int* bc_out, IJK* base_ijk) {
    uint64_t h = 0x00001fffffffffffULL | (1ULL << 59) | ((uint64_t)res << 52);
    for (int r = res - 1; r >= 0; r--) {
        IJK last = ijk, c;
        int i = ijk.i - ijk.k, j = ijk.j - ijk.k;
        if ((r + 1) & 1) {
            ijk.i = round_div7(3 * i - j);
            ijk.j = round_div7(i + 2 * j);
            ijk.k = 0;
            ijk_normalize(ijk);
            c.i = 3 * ijk.i + ijk.j;
            c.j = 3 * ijk.j + ijk.k;
            c.k = ijk.i + 3 * ijk.k;
        } else {
            ijk.i = round_div7(2 * i + j);
            ijk.j = round_div7(3 * j - i);
            ijk.k = 0;
            ijk_normalize(ijk);
            c.i = 3 * ijk.i + ijk.k;
            c.j = ijk.i + 3 * ijk.j;
            c.k = ijk.j + 3 * ijk.k;
        }
        ijk_normalize(c);
        IJK d = {last.i - c.i, last.j - c.j, last.k - c.k};
        ijk_normalize(d);
        int digit = (d.i <= 1 && d.j <= 1 && d.k <= 1) ? (d.i << 2) | (d.j << 1) | d.k : 7;
        h = set_digit(h, r + 1, digit);
    }
    *base_ijk = ijk;
    if (ijk.i > 2 || ijk.j > 2 || ijk.k > 2) return 0;
    int packed = kH3FaceIjkBaseCells[face][ijk.i][ijk.j][ijk.k];
    int bc = packed >> 3;
    *bc_out = bc;
    h |= (uint64_t)bc << 45;
    if (kH3BaseCellData[bc][4]) {
        if (leading_nonzero_digit(h, res) == 1) {
            bool cw = kH3BaseCellData[bc][5] == face || kH3BaseCellData[bc][6] == face;
            h = rotate_all(h, res, !cw);
        }
        for (int i = 0; i < rots; i++) h = rotate_pent60ccw(h, res);
    }
    return h;
}

int main() {
    const int pents[12] = {4, 14, 24, 38, 49, 58, 63, 72, 83, 97, 107, 117};
    for (int pi = 0; pi < 12; pi++) {
        const int p = pents[pi];
        // (face, corner) -> rotations consistent with every cell seen there
        std::map<std::pair<int, int>, std::set<int>> ok;
        std::map<std::pair<int, int>, int> seen, current;
        for (int res = 1; res <= 4; res++) {
            int nd = 1;
            for (int q = 0; q < res; q++) nd *= 7;
            for (int code = 0; code < nd; code++) {
                uint64_t h = 0x00001fffffffffffULL | (1ULL << 59) | ((uint64_t)res << 52) | ((uint64_t)p << 45);
                int t = code;
                for (int r = res; r >= 1; r--) {
                    h = set_digit(h, r, t % 7);
                    t /= 7;
                }
                if (leading_nonzero_digit(h, res) == 1) continue;
                double lat, lon;
                if (!h3geom::h3_to_geo(h, &lat, &lon)) continue;
                int face;
                IJK ijk;
                geo_face_ijk(lat, lon, res, &face, &ijk);
                int bc;
                IJK bijk;
                std::set<int> good;
                for (int rots = 0; rots < 6; rots++)
                    if (to_h3_rot(face, ijk, res, rots, &bc, &bijk) == h) good.insert(rots);
                if (bc != p) continue;  // (the centre rounds into another base cell: not this table entry)
                const int corner = bijk.i == 2 ? 0 : (bijk.j == 2 ? 1 : 2);
                auto key = std::make_pair(face, corner);
                current[key] = kH3FaceIjkBaseCells[face][bijk.i][bijk.j][bijk.k] & 7;
                if (!seen[key]++) ok[key] = good;
                else {
                    std::set<int> x;
                    for (int v : ok[key])
                        if (good.count(v)) x.insert(v);
                    ok[key] = x;
                }
            }
        }
        printf("pentagon %3d:", p);
        for (auto& kv : ok) {
            printf("  face %2d corner %d (cells %4d) table %d ok {", kv.first.first, kv.first.second, seen[kv.first], current[kv.first]);
            for (int v : kv.second) printf("%d", v);
            printf("}");
        }
        printf("\n");
    }
    return 0;
}
