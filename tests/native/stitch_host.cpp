// CPU wrapper of isect_geom.cpp (the host stitching of st_intersection_aggregate's per-cell
// boundaries into WKB) for tests/test_intersection_agg.py.
#include <string.h>

#include "isect_geom.h"

// returns the WKB size (written to out when <= cap), -1 when the edges do not close into rings
extern "C" long stitch_host(const double* edges, long n, double snap, unsigned char* out, long cap, double* area) {
    std::vector<uint8_t> w;
    if (!mosaic::isect_geom::stitch_wkb(edges, (size_t)n, snap, w, area)) return -1;
    if ((long)w.size() <= cap) memcpy(out, w.data(), w.size());
    return (long)w.size();
}
