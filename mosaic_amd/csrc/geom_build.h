// Host-side decoding of chip / geometry WKB into the flat ring layout of pip_device.h.
// Accepts what JTS WKBReader accepts for the chip column (MosaicGeometryJTS.scala:147, 200):
// Polygon (3) and MultiPolygon (6), either byte order, ISO Z/M (1000/2000/3000) and EWKB
// (Z/M/SRID flag bits) variants; Z and M ordinates are skipped.  Zero-length input means "no
// geometry" (a null wkb / a core chip with keepCoreGeom = false) and decodes to an empty geometry.
#pragma once
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <limits>
#include <string>
#include <vector>

#include "pip_device.h"

namespace mosaic {

struct GeomBuilder {
    std::vector<pip::Vec2> verts;
    std::vector<uint32_t> ring_start{0};
    std::vector<pip::Box> ring_bbox;
    std::vector<uint32_t> part_ring{0};
    std::vector<uint32_t> geom_part{0};
    std::vector<pip::Box> geom_bbox;
    std::string error;

    struct Reader {
        const uint8_t* p;
        size_t len, pos;
        bool fail = false;
        uint8_t u8() {
            if (pos + 1 > len) {
                fail = true;
                return 0;
            }
            return p[pos++];
        }
        uint32_t u32(bool le) {
            if (pos + 4 > len) {
                fail = true;
                return 0;
            }
            const uint8_t* b = p + pos;
            pos += 4;
            return le ? (uint32_t)b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16 | (uint32_t)b[3] << 24
                      : (uint32_t)b[3] | (uint32_t)b[2] << 8 | (uint32_t)b[1] << 16 | (uint32_t)b[0] << 24;
        }
        double f64(bool le) {
            if (pos + 8 > len) {
                fail = true;
                return 0;
            }
            uint64_t u = 0;
            for (int i = 0; i < 8; i++) u |= (uint64_t)p[pos + (le ? i : 7 - i)] << (8 * i);
            pos += 8;
            double d;
            memcpy(&d, &u, 8);
            return d;
        }
    };

    static bool header(Reader& r, bool& le, uint32_t& type, int& dims) {
        uint8_t bo = r.u8();
        if (r.fail || bo > 1) return false;
        le = bo == 1;
        uint32_t t = r.u32(le);
        if (r.fail) return false;
        bool z = t & 0x80000000u, m = t & 0x40000000u, srid = t & 0x20000000u;
        t &= 0x0fffffffu;
        if (t >= 3000) {
            z = m = true;
            t -= 3000;
        } else if (t >= 2000) {
            m = true;
            t -= 2000;
        } else if (t >= 1000) {
            z = true;
            t -= 1000;
        }
        if (srid) r.u32(le);
        type = t;
        dims = 2 + (z ? 1 : 0) + (m ? 1 : 0);
        return !r.fail;
    }

    bool polygon(Reader& r, bool le, int dims) {
        uint32_t nrings = r.u32(le);
        if (r.fail) return false;
        for (uint32_t k = 0; k < nrings; k++) {
            uint32_t npts = r.u32(le);
            if (r.fail || (uint64_t)npts * 8 * dims > r.len - r.pos) return false;
            pip::Box b = {INFINITY, INFINITY, -INFINITY, -INFINITY};
            for (uint32_t i = 0; i < npts; i++) {
                double x = r.f64(le), y = r.f64(le);
                for (int d = 2; d < dims; d++) r.f64(le);
                verts.push_back({x, y});
                b.minx = std::min(b.minx, x);
                b.maxx = std::max(b.maxx, x);
                b.miny = std::min(b.miny, y);
                b.maxy = std::max(b.maxy, y);
            }
            ring_bbox.push_back(b);
            ring_start.push_back((uint32_t)verts.size());
        }
        part_ring.push_back((uint32_t)ring_bbox.size());
        return !r.fail;
    }

    // Appends one geometry; returns false (and sets error) on malformed input.
    bool add(const uint8_t* wkb, size_t len) {
        size_t v0 = verts.size();
        if (len > 0) {
            Reader r{wkb, len, 0};
            bool le;
            uint32_t type;
            int dims;
            bool ok = header(r, le, type, dims);
            if (ok && type == 3) {
                ok = polygon(r, le, dims);
            } else if (ok && type == 6) {
                uint32_t nparts = r.u32(le);
                ok = !r.fail;
                for (uint32_t p = 0; ok && p < nparts; p++) {
                    bool le2;
                    uint32_t t2;
                    int d2;
                    ok = header(r, le2, t2, d2) && t2 == 3 && polygon(r, le2, d2);
                }
            } else if (ok) {
                error = "unsupported WKB geometry type " + std::to_string(type) + " (Polygon/MultiPolygon expected)";
                return false;
            }
            if (!ok) {
                error = "malformed WKB";
                return false;
            }
            if (verts.size() > std::numeric_limits<uint32_t>::max()) {
                error = "too many vertices";
                return false;
            }
        }
        geom_part.push_back((uint32_t)(part_ring.size() - 1));
        pip::Box b = {INFINITY, INFINITY, -INFINITY, -INFINITY};
        for (size_t i = v0; i < verts.size(); i++) {
            b.minx = std::min(b.minx, verts[i].x);
            b.maxx = std::max(b.maxx, verts[i].x);
            b.miny = std::min(b.miny, verts[i].y);
            b.maxy = std::max(b.maxy, verts[i].y);
        }
        geom_bbox.push_back(b);
        return true;
    }
};

}  // namespace mosaic
