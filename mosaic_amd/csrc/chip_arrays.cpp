// The array form of the chip join's build side: PointInPolygonJoin.joinArrayRows
// (sql/join/PointInPolygonJoin.scala:39-66) joins a point to a polygon row when the row's chip array
// (grid_tessellate / MosaicFill output, struct<chips: array<struct<is_core, index_id, wkb>>>) holds
// the point's cell, and then tests only the FIRST chip with that cell (array_position +
// element_at): at most one pair per (point, polygon row).  The exploded form (joinExplodedRows,
// :68-84) tests every chip row.  So the array form is the exploded join over the chip arrays with
// each row's later duplicates of a cell removed -- which is what this wrapper builds before handing
// the rows to mosaic_chip_table_create.
#include <stdint.h>

#include <string>
#include <unordered_set>
#include <vector>

#include "../../include/mosaic_hip.h"

extern "C" int mosaic_tess_fail(int code, const char* msg);  // defined in mosaic_hip.hip

extern "C" int mosaic_chip_table_create_arrays(mosaic_ctx* ctx, int grid, int res, int32_t n_polygons,
                                               const int64_t* chip_offsets, const uint8_t* is_core,
                                               const int64_t* index_id, const int64_t* wkb_offsets,
                                               const uint8_t* wkb, mosaic_chips** out) {
    if (!ctx || !out || n_polygons < 0 || (n_polygons > 0 && !chip_offsets))
        return mosaic_tess_fail(MOSAIC_E_ARG, "invalid argument");
    const int64_t n = n_polygons > 0 ? chip_offsets[n_polygons] - chip_offsets[0] : 0;
    if (n < 0) return mosaic_tess_fail(MOSAIC_E_ARG, "chip_offsets must be non-decreasing");
    if (n > 0 && (!is_core || !index_id || !wkb_offsets)) return mosaic_tess_fail(MOSAIC_E_ARG, "invalid argument");
    const int64_t base = n_polygons > 0 ? chip_offsets[0] : 0;
    std::vector<uint8_t> core;
    std::vector<int64_t> ids, offs{0};
    std::vector<int32_t> keys;
    std::vector<uint8_t> bytes;
    core.reserve(n);
    ids.reserve(n);
    keys.reserve(n);
    offs.reserve(n + 1);
    std::unordered_set<int64_t> seen;
    for (int32_t p = 0; p < n_polygons; p++) {
        if (chip_offsets[p + 1] < chip_offsets[p]) return mosaic_tess_fail(MOSAIC_E_ARG, "chip_offsets must be non-decreasing");
        seen.clear();
        for (int64_t i = chip_offsets[p]; i < chip_offsets[p + 1]; i++) {
            if (!seen.insert(index_id[i]).second) continue;  // array_position finds the first chip of the cell
            core.push_back(is_core[i]);
            ids.push_back(index_id[i]);
            keys.push_back(p);
            const int64_t a = wkb_offsets[i - base], b = wkb_offsets[i - base + 1];
            if (b < a) return mosaic_tess_fail(MOSAIC_E_ARG, "wkb_offsets must be non-decreasing");
            bytes.insert(bytes.end(), wkb + a, wkb + b);
            offs.push_back((int64_t)bytes.size());
        }
    }
    return mosaic_chip_table_create(ctx, grid, res, (int64_t)ids.size(), core.data(), ids.data(), offs.data(),
                                    bytes.data(), keys.data(), n_polygons, out);
}
