// Probe (not the product): statistics of the binned join's tile images (tile_images.h) for a chip
// set in chips.bin format (tools/probes/images/dump_chips.py): per record chips, how many keep
// their vertices in the image, and the image's word budget by part.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <unordered_map>
#include <vector>

#include "../../../mosaic_amd/csrc/geom_build.h"
#include "../../../mosaic_amd/csrc/tile_images.h"
#include "../../../mosaic_amd/csrc/tiles_build.cpp"

using namespace mosaic;

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    int32_t res = 0;
    uint32_t nchips = 0;
    if (fread(&res, 4, 1, f) != 1 || fread(&nchips, 4, 1, f) != 1) return 2;
    struct Row {
        int64_t cell;
        uint8_t core;
        int32_t key;
        std::vector<uint8_t> wkb;
    };
    std::vector<Row> rows(nchips);
    for (auto& r : rows) {
        uint32_t len = 0;
        if (fread(&r.cell, 8, 1, f) != 1 || fread(&r.core, 1, 1, f) != 1 || fread(&r.key, 4, 1, f) != 1 ||
            fread(&len, 4, 1, f) != 1)
            return 2;
        r.wkb.resize(len);
        if (len && fread(r.wkb.data(), 1, len, f) != len) return 2;
    }
    fclose(f);
    std::stable_sort(rows.begin(), rows.end(), [](const Row& a, const Row& b) { return a.cell < b.cell; });
    GeomBuilder gb;
    std::vector<uint32_t> meta(nchips);
    for (uint32_t k = 0; k < nchips; k++) {
        meta[k] = ((uint32_t)rows[k].key << 1) | (rows[k].core ? 1u : 0u);
        if (!gb.add(rows[k].core ? nullptr : rows[k].wkb.data(), rows[k].core ? 0 : rows[k].wkb.size())) return 3;
    }
    std::vector<int64_t> cells;
    std::vector<uint32_t> first, count;
    for (uint32_t k = 0; k < nchips; k++) {
        if (cells.empty() || cells.back() != rows[k].cell) {
            cells.push_back(rows[k].cell);
            first.push_back(k);
            count.push_back(0);
        }
        count.back()++;
    }
    const uint32_t n = (uint32_t)cells.size();
    std::unordered_map<int64_t, int64_t> slot;
    for (uint32_t k = 0; k < n; k++) slot.emplace(cells[k], (int64_t)k);
    auto slot_of = [&](int64_t h) -> int64_t {
        auto it = slot.find(h);
        return it == slot.end() ? -1 : it->second;
    };
    tiles::Builder tb;
    if (!tb.build(res, cells, slot_of)) {
        fprintf(stderr, "not built: %s\n", tb.why);
        printf("0 0 0 0\n");
        return 0;
    }
    binned::ImageSource is;
    is.recs = tb.recs.data();
    is.n_recs = tb.recs.size();
    is.grid = tb.grid;
    is.tile_idx = tb.tile_idx.data();
    is.entries = tb.entries.data();
    is.slot_first = first.data();
    is.slot_count = count.data();
    is.meta = meta.data();
    is.store = pip::GeomStore{gb.verts.data(), gb.ring_start.data(), gb.ring_bbox.data(), gb.part_ring.data(),
                              gb.geom_part.data(), gb.geom_bbox.data()};
    is.threads = 8;
    binned::ImageSet set;
    if (!binned::build_tile_images(is, set)) return 4;
    long images = 0, chips = 0, glob = 0;
    double w_rast = 0, w_chip = 0, w_vert = 0;
    for (size_t k = 0; k < set.off.size(); k++) {
        if (set.off[k] == binned::kNoImage) continue;
        images++;
        const uint32_t* im = set.words.data() + set.off[k];
        chips += im[0];
        for (uint32_t c = 0; c < im[0]; c++)
            if (!(im[im[2] + binned::kImgChipWords * c] & 1u) && (im[im[2] + binned::kImgChipWords * c + 1] >> 16) == binned::kImgGlobal) glob++;
        w_rast += im[2] - im[4];
        w_chip += im[3] - im[2];
        w_vert += 2.0 * im[1];
    }
    printf("records %zu image keys %zu images %ld (levels %u %u %u) chips in images %ld global-ring %ld words %zu max %u\n",
           tb.recs.size(), set.off.size(), images, set.levels[0], set.levels[1], set.levels[2], chips, glob,
           set.words.size(), set.max_words);
    printf("avg words: raster %.0f chips %.0f verts %.0f (cap %u)\n", w_rast / images, w_chip / images, w_vert / images,
           binned::kImgCapWords);
    return 0;
}
