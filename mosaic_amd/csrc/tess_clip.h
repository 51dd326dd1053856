// k_tess_clip_ll (tess_clip.hip): the device side of the reference-style border chips (llclip.h) for
// mosaic_tessellate_gpu, one lane per border candidate.  HIP-only declarations shared by
// tess_clip.hip and the host orchestration in mosaic_hip.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "llclip.h"
#include "tess_gpu.h"

namespace mosaic {
namespace tessll {

// per-lane workspace (chains of the ring walks, result rings); a task needing more goes to the host
static constexpr int kLLChains = 24, kLLOut = 12;

struct ClipLLArgs {
    const double* gxy;  // the geometries' rings in output coordinates (lon / lat degrees, BNG metres)
    const int64_t *ring_offsets, *part_rings, *geom_parts;
    const int32_t* cand_geom;
    const int64_t* cand_id;  // mode 0: the candidates' H3 ids (the cell polygon is h3ToGeoBoundary)
    const double* clip;      // mode 1: explicit cell polygons, nv vertices per candidate (ccw, open)
    int nv, mode;
    const int64_t* tasks;  // the border candidates
    int64_t n_tasks;
    llclip::Chain* wch;  // kLLChains per lane
    llclip::Out* wout;   // kLLOut per lane
    double* out;         // result vertices (interleaved)
    unsigned long long* counters;  // [0] vertices, [1] rings, [2] polygons
    int64_t out_cap, ring_cap, part_cap;
    tessclip::ClipRing* rings;
    tessclip::ClipPart* parts;
    uint8_t* status;  // per task: 0 chip written (or none), 1 to the host, 2 written and equal to the cell
    const double* blk;         // ring indexes (llclip::Geom; null: none)
    const int64_t* ring_blk;
    const uint8_t* ring_ccw;
};

// launch over `lanes` lanes (grid-stride over the tasks)
hipError_t launch_clip_ll(const ClipLLArgs& a, int64_t lanes, hipStream_t stream);
// the ring indexes of rings [0, n_rings) (llclip::ring_blocks_one, one lane per ring); ring_blk given
hipError_t launch_ring_blocks(const int64_t* ro, const double* xy, int64_t n_rings, const int64_t* ring_blk, double* blk,
                              uint8_t* ccw, hipStream_t stream);

// layout fingerprint of the records mosaic_hip.hip and tess_clip.hip share (join_binned.h's rationale)
static constexpr uint64_t layout_fingerprint() {
    uint64_t h = 0xcbf29ce484222325ULL;
    for (uint64_t v : {(uint64_t)sizeof(ClipLLArgs), (uint64_t)sizeof(llclip::Chain), (uint64_t)sizeof(llclip::Out),
                       (uint64_t)sizeof(tessclip::ClipRing), (uint64_t)sizeof(tessclip::ClipPart),
                       (uint64_t)offsetof(ClipLLArgs, status), (uint64_t)kLLChains, (uint64_t)kLLOut})
        h = h * 0x100000001b3ULL ^ v;
    return h;
}

}  // namespace tessll
}  // namespace mosaic
