// Border-chip clipping of mosaic_tessellate_gpu on the GPU (k_tess_clip in mosaic_hip.hip), shared by
// the host side of the producer (tessellate.cpp, g++) and the device side (hipcc).  The kernel runs
// tessellate.cpp's emit_cell border branch -- Sutherland-Hodgman of every ring of the candidate's
// geometry against the cell's convex clip polygon, the degenerate-ring and net-area tests, the
// mapping of computed vertices back to output coordinates (original vertices kept exact) -- with
// the same arithmetic, so the chips are identical byte for byte; the host writes the WKB.
#pragma once
#include <stdint.h>

#include <vector>

struct mosaic_ctx;

namespace mosaic {
namespace tessclip {

struct ClipRing {  // one kept output ring (closed: n vertices, the first repeated last)
    int64_t cand;
    int32_t part, ring;  // part and ring index within the candidate's geometry
    int64_t off;         // first vertex in ClipResult::verts (vertex units)
    int32_t n;
    int32_t pad;
};
struct ClipPart {  // a part that produced rings: kept when its net area > area_eps
    int64_t cand;
    int32_t part, keep;
};
struct ClipResult {
    std::vector<uint8_t> redo;  // per task: 1 = the kernel ran out of scratch / output; clip on the host
    std::vector<ClipRing> rings;
    std::vector<ClipPart> parts;
    std::vector<double> verts;  // output coordinates, interleaved
    double kernel_ms = 0;
};

// mode 0: H3 -- rings in the face plane (pxy), computed vertices mapped to lon / lat through the
// geometry's face (gface) at resolution res; mode 1: identity (BNG metres).  tasks: the border
// candidates to clip; clip: nv vertices per candidate (counter-clockwise, open).
int clip_border(mosaic_ctx* ctx, int64_t n_geoms, const int64_t* geom_parts, const int64_t* part_rings,
                const int64_t* ring_offsets, const double* pxy, const double* gxy, const int32_t* gface, int res, int mode,
                int64_t n_tasks, const int64_t* tasks, const int32_t* cand_geom, int64_t n_cand, const double* clip, int nv,
                double area_eps, ClipResult* out);

// mosaic_tessellate_gpu's H3 branch as one device session (mosaic_hip.hip): the geometry batch (rings
// in the face plane and in lon / lat, each geometry's face) is uploaded once; per chunk of candidates
// (geometry, face-plane centre) the hexagon clip polygons (D pieces per side, corner offsets dx / dy)
// are generated on the device, classified (cls: 0 dropped, 1 core, 2 border) and the border ones
// clipped (tasks: their candidate indices; out as clip_border's).
struct H3Session;
int h3_session_begin(mosaic_ctx* ctx, int64_t n_geoms, const int64_t* geom_parts, const int64_t* part_rings,
                     const int64_t* ring_offsets, const double* pxy, const double* gxy, const int32_t* gface, int res, int D,
                     const double* dx, const double* dy, H3Session** out);
// clip_xy / clip_n / nv_max: explicit clip polygons instead of the hexagons of cxy (the per-face
// pieces of cells of face-spanning geometries): clip_n[k] open counter-clockwise vertices of
// candidate k at clip_xy + 2 nv_max k.
int h3_session_chunk(H3Session* s, int64_t n_cand, const int32_t* cand_geom, const double* cxy, double eps,
                     double area_eps, uint8_t* cls, std::vector<int64_t>& tasks, ClipResult* out,
                     const double* clip_xy = nullptr, const int32_t* clip_n = nullptr, int nv_max = 0);
void h3_session_end(H3Session* s);

}  // namespace tessclip
}  // namespace mosaic
