// Border-chip clipping of mosaic_tessellate_gpu on the GPU (k_tess_clip_ll in tess_clip.hip, the
// reference-style clip of llclip.h), shared by the host side of the producer (tessellate.cpp, g++) and
// the device side (hipcc): result records the kernel writes and tessellate.cpp turns into WKB.
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
    std::vector<uint8_t> status;  // per task: 0 done (chip or none), 1 clip on the host, 2 done and equal to the cell
    std::vector<ClipRing> rings;
    std::vector<ClipPart> parts;
    std::vector<double> verts;  // output coordinates, interleaved
    double kernel_ms = 0;
};

// The border candidates `tasks` of explicit cell polygons (clip: nv vertices per candidate,
// counter-clockwise, open; BNG squares) clipped on the device against geometries in output
// coordinates (xy).
int clip_ll(mosaic_ctx* ctx, int64_t n_geoms, const int64_t* geom_parts, const int64_t* part_rings,
            const int64_t* ring_offsets, const double* xy, const std::vector<int64_t>& tasks, const int32_t* cand_geom,
            int64_t n_cand, const double* clip, int nv, ClipResult* out);

// mosaic_tessellate_gpu's H3 branch as one device session (mosaic_hip.hip): the geometry batch (rings
// in the face plane and in lon / lat, each geometry's face) is uploaded once; per chunk of candidates
// (geometry, face-plane centre, H3 id) the hexagon clip polygons (D pieces per side, corner offsets
// dx / dy) are generated on the device and classified in the face plane (cls: 0 dropped, 1 core,
// 2 border); the border ones are clipped in lon / lat against their cells' boundaries (tasks: their
// candidate indices; out as clip_ll's).
struct H3Session;
int h3_session_begin(mosaic_ctx* ctx, int64_t n_geoms, const int64_t* geom_parts, const int64_t* part_rings,
                     const int64_t* ring_offsets, const double* pxy, const double* gxy, const int32_t* gface, int res, int D,
                     const double* dx, const double* dy, H3Session** out);
// cand_id == nullptr: classification only.  clip_xy / clip_n / nv_max: explicit clip polygons
// instead of the hexagons of cxy (the per-face pieces of cells of face-spanning geometries): clip_n[k]
// open counter-clockwise vertices of candidate k at clip_xy + 2 nv_max k.
int h3_session_chunk(H3Session* s, int64_t n_cand, const int32_t* cand_geom, const double* cxy, double eps, uint8_t* cls,
                     std::vector<int64_t>& tasks, ClipResult* out, const int64_t* cand_id,
                     const double* clip_xy = nullptr, const int32_t* clip_n = nullptr, int nv_max = 0);
// h3ToGeoBoundary of cells on the device (JDK 8 toDegrees, (lng, lat) degrees): v gets 20 doubles per id,
// cnt the vertex count (0: not a valid cell) -- the core chips' geometry, which costs ~56 us per cell
// on the host (x87-exact steps emulated)
int h3_cell_vertices(H3Session* s, const std::vector<int64_t>& ids, std::vector<double>& v, std::vector<int32_t>& cnt);
void h3_session_end(H3Session* s);

}  // namespace tessclip
}  // namespace mosaic
