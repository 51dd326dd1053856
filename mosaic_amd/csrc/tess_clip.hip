// k_tess_clip_ll: border chips of mosaic_tessellate_gpu the way the reference builds them (llclip.h,
// IndexSystem.getBorderChips: geometry n indexToGeometry(cell) in lon / lat), one lane per border
// candidate.  The lane builds the cell polygon (H3: h3ToGeoBoundary in degrees, h3_geom.h; BNG: the
// square), runs llclip::clip over the candidate's geometry -- the host producer's routine, the same
// IEEE operations (-ffp-contract=off) -- and writes the result rings from their lowest vertex into
// space taken with one atomic per counter, so tessellate.cpp writes the host producer's WKB bytes.
// Tasks whose ring walks exceed the lane's workspace, whose cell is not a planar polygon or whose
// output exceeds the buffers come back with status 1 and are clipped on the host.
#include <hip/hip_runtime.h>

#include "h3_geom.h"
#include "tess_clip.h"

namespace mosaic {
namespace tessll {

__global__ void __launch_bounds__(256) k_tess_clip_ll(ClipLLArgs a) {
    const int64_t lane = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n_lanes = (int64_t)gridDim.x * blockDim.x;
    llclip::Work w{a.wch + lane * kLLChains, kLLChains, a.wout + lane * kLLOut, kLLOut, 0, 0};
    for (int64_t t = lane; t < a.n_tasks; t += n_lanes) {
        const int64_t k = a.tasks[t];
        const int g = a.cand_geom[k];
        llclip::Cell C;
        bool ok;
        if (a.mode == 0) {
            double b[20];
            const int nb = h3geom::h3_to_geo_boundary((uint64_t)a.cand_id[k], b);
            ok = nb >= 3 && nb <= 16;
            if (ok) {
                C.nc = nb;
                for (int v = 0; v < nb; v++)
                    C.v[v] = llclip::Pt{h3geom::to_degrees(b[2 * v + 1], 8), h3geom::to_degrees(b[2 * v], 8)};
                llclip::cell_init(C);
                ok = llclip::cell_ok(C, true);
            }
        } else {
            ok = a.nv >= 3 && a.nv <= 16;
            if (ok) {
                C.nc = a.nv;
                for (int v = 0; v < a.nv; v++)
                    C.v[v] = llclip::Pt{a.clip[2 * (a.nv * k + v)], a.clip[2 * (a.nv * k + v) + 1]};
                llclip::cell_init(C);
                ok = llclip::cell_ok(C, false);
            }
        }
        if (!ok) {
            a.status[t] = 1;
            continue;
        }
        const llclip::Geom gg{a.gxy, a.ring_offsets, a.part_rings, a.geom_parts[g], a.geom_parts[g + 1], a.blk, a.ring_blk, a.ring_ccw};
        int32_t polys = 0;
        bool is_cell = false;
        const int st = llclip::clip(gg, C, w, 1e-12 * llclip::cell_area2(C), &polys, &is_cell);
        if (st != llclip::kOk) {
            a.status[t] = 1;
            continue;
        }
        if (polys == 0) {
            a.status[t] = 0;
            continue;
        }
        int64_t tot = 0;
        for (int32_t o = 0; o < w.n_out; o++) tot += w.out[o].npts + 1;
        const unsigned long long off0 = atomicAdd(&a.counters[0], (unsigned long long)tot);
        const unsigned long long rid = atomicAdd(&a.counters[1], (unsigned long long)w.n_out);
        const unsigned long long pid = atomicAdd(&a.counters[2], (unsigned long long)polys);
        if ((int64_t)(off0 + tot) > a.out_cap || (int64_t)(rid + w.n_out) > a.ring_cap ||
            (int64_t)(pid + polys) > a.part_cap) {
            a.status[t] = 1;
            continue;
        }
        int64_t off = (int64_t)off0;
        int32_t poly = -1, ring = 0;
        for (int32_t o = 0; o < w.n_out; o++) {
            const llclip::Out& r = w.out[o];
            if (!r.hole) {
                poly++;
                ring = 0;
                a.parts[pid + poly] = tessclip::ClipPart{k, poly, 1};
            }
            llclip::write_ring(gg, C, w, r, a.out + 2 * off);
            a.rings[rid + o] = tessclip::ClipRing{k, poly, ring++, off, r.npts + 1, 0};
            off += r.npts + 1;
        }
        a.status[t] = is_cell ? 2 : 0;
    }
}

__global__ void __launch_bounds__(256) k_ring_blocks(const int64_t* ro, const double* xy, int64_t n_rings, const int64_t* ring_blk,
                                                     double* blk, uint8_t* ccw) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_rings; r += step)
        llclip::ring_blocks_one(ro, xy, r, blk + 4 * ring_blk[r], ccw + r);
}

hipError_t launch_ring_blocks(const int64_t* ro, const double* xy, int64_t n_rings, const int64_t* ring_blk, double* blk,
                              uint8_t* ccw, hipStream_t stream) {
    if (n_rings <= 0) return hipSuccess;
    const int64_t blocks = (n_rings + 255) / 256 < 65536 ? (n_rings + 255) / 256 : 65536;
    hipLaunchKernelGGL(k_ring_blocks, dim3((unsigned)blocks), dim3(256), 0, stream, ro, xy, n_rings, ring_blk, blk, ccw);
    return hipGetLastError();
}

hipError_t launch_clip_ll(const ClipLLArgs& a, int64_t lanes, hipStream_t stream) {
    const int64_t blocks = (lanes + 255) / 256;
    hipLaunchKernelGGL(k_tess_clip_ll, dim3((unsigned)blocks), dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace tessll
}  // namespace mosaic

extern "C" uint64_t mosaic_layout_tess_clip(void) { return mosaic::tessll::layout_fingerprint(); }
