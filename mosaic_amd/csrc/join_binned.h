// Host interface of the binned chip join (join_binned.hip): scratch owned by a thread state of
// mosaic_hip.hip and the one launcher run_join calls.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "join_common.h"
#include "tile_images.h"

namespace binned {

// sorted point values: coordinates, plus the source row for the pairs output
struct Pt {
    double x, y;
};
struct PtRow {
    double x, y;
    long long row;
};
__host__ __device__ inline void set_row(Pt&, int64_t) {}
__host__ __device__ inline void set_row(PtRow& p, int64_t r) { p.row = (long long)r; }
__host__ __device__ inline int64_t row_of(const Pt&, int64_t i) { return i; }
__host__ __device__ inline int64_t row_of(const PtRow& p, int64_t) { return (int64_t)p.row; }
inline const long long* row_map(const Pt*) { return nullptr; }
inline const long long* row_map(const PtRow* p) { return &p->row; }

struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
    hipError_t reserve(size_t n) {
        if (n <= bytes) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        hipError_t e = hipMalloc(&p, n);
        if (e == hipSuccess) bytes = n;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

struct Scratch {
    Buf keys[2], vals[2], temp, n_skip, status;
    JoinArgs exact_args;  // the join's arguments as the exact-H3 pass must read them (sorted points)
    int64_t sorted_rows = 0;  // rows the last join() sorted (after k_bin_cover's drops)
    int spin_cap = 1 << 20;   // k_bin_cover's look-back polls before it gives up (< 0: give up at once)
    int lookback_failed = 0;  // the last join() reran k_bin_cover uncompacted
    size_t held() const {
        return keys[0].bytes + keys[1].bytes + vals[0].bytes + vals[1].bytes + temp.bytes + n_skip.bytes + status.bytes;
    }
    void release() {
        for (Buf* b : {&keys[0], &keys[1], &vals[0], &vals[1], &temp, &n_skip, &status}) b->release();
    }
};

// the device copy of a tile_images.h ImageSet
struct Images {
    const uint32_t* words = nullptr;  // nullptr: no images (k_bin_keys and k_join_binned run)
    const uint32_t* off = nullptr;    // per image key - 2
    const uint32_t* rec = nullptr;    // per image key - 2: the tile record
    const uint32_t* bin_map = nullptr;  // per tile: kBinMapWords (k_bin_cover)
    uint32_t max_words = 0;
    uint32_t n_images = 0;
};

// Rows [lo, n) of a.x / a.y: key, sort, join (enqueued on stream).  max_code: the largest tile code
// (tile records + 1).  s.exact_args receives the JoinArgs the exact-H3 pass runs with.
hipError_t join(const JoinArgs& a, int64_t lo, int64_t n, uint32_t max_code, bool lds_counts, int n_cu,
                const Images& img, Scratch& s, hipStream_t stream);

}  // namespace binned

// Layout fingerprint of the structs the translation units hand each other (JoinArgs, StreamArgs,
// BngStreamArgs, binned::Scratch / Images, by size and the offsets the other side reads).  Every TU
// reports the value its own compilation of these headers gives (mosaic_layout_*); mosaic_init refuses
// to run when they differ.  Round 5's A/B library linked a join_binned.o built against an older
// join_binned.h (Scratch without `slots`: 16 bytes shorter) into a mosaic_hip.o built against the new
// one: join() wrote s.exact_args where mosaic_hip.o did not read it, and the exact-H3 pass ran with
// shifted pointers -- the illegal-address fault of gpurun_out/r05h.
#define MOSAIC_FP_MIX(h, v) ((h) * 0x100000001b3ULL ^ (uint64_t)(v))
static constexpr uint64_t mosaic_layout_fingerprint() {
    uint64_t h = 0xcbf29ce484222325ULL;
    h = MOSAIC_FP_MIX(h, sizeof(JoinArgs));
    h = MOSAIC_FP_MIX(h, sizeof(StreamArgs));
    h = MOSAIC_FP_MIX(h, sizeof(BngStreamArgs));
    h = MOSAIC_FP_MIX(h, sizeof(binned::Scratch));
    h = MOSAIC_FP_MIX(h, offsetof(binned::Scratch, exact_args));
    h = MOSAIC_FP_MIX(h, offsetof(binned::Scratch, sorted_rows));
    h = MOSAIC_FP_MIX(h, offsetof(binned::Scratch, spin_cap));
    h = MOSAIC_FP_MIX(h, offsetof(binned::Scratch, lookback_failed));
    h = MOSAIC_FP_MIX(h, sizeof(binned::Images));
    h = MOSAIC_FP_MIX(h, offsetof(JoinArgs, res));
    h = MOSAIC_FP_MIX(h, offsetof(JoinArgs, counts));
    return h;
}
#undef MOSAIC_FP_MIX
