// H3 v3.7 neighbour traversal (algos.c), restated for the device and the host: h3NeighborRotations
// with the base-cell neighbour / rotation tables (h3_neighbor_tables.h, tools/h3gen_neighbors.py),
// hexRangeDistances, hexRing and the _kRingInternal fallback H3 takes near pentagons -- so that
// grid_cellkring / grid_cellkloop (H3IndexSystem.kRing / kLoop, core/index/H3IndexSystem.scala:
// 154-177, through h3-java 3.7.0's kRing / hexRing) and polyfill's kRing(1) give the reference's
// cells in the reference's order everywhere, pentagons included:
//   kRing(origin, k): hexRangeDistances' walk order when it succeeds; otherwise H3 wipes the
//     output and runs _kRingInternal, a depth-first search that uses the output array as an
//     open-addressing hash set (slot origin % maxKringSize, linear probing), and h3-java returns
//     the set's non-zero slots in slot order;
//   kLoop(origin, k): hexRing's order when it succeeds; otherwise the reference's own fallback
//     (H3IndexSystem.scala:169-176): kRing(k).toSet diff kRing(k - 1).toSet, in Scala 2.12
//     immutable HashSet iteration order.
// Integer-only, no recursion (the search keeps an explicit stack of depth <= k + 1).
#pragma once
#include <stdint.h>

#include "h3_device.h"

namespace mosaic {
namespace h3nb {

#if defined(__HIPCC__)
#define H3_TABLE static __constant__ const
#else
#define H3_TABLE static const
#endif
#include "h3_neighbor_tables.h"
#undef H3_TABLE

static const int kInvalidBaseCell = 127;
// algos.c DIRECTIONS (hexRange's side order) and NEXT_RING_DIRECTION
static const int kNextRing = 4;  // I_AXES_DIGIT
MOSAIC_HD int direction(int i) {
    const int d[6] = {2, 3, 1, 5, 4, 6};  // J, JK, K, IK, I, IJ
    return d[i];
}

MOSAIC_HD int res_of(uint64_t h) { return (int)((h >> 52) & 15); }
MOSAIC_HD int base_cell_of(uint64_t h) { return (int)((h >> 45) & 127); }
MOSAIC_HD uint64_t with_base_cell(uint64_t h, int bc) { return (h & ~((uint64_t)127 << 45)) | ((uint64_t)bc << 45); }
MOSAIC_HD bool base_is_pentagon(int bc) { return bc < 122 && h3::kH3BaseCellData[bc][4] != 0; }
MOSAIC_HD bool base_is_polar_pentagon(int bc) { return bc == 4 || bc == 117; }
MOSAIC_HD bool base_cw_offset(int bc, int face) { return h3::kH3BaseCellData[bc][5] == face || h3::kH3BaseCellData[bc][6] == face; }
// h3IsPentagon
MOSAIC_HD bool is_pentagon(uint64_t h) {
    return base_is_pentagon(base_cell_of(h)) && h3::leading_nonzero_digit(h, res_of(h)) == 0;
}
MOSAIC_HD uint64_t rotate60ccw(uint64_t h) { return h3::rotate_all(h, res_of(h), true); }
MOSAIC_HD uint64_t rotate60cw(uint64_t h) { return h3::rotate_all(h, res_of(h), false); }
// _h3RotatePent60ccw
MOSAIC_HD uint64_t rotate_pent60ccw(uint64_t h) { return h3::rotate_pent60ccw(h, res_of(h)); }

// algos.c h3NeighborRotations: the neighbour of origin in direction dir (rotated ccw by *rotations
// first), updating *rotations; 0 (H3_NULL) where the step enters a pentagon's deleted k axis.
MOSAIC_HD uint64_t neighbor_rotations(uint64_t origin, int dir, int* rotations) {
    uint64_t out = origin;
    for (int i = 0; i < *rotations; i++) dir = h3::rotate60ccw(dir);
    int new_rotations = 0;
    const int old_bc = base_cell_of(out);
    const int old_leading = h3::leading_nonzero_digit(out, res_of(out));
    int r = res_of(out) - 1;
    while (true) {
        if (r == -1) {
            out = with_base_cell(out, kH3BaseCellNeighbors[old_bc][dir]);
            new_rotations = kH3BaseCellNeighborRots[old_bc][dir];
            if (base_cell_of(out) == kInvalidBaseCell) {
                // the deleted k vertex at the base cell level: this edge borders another neighbour
                out = with_base_cell(out, kH3BaseCellNeighbors[old_bc][5]);  // IK_AXES_DIGIT
                new_rotations = kH3BaseCellNeighborRots[old_bc][5];
                out = rotate60ccw(out);
                *rotations = *rotations + 1;
            }
            break;
        }
        const int old_digit = h3::get_digit(out, r + 1);
        int next_dir;
        // isResClassIII(r + 1): odd resolutions
        if ((r + 1) & 1) {
            out = h3::set_digit(out, r + 1, kH3NewDigitII[old_digit][dir]);
            next_dir = kH3NewAdjustmentII[old_digit][dir];
        } else {
            out = h3::set_digit(out, r + 1, kH3NewDigitIII[old_digit][dir]);
            next_dir = kH3NewAdjustmentIII[old_digit][dir];
        }
        if (next_dir != 0) {
            dir = next_dir;
            r--;
        } else {
            break;
        }
    }
    const int new_bc = base_cell_of(out);
    if (base_is_pentagon(new_bc)) {
        bool already_adjusted_k = false;
        // force rotation out of the missing k-axes sub-sequence
        if (h3::leading_nonzero_digit(out, res_of(out)) == 1) {
            if (old_bc != new_bc) {
                // traversed into the deleted k subsequence of a pentagon base cell: rotate out
                // of it according to how we got here (cw / ccw offset face; default ccw)
                if (base_cw_offset(new_bc, h3::kH3BaseCellData[old_bc][0])) out = rotate60cw(out);
                else out = rotate60ccw(out);
                already_adjusted_k = true;
            } else {
                // into the deleted k subsequence from within the same pentagon base cell
                if (old_leading == 0) return 0;  // undefined: the k direction is deleted from here
                if (old_leading == 3) {          // JK_AXES_DIGIT
                    out = rotate60ccw(out);
                    *rotations = *rotations + 1;
                } else if (old_leading == 5) {   // IK_AXES_DIGIT
                    out = rotate60cw(out);
                    *rotations = *rotations + 5;
                } else {
                    return 0;  // (should never occur)
                }
            }
        }
        for (int i = 0; i < new_rotations; i++) out = rotate_pent60ccw(out);
        // account for differing orientation of the base cells (this edge might not follow
        // properties of some other edges)
        if (old_bc != new_bc) {
            if (base_is_polar_pentagon(new_bc)) {
                // 'polar' base cells behave differently because they have all i neighbours
                if (old_bc != 118 && old_bc != 8 && h3::leading_nonzero_digit(out, res_of(out)) != 3) *rotations = *rotations + 1;
            } else if (h3::leading_nonzero_digit(out, res_of(out)) == 5 && !already_adjusted_k) {
                // the distortion the deleted k subsequence introduces to the 5 neighbour
                *rotations = *rotations + 1;
            }
        }
    } else {
        for (int i = 0; i < new_rotations; i++) out = rotate60ccw(out);
    }
    *rotations = (*rotations + new_rotations) % 6;
    return out;
}

MOSAIC_HD int max_kring_size(int k) { return 3 * k * (k + 1) + 1; }

// hexRangeDistances (distances not kept): true on success, with out[0 .. max_kring_size(k)) in
// H3's order; false (contents undefined) where a pentagon is met
MOSAIC_HD bool hex_range(uint64_t origin, int k, int64_t* out) {
    int idx = 0;
    out[idx++] = (int64_t)origin;
    if (is_pentagon(origin)) return false;
    int ring = 1, dir = 0, i = 0, rotations = 0;
    while (ring <= k) {
        if (dir == 0 && i == 0) {
            origin = neighbor_rotations(origin, kNextRing, &rotations);
            if (origin == 0) return false;
            if (is_pentagon(origin)) return false;
        }
        origin = neighbor_rotations(origin, direction(dir), &rotations);
        if (origin == 0) return false;
        out[idx++] = (int64_t)origin;
        i++;
        if (i == ring) {
            i = 0;
            dir++;
            if (dir == 6) {
                dir = 0;
                ring++;
            }
        }
        if (is_pentagon(origin)) return false;
    }
    return true;
}

// hexRing: true on success with out[0 .. 6k) (k >= 1) in H3's order
MOSAIC_HD bool hex_ring(uint64_t origin, int k, int64_t* out) {
    if (k == 0) {
        out[0] = (int64_t)origin;
        return true;
    }
    int idx = 0, rotations = 0;
    if (is_pentagon(origin)) return false;
    for (int ring = 0; ring < k; ring++) {
        origin = neighbor_rotations(origin, kNextRing, &rotations);
        if (origin == 0) return false;
        if (is_pentagon(origin)) return false;
    }
    const uint64_t last = origin;
    out[idx++] = (int64_t)origin;
    for (int dir = 0; dir < 6; dir++) {
        for (int pos = 0; pos < k; pos++) {
            origin = neighbor_rotations(origin, direction(dir), &rotations);
            if (origin == 0) return false;
            // the very last index was already added, but it is still walked to for the
            // pentagonal distortion check below
            if (pos != k - 1 || dir != 5) {
                out[idx++] = (int64_t)origin;
                if (is_pentagon(origin)) return false;
            }
        }
    }
    return last == origin;  // otherwise pentagonal distortion occurred
}

// _kRingInternal(origin, k, out, distances, maxIdx, 0) into a zeroed table out[maxIdx] with
// distances dist[maxIdx]: the same depth-first visiting order as H3's recursion, on an explicit
// stack of k + 1 frames.  A frame is one word: the cell with its next direction index in the
// reserved bits 56-58 (zero in every valid cell index).  stack: k + 1 words of scratch, or null for
// k < kLocalDepth (a private array).
static const int kLocalDepth = 63;
MOSAIC_HD void kring_internal(uint64_t origin, int k, int64_t* out, int32_t* dist, int max_idx, uint64_t* stack) {
    uint64_t local[kLocalDepth + 1];
    uint64_t* st = stack ? stack : local;
    const uint64_t kDirMask = 7ULL << 56;
    // visit(cell, cur_k): true if its neighbours are to be searched
    auto visit = [&](uint64_t cell, int cur_k) -> bool {
        if (cell == 0) return false;
        int off = (int)(cell % (uint64_t)max_idx);
        int probes = 0;
        while (out[off] != 0 && (uint64_t)out[off] != cell) {
            off = (off + 1) % max_idx;
            if (++probes >= max_idx) return false;  // (a full table: not reachable with H3's neighbours)
        }
        if ((uint64_t)out[off] == cell && dist[off] <= cur_k) return false;
        out[off] = (int64_t)cell;
        dist[off] = cur_k;
        return cur_k < k;
    };
    if (!stack && k > kLocalDepth) return;  // (callers pass scratch beyond kLocalDepth)
    if (!visit(origin, 0)) return;
    st[0] = origin;
    int sp = 1;
    while (sp > 0) {
        const uint64_t f = st[sp - 1];
        const int i = (int)((f >> 56) & 7);
        if (i == 6) {
            sp--;
            continue;
        }
        st[sp - 1] = f + (1ULL << 56);
        int rotations = 0;
        const uint64_t nb = neighbor_rotations(f & ~kDirMask, direction(i), &rotations);
        if (visit(nb, sp)) st[sp++] = nb;  // (the new frame's depth: cur_k + 1 = sp <= k)
    }
}

// h3IsValid (h3Index.c, v3.7): a cell index (mode 1, reserved bits 0), base cell < 122, digits
// 1..res in 0..6 and the rest 7, and no leading k digit in a pentagon base cell
MOSAIC_HD bool is_valid_cell(uint64_t h) {
    if (h >> 63) return false;
    if (((h >> 59) & 15) != 1) return false;
    if (((h >> 56) & 7) != 0) return false;
    const int bc = base_cell_of(h), res = res_of(h);
    if (bc >= 122) return false;
    // digits 1 .. res are not 7, digits res + 1 .. 15 are 7 (bit tests, no loop: see
    // h3::leading_nonzero_digit)
    const uint64_t low = 0x1249249249249ULL, D = h & 0x1fffffffffffULL;
    const uint64_t seven = D & (D >> 1) & (D >> 2) & low;  // bit 3j: digit 15 - j is 7
    const uint64_t unused = low & ((1ULL << (3 * (15 - res))) - 1ULL);
    if ((seven & unused) != unused || (seven & ~unused) != 0) return false;
    return !(base_is_pentagon(bc) && h3::leading_nonzero_digit(h, res) == 1);
}

// Scala 2.12 immutable.HashSet iteration order of Long elements (the hash trie walks 5-bit groups
// of improve(elem.##) from the lowest): a sort key
MOSAIC_HD uint64_t scala_set_order_key(int64_t v) {
    const int32_t iv = (int32_t)v;
    const int32_t hc = (int64_t)iv == v ? iv : (int32_t)(v ^ (int64_t)((uint64_t)v >> 32));
    uint32_t h = (uint32_t)hc;
    h = h + ~(h << 9);
    h = h ^ (h >> 14);
    h = h + (h << 4);
    h = h ^ (h >> 10);
    uint64_t key = 0;
    for (int level = 0; level < 7; level++) key = key << 5 | ((h >> (5 * level)) & 31u);
    return key;
}

// A kRing (loop 0) / kLoop (loop 1) row by H3's fast walks: the count written to out, -3 when H3
// would fall back (a pentagon met: kring_slow), -2 for an index that is not a valid cell.
MOSAIC_HD int kring_fast(uint64_t origin, int k, int loop, int64_t* out) {
    if (!is_valid_cell(origin)) return -2;
    if (loop) return hex_ring(origin, k, out) ? (k ? 6 * k : 1) : -3;
    return hex_range(origin, k, out) ? max_kring_size(k) : -3;
}

// The device runs the fallback for k <= kSlowMaxK (H3's search makes ~5 k^3 dependent visits: ~5e6
// at k = 100, 1e7 at 128); rows beyond it run this same code on host threads (mosaic_cell_kring).
static const int kSlowMaxK = 128;

// The fallback rows (kring_fast == -3): kRing = _kRingInternal's table read in slot order (h3-java
// drops its zeros); kLoop = the reference's kRing(k).toSet diff kRing(k - 1).toSet in Scala HashSet
// order (H3IndexSystem.scala:169-176).  Scratch: tab[max_kring_size(k) + max_kring_size(k - 1)]
// (int64), dist[max_kring_size(k)] (int32), stack[k + 1] (null for k <= kLocalDepth).  Returns the
// count in out.
MOSAIC_HD int kring_slow(uint64_t origin, int k, int loop, int64_t* out, int64_t* tab, int32_t* dist,
                         uint64_t* stack = nullptr) {
    if (!stack && k > kLocalDepth) return -2;
    const int m = max_kring_size(k);
    for (int i = 0; i < m; i++) tab[i] = 0, dist[i] = 0;
    kring_internal(origin, k, tab, dist, m, stack);
    int n = 0;
    if (!loop) {
        for (int i = 0; i < m; i++)
            if (tab[i]) out[n++] = tab[i];
        return n;
    }
    // kRing(k - 1) as a hash table of its own (the same search), then the cells of ring k
    const int m1 = k ? max_kring_size(k - 1) : 1;
    int64_t* tab1 = tab + m;
    for (int i = 0; i < m1; i++) tab1[i] = 0, dist[i] = 0;
    if (k) kring_internal(origin, k - 1, tab1, dist, m1, stack);
    for (int i = 0; i < m; i++) {
        const int64_t c = tab[i];
        if (!c) continue;
        bool in1 = false;
        if (k) {
            int off = (int)((uint64_t)c % (uint64_t)m1);
            for (int p = 0; p < m1 && tab1[off]; p++) {
                if (tab1[off] == c) {
                    in1 = true;
                    break;
                }
                off = (off + 1) % m1;
            }
        }
        if (!in1) out[n++] = c;
    }
    // Scala HashSet order (insertion sort: a ring holds at most 6k cells)
    for (int i = 1; i < n; i++) {
        const int64_t v = out[i];
        const uint64_t kv = scala_set_order_key(v);
        int j = i - 1;
        while (j >= 0 && scala_set_order_key(out[j]) > kv) {
            out[j + 1] = out[j];
            j--;
        }
        out[j + 1] = v;
    }
    return n;
}

}  // namespace h3nb
}  // namespace mosaic
