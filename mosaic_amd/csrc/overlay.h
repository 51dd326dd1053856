// Polygon overlay of one (group, cell) unit of st_intersection_aggregate (reference
// expressions/geometry/ST_IntersectionAggregate.scala:40-72): the union the reference folds per
// (left id, right id) group -- per joined chip pair the cell (both core), the other chip (one core)
// or left.wkb intersection right.wkb -- restricted to one cell is, since every chip lies in its cell
// and a core chip is the whole cell,
//     (union of the group's left chips in the cell) n (union of its right chips in the cell)
// (with "the cell" for a side holding a core chip).  This routine computes the boundary of that set
// as directed edges, interior on the left, for the host to stitch across cells into the group's
// polygons (isect_geom.cpp).  One lane per unit on the GPU (k_isect_overlay), or host threads in
// the self-check (tests/native/overlay_host.cpp); plain arrays in caller scratch, no allocation.
//
// Method (an arrangement overlay, labelled by faces):
//  1. edges of every polygon part of the unit;
//  2. noding: every edge is split where another edge's endpoint lies on it (within tol) and at
//     proper crossings (the same computed point for both edges);
//  3. node clustering: sub-edge endpoints within tol are one node (so coordinates computed in two
//     chips, equal up to rounding, meet);
//  4. the unique undirected edges as half-edge pairs; at every node the outgoing half-edges sorted
//     by angle; the face cycles traced (next = the first outgoing half-edge clockwise from the way
//     back, the face on the left);
//  5. every face cycle labelled once, on the left of its longest half-edge, even-odd per part: a ray
//     from the edge's midpoint (+x for a steep edge, +y for a flat one, so it meets neither end
//     after rounding) counts the part's crossings with the part edges the unique edge was cut from
//     excluded -- that is the parity on the side the ray leaves from, and the other side differs
//     by the number of excluded edges of the part (a zero-width bridge changes nothing); no offset
//     point, so a face that is a sliver along that edge is labelled as exactly as a fat one.  A and
//     B are the unions of their parts, the label A n B; a half-edge is emitted when its cycle is in
//     and its twin's cycle is out.  The emitted set is the boundary of a union of face cycles, so it
//     is closed whatever the labels are: near-degenerate input (a chip ring crossing itself by a
//     rounding sliver, a vertex within tol of an edge) can at worst mislabel a sliver, never leave a
//     dangling edge.
#pragma once
#include <math.h>
#include <stdint.h>

#include "pip_device.h"

namespace mosaic {
namespace overlay {

struct Edge {
    double x0, y0, x1, y1;
    int32_t poly;  // index into the unit's part list
    int32_t pad;
};
struct Split {
    int32_t edge;
    int32_t pad;
    double t, x, y;
};
struct PartRef {
    uint32_t part;    // part index in its store
    uint32_t set;     // 0: A (left), 1: B (right)
    uint32_t e0, e1;  // its edges in the scratch edge list (filled by unit_boundary)
};

struct Scratch {
    Edge* edges;
    int e_cap;
    Split* splits;
    int s_cap;
    double* px;
    double* py;
    int32_t* pnode;
    int32_t* porder;
    int p_cap;
    uint64_t* keys;    // sub-edges (point pairs), then node pairs sorted, then the unique edges
    int32_t* rec_edge; // per sub-edge record: the edge it was cut from (sorted with keys)
    int32_t* ue_rec;   // unique edge q: its records are [ue_rec[q], ue_rec[q + 1])
    int r_cap;
    double* he_ang;   // per half-edge (2 r_cap): angle at its origin
    int32_t* he_ord;  // half-edges sorted by (origin, angle)
    int32_t* he_pos;  // position of a half-edge in he_ord
    int32_t* he_cyc;  // its face cycle
    double* cy_len;   // per cycle: longest half-edge length, which half-edge, label
    int32_t* cy_best;
    int32_t* cy_lab;
};

// bytes of scratch for a unit of e edges (the layout of make_scratch)
MOSAIC_HD int64_t scratch_bytes(int64_t e) {
    const int64_t s = 4 * e + 64, p = 2 * e + s, r = e + s;
    return e * (int64_t)sizeof(Edge) + s * (int64_t)sizeof(Split) + p * 24 + r * 16 + 2 * r * 36 + 128;
}
MOSAIC_HD Scratch make_scratch(void* base, int64_t e) {
    const int64_t s = 4 * e + 64, p = 2 * e + s, r = e + s;
    char* b = (char*)base;
    Scratch sc;
    sc.edges = (Edge*)b;
    b += e * sizeof(Edge);
    sc.splits = (Split*)b;
    b += s * sizeof(Split);
    sc.keys = (uint64_t*)b;
    b += r * 8;
    sc.rec_edge = (int32_t*)b;
    b += r * 4;
    sc.ue_rec = (int32_t*)b;
    b += (r + 1) * 4;
    b = (char*)(((uintptr_t)b + 7) & ~(uintptr_t)7);
    sc.px = (double*)b;
    b += p * 8;
    sc.py = (double*)b;
    b += p * 8;
    sc.he_ang = (double*)b;
    b += 2 * r * 8;
    sc.cy_len = (double*)b;
    b += 2 * r * 8;
    sc.pnode = (int32_t*)b;
    b += p * 4;
    sc.porder = (int32_t*)b;
    b += p * 4;
    sc.he_ord = (int32_t*)b;
    b += 2 * r * 4;
    sc.he_pos = (int32_t*)b;
    b += 2 * r * 4;
    sc.he_cyc = (int32_t*)b;
    b += 2 * r * 4;
    sc.cy_best = (int32_t*)b;
    b += 2 * r * 4;
    sc.cy_lab = (int32_t*)b;
    sc.e_cap = (int)e;
    sc.s_cap = (int)s;
    sc.p_cap = (int)p;
    sc.r_cap = (int)r;
    return sc;
}

// edges of a part (all its rings)
MOSAIC_HD int part_edges(const pip::GeomStore& s, uint32_t part) {
    int n = 0;
    for (uint32_t r = s.part_ring[part]; r < s.part_ring[part + 1]; r++) {
        const uint32_t k = s.ring_start[r + 1] - s.ring_start[r];
        n += k > 1 ? (int)k - 1 : 0;
    }
    return n;
}

// point on the interior of segment (a, b) within tol (and not within tol of an end): its parameter
MOSAIC_HD bool on_interior(double ax, double ay, double bx, double by, double qx, double qy, double tol, double* t) {
    const double dx = bx - ax, dy = by - ay;
    const double l2 = dx * dx + dy * dy;
    if (l2 == 0.0) return false;
    const double u = ((qx - ax) * dx + (qy - ay) * dy) / l2;
    if (u <= 0.0 || u >= 1.0) return false;
    const double ex = ax + u * dx - qx, ey = ay + u * dy - qy;
    if (ex * ex + ey * ey > tol * tol) return false;
    const double da = (qx - ax) * (qx - ax) + (qy - ay) * (qy - ay), db = (qx - bx) * (qx - bx) + (qy - by) * (qy - by);
    if (da <= tol * tol || db <= tol * tol) return false;
    *t = u;
    return true;
}

MOSAIC_HD bool near_pt(double ax, double ay, double bx, double by, double tol) {
    return fabs(ax - bx) <= tol && fabs(ay - by) <= tol;
}

// shell sorts (no recursion, no allocation)
MOSAIC_HD void sort_splits(Split* a, int n) {
    int gap = 1;
    while (gap < n / 3) gap = 3 * gap + 1;
    for (; gap > 0; gap /= 3)
        for (int i = gap; i < n; i++) {
            const Split v = a[i];
            int j = i;
            while (j >= gap && (a[j - gap].edge > v.edge || (a[j - gap].edge == v.edge && a[j - gap].t > v.t))) {
                a[j] = a[j - gap];
                j -= gap;
            }
            a[j] = v;
        }
}
MOSAIC_HD void sort_keys(uint64_t* a, int32_t* b, int n) {
    int gap = 1;
    while (gap < n / 3) gap = 3 * gap + 1;
    for (; gap > 0; gap /= 3)
        for (int i = gap; i < n; i++) {
            const uint64_t v = a[i];
            const int32_t w = b[i];
            int j = i;
            while (j >= gap && a[j - gap] > v) {
                a[j] = a[j - gap];
                b[j] = b[j - gap];
                j -= gap;
            }
            a[j] = v;
            b[j] = w;
        }
}
// half-edge h of unique edge h / 2: origin = the key's first node for even h, second for odd h
MOSAIC_HD int he_origin(const uint64_t* keys, int h) {
    return (h & 1) ? (int)(uint32_t)keys[h >> 1] : (int)(keys[h >> 1] >> 32);
}
MOSAIC_HD void sort_half_edges(int32_t* idx, const uint64_t* keys, const double* ang, int n) {
    int gap = 1;
    while (gap < n / 3) gap = 3 * gap + 1;
    for (; gap > 0; gap /= 3)
        for (int i = gap; i < n; i++) {
            const int32_t v = idx[i];
            const int ov = he_origin(keys, v);
            int j = i;
            while (j >= gap) {
                const int32_t w = idx[j - gap];
                const int ow = he_origin(keys, w);
                if (!(ow > ov || (ow == ov && ang[w] > ang[v]))) break;
                idx[j] = w;
                j -= gap;
            }
            idx[j] = v;
        }
}
MOSAIC_HD void sort_by_x(int32_t* idx, const double* px, int n) {
    int gap = 1;
    while (gap < n / 3) gap = 3 * gap + 1;
    for (; gap > 0; gap /= 3)
        for (int i = gap; i < n; i++) {
            const int32_t v = idx[i];
            int j = i;
            while (j >= gap && px[idx[j - gap]] > px[v]) {
                idx[j] = idx[j - gap];
                j -= gap;
            }
            idx[j] = v;
        }
}

enum { kNeedA = 1, kNeedB = 2 };

// The unit's result boundary.  parts[0 .. n_parts): the parts of both sets; need: kNeedA | kNeedB
// (a set not needed covers the whole cell: a core chip on that side).  Emits the directed result
// edges to out[4 k .. 4 k + 3] = (x0, y0, x1, y1), at most out_cap; *area = their shoelace area
// (relative to the first vertex).  Returns the number of edges, or -1 when a capacity is exceeded.
MOSAIC_HD int unit_boundary(const pip::GeomStore* st, PartRef* parts, int n_parts, int need, Scratch& sc,
                            double* out, int out_cap, double* area) {
    *area = 0.0;
    // 1. edges, and the coordinate scale
    int ne = 0;
    double scale = 1.0;
    for (int k = 0; k < n_parts; k++) {
        const pip::GeomStore& s = st[parts[k].set];
        const uint32_t p = parts[k].part;
        parts[k].e0 = (uint32_t)ne;
        for (uint32_t r = s.part_ring[p]; r < s.part_ring[p + 1]; r++) {
            for (uint32_t i = s.ring_start[r]; i + 1 < s.ring_start[r + 1]; i++) {
                const pip::Vec2 a = s.verts[i], b = s.verts[i + 1];
                if (a.x == b.x && a.y == b.y) continue;
                if (ne >= sc.e_cap) return -1;
                sc.edges[ne++] = Edge{a.x, a.y, b.x, b.y, k, 0};
                scale = fmax(scale, fmax(fmax(fabs(a.x), fabs(a.y)), fmax(fabs(b.x), fabs(b.y))));
            }
        }
        parts[k].e1 = (uint32_t)ne;
    }
    if (ne == 0) return 0;
    const double tol = scale * 9.094947017729282e-13;  // 2^-40
    // 2. noding
    int ns = 0;
    for (int i = 0; i < ne; i++) {
        const Edge ei = sc.edges[i];
        const double iminx = fmin(ei.x0, ei.x1) - tol, imaxx = fmax(ei.x0, ei.x1) + tol;
        const double iminy = fmin(ei.y0, ei.y1) - tol, imaxy = fmax(ei.y0, ei.y1) + tol;
        for (int j = i + 1; j < ne; j++) {
            const Edge ej = sc.edges[j];
            if (fmax(ej.x0, ej.x1) < iminx || fmin(ej.x0, ej.x1) > imaxx || fmax(ej.y0, ej.y1) < iminy ||
                fmin(ej.y0, ej.y1) > imaxy)
                continue;
            double t;
            bool touch = false;
            // endpoints of one on the interior of the other
            if (on_interior(ei.x0, ei.y0, ei.x1, ei.y1, ej.x0, ej.y0, tol, &t)) {
                if (ns >= sc.s_cap) return -1;
                sc.splits[ns++] = Split{i, 0, t, ej.x0, ej.y0};
                touch = true;
            }
            if (on_interior(ei.x0, ei.y0, ei.x1, ei.y1, ej.x1, ej.y1, tol, &t)) {
                if (ns >= sc.s_cap) return -1;
                sc.splits[ns++] = Split{i, 0, t, ej.x1, ej.y1};
                touch = true;
            }
            if (on_interior(ej.x0, ej.y0, ej.x1, ej.y1, ei.x0, ei.y0, tol, &t)) {
                if (ns >= sc.s_cap) return -1;
                sc.splits[ns++] = Split{j, 0, t, ei.x0, ei.y0};
                touch = true;
            }
            if (on_interior(ej.x0, ej.y0, ej.x1, ej.y1, ei.x1, ei.y1, tol, &t)) {
                if (ns >= sc.s_cap) return -1;
                sc.splits[ns++] = Split{j, 0, t, ei.x1, ei.y1};
                touch = true;
            }
            if (touch) continue;
            if (near_pt(ei.x0, ei.y0, ej.x0, ej.y0, tol) || near_pt(ei.x0, ei.y0, ej.x1, ej.y1, tol) ||
                near_pt(ei.x1, ei.y1, ej.x0, ej.y0, tol) || near_pt(ei.x1, ei.y1, ej.x1, ej.y1, tol))
                continue;  // (meeting at a shared end: nothing to split)
            // proper crossing: orientations relative to ei's start
            const double ax = ei.x1 - ei.x0, ay = ei.y1 - ei.y0;
            const double c0x = ej.x0 - ei.x0, c0y = ej.y0 - ei.y0, c1x = ej.x1 - ei.x0, c1y = ej.y1 - ei.y0;
            const double d1 = ax * c0y - ay * c0x, d2 = ax * c1y - ay * c1x;
            if (!((d1 > 0 && d2 < 0) || (d1 < 0 && d2 > 0))) continue;
            const double bx = c1x - c0x, by = c1y - c0y;
            const double d3 = bx * (-c0y) - by * (-c0x), d4 = bx * (ay - c0y) - by * (ax - c0x);
            if (!((d3 > 0 && d4 < 0) || (d3 < 0 && d4 > 0))) continue;
            const double u = d1 / (d1 - d2);  // along ej
            const double xx = ej.x0 + u * (ej.x1 - ej.x0), xy = ej.y0 + u * (ej.y1 - ej.y0);
            const double l2i = ax * ax + ay * ay;
            const double ti = ((xx - ei.x0) * ax + (xy - ei.y0) * ay) / l2i;
            if (ns + 2 > sc.s_cap) return -1;
            if (!near_pt(xx, xy, ei.x0, ei.y0, tol) && !near_pt(xx, xy, ei.x1, ei.y1, tol))
                sc.splits[ns++] = Split{i, 0, fmin(fmax(ti, 0.0), 1.0), xx, xy};
            if (!near_pt(xx, xy, ej.x0, ej.y0, tol) && !near_pt(xx, xy, ej.x1, ej.y1, tol))
                sc.splits[ns++] = Split{j, 0, u, xx, xy};
        }
    }
    sort_splits(sc.splits, ns);
    // 3. points of the sub-edges (per edge: start, its splits in order, end)
    int np = 0, nr = 0;
    int si = 0;
    for (int e = 0; e < ne; e++) {
        const Edge ed = sc.edges[e];
        int first = np;
        if (np >= sc.p_cap) return -1;
        sc.px[np] = ed.x0, sc.py[np] = ed.y0, np++;
        for (; si < ns && sc.splits[si].edge == e; si++) {
            if (np >= sc.p_cap) return -1;
            sc.px[np] = sc.splits[si].x, sc.py[np] = sc.splits[si].y, np++;
        }
        if (np >= sc.p_cap) return -1;
        sc.px[np] = ed.x1, sc.py[np] = ed.y1, np++;
        for (int k = first; k + 1 < np; k++) {
            if (nr >= sc.r_cap) return -1;
            // (node pair filled in after the clustering; the point indices meanwhile)
            sc.rec_edge[nr] = e;
            sc.keys[nr++] = (uint64_t)(uint32_t)k << 32 | (uint32_t)(k + 1);
        }
    }
    // clustering: a point joins the node of an earlier point (in x order) within tol
    for (int k = 0; k < np; k++) sc.porder[k] = k;
    sort_by_x(sc.porder, sc.px, np);
    for (int q = 0; q < np; q++) {
        const int k = sc.porder[q];
        int node = k;
        for (int w = q - 1; w >= 0; w--) {
            const int j = sc.porder[w];
            if (sc.px[k] - sc.px[j] > tol) break;
            if (fabs(sc.py[k] - sc.py[j]) <= tol) {
                node = sc.pnode[j];
                break;
            }
        }
        sc.pnode[k] = node;
    }
    // 4. unique undirected edges (node pairs), their half-edges, the face cycles
    int nk = 0;
    for (int q = 0; q < nr; q++) {
        const int a = (int)(sc.keys[q] >> 32), b = (int)(uint32_t)sc.keys[q];
        const int na = sc.pnode[a], nb = sc.pnode[b];
        if (na == nb) continue;
        sc.rec_edge[nk] = sc.rec_edge[q];
        sc.keys[nk++] = na < nb ? ((uint64_t)(uint32_t)na << 32 | (uint32_t)nb) : ((uint64_t)(uint32_t)nb << 32 | (uint32_t)na);
    }
    sort_keys(sc.keys, sc.rec_edge, nk);
    int nu = 0;
    for (int q = 0; q < nk; q++)
        if (q == 0 || sc.keys[q] != sc.keys[q - 1]) sc.ue_rec[nu++] = q;
    sc.ue_rec[nu] = nk;
    for (int q = 0; q < nu; q++) sc.keys[q] = sc.keys[sc.ue_rec[q]];  // (in place: ue_rec[q] >= q)
    const int nh = 2 * nu;
    for (int h = 0; h < nh; h++) {
        const int o = he_origin(sc.keys, h), d = he_origin(sc.keys, h ^ 1);
        sc.he_ang[h] = atan2(sc.py[d] - sc.py[o], sc.px[d] - sc.px[o]);
        sc.he_ord[h] = h;
        sc.he_cyc[h] = -1;
    }
    sort_half_edges(sc.he_ord, sc.keys, sc.he_ang, nh);
    for (int q = 0; q < nh; q++) sc.he_pos[sc.he_ord[q]] = q;
    // next(h) at h's destination: the outgoing half-edge just clockwise of twin(h) (the previous one in
    // the node's angle order, cyclically)
    auto next_he = [&](int h) -> int {
        const int t = h ^ 1;
        const int o = he_origin(sc.keys, t);
        const int q = sc.he_pos[t];
        if (q > 0 && he_origin(sc.keys, sc.he_ord[q - 1]) == o) return sc.he_ord[q - 1];
        int z = q;  // wrap: the node's last outgoing half-edge
        while (z + 1 < nh && he_origin(sc.keys, sc.he_ord[z + 1]) == o) z++;
        return sc.he_ord[z];
    };
    int nc = 0;
    for (int h0 = 0; h0 < nh; h0++) {
        if (sc.he_cyc[h0] >= 0) continue;
        double best = -1.0;
        int bh = h0;
        for (int h = h0, guard = 0; sc.he_cyc[h] < 0 && guard <= nh; h = next_he(h), guard++) {
            sc.he_cyc[h] = nc;
            const int o = he_origin(sc.keys, h), d = he_origin(sc.keys, h ^ 1);
            const double l = fabs(sc.px[d] - sc.px[o]) + fabs(sc.py[d] - sc.py[o]);
            if (l > best) best = l, bh = h;
        }
        sc.cy_best[nc] = bh;
        sc.cy_len[nc] = best;
        nc++;
    }
    // 5. a label per face cycle: the side of its longest half-edge, by the excluded-edge ray
    for (int c = 0; c < nc; c++) {
        const int h = sc.cy_best[c];
        const int q = h >> 1;
        const int u = (int)(sc.keys[q] >> 32), v = (int)(uint32_t)sc.keys[q];  // canonical u -> v
        const double ux = sc.px[u], uy = sc.py[u], vx = sc.px[v], vy = sc.py[v];
        const double mx = 0.5 * (ux + vx), my = 0.5 * (uy + vy);
        const bool flat = fabs(vx - ux) > fabs(vy - uy);
        // the side of u -> v the ray leaves from: +y leaves a rightward edge's left, +x a downward one's
        const bool from_left = flat ? (vx > ux) : (vy < uy);
        const bool want_left = (h & 1) == 0;  // h's left side is u -> v's left for h = u -> v
        const int r0 = sc.ue_rec[q], r1 = sc.ue_rec[q + 1];
        bool ain = false, bin = false;
        for (int k = 0; k < n_parts; k++) {
            bool par = false;
            int n_excl = 0;
            for (uint32_t e = parts[k].e0; e < parts[k].e1; e++) {
                bool excl = false;
                for (int z = r0; z < r1; z++) excl |= sc.rec_edge[z] == (int32_t)e;
                if (excl) {
                    n_excl++;
                    continue;
                }
                const Edge& ed = sc.edges[e];
                if (!flat) {
                    if ((ed.y0 > my) != (ed.y1 > my)) {
                        const double xc = ed.x0 + (ed.x1 - ed.x0) * (my - ed.y0) / (ed.y1 - ed.y0);
                        if (xc > mx) par = !par;
                    }
                } else {
                    if ((ed.x0 > mx) != (ed.x1 > mx)) {
                        const double yc = ed.y0 + (ed.y1 - ed.y0) * (mx - ed.x0) / (ed.x1 - ed.x0);
                        if (yc > my) par = !par;
                    }
                }
            }
            const bool in = (want_left == from_left) ? par : (par != ((n_excl & 1) != 0));
            if (parts[k].set == 0) ain |= in;
            else bin |= in;
        }
        sc.cy_lab[c] = (!(need & kNeedA) || ain) && (!(need & kNeedB) || bin);
    }
    int nout = 0;
    double acc = 0.0;
    const double ox = sc.edges[0].x0, oy = sc.edges[0].y0;
    for (int h = 0; h < nh; h++) {
        if (!sc.cy_lab[sc.he_cyc[h]] || sc.cy_lab[sc.he_cyc[h ^ 1]]) continue;
        if (nout >= out_cap) return -1;
        const int o = he_origin(sc.keys, h), d = he_origin(sc.keys, h ^ 1);
        double* q = out + 4 * nout++;
        q[0] = sc.px[o], q[1] = sc.py[o], q[2] = sc.px[d], q[3] = sc.py[d];
        acc += (q[0] - ox) * (q[3] - oy) - (q[2] - ox) * (q[1] - oy);
    }
    *area = 0.5 * acc;
    return nout;
}

}  // namespace overlay
}  // namespace mosaic
