// Host stitching of st_intersection_aggregate's geometry (isect_geom.h).  The reference folds a
// group's pieces with JTS union (expressions/geometry/ST_IntersectionAggregate.scala:40-72), so its
// result is dissolved: pieces of adjacent cells form one polygon, and the shared cell sides vanish.
// Here the per-cell boundaries (overlay.h, one GPU lane per (group, cell)) are joined:
//  1. endpoints within tol are one node (the same point computed in two cells differs by ulps);
//  2. an edge is split at every node on its interior (a cell side one cell covers whole and the
//     neighbour in part);
//  3. opposite directed copies of an edge cancel (a side both cells cover is interior);
//  4. rings are traced, at every node turning to the first outgoing edge clockwise from the way
//     back, which yields minimal rings (two pieces touching at a vertex stay two polygons, as JTS
//     builds them); counter-clockwise rings (interior left) are shells, clockwise ones holes; a
//     hole goes to the smallest shell holding a point just inside the result next to it;
//  5. JTS WKBWriter output: big-endian 2D, shells clockwise and holes counter-clockwise (JTS
//     OverlayNG's orientation), each ring closed.
// Vertex order and ring start are not JTS's (its result depends on Spark's aggregation order); the
// set is pinned instead (tests/test_intersection_agg.py: symmetric difference with the exact set).
#include "isect_geom.h"

#include <math.h>
#include <string.h>

#include <algorithm>
#include <unordered_map>

namespace mosaic {
namespace isect_geom {

namespace {

struct P {
    double x, y;
};

bool on_interior(P a, P b, P q, double tol, double* t) {
    const double dx = b.x - a.x, dy = b.y - a.y;
    const double l2 = dx * dx + dy * dy;
    if (l2 == 0.0) return false;
    const double u = ((q.x - a.x) * dx + (q.y - a.y) * dy) / l2;
    if (u <= 0.0 || u >= 1.0) return false;
    const double ex = a.x + u * dx - q.x, ey = a.y + u * dy - q.y;
    if (ex * ex + ey * ey > tol * tol) return false;
    if (fabs(q.x - a.x) <= tol && fabs(q.y - a.y) <= tol) return false;
    if (fabs(q.x - b.x) <= tol && fabs(q.y - b.y) <= tol) return false;
    *t = u;
    return true;
}

void put_u8(std::vector<uint8_t>& o, uint8_t v) { o.push_back(v); }
void put_u32(std::vector<uint8_t>& o, uint32_t v) {
    for (int s = 24; s >= 0; s -= 8) o.push_back((uint8_t)(v >> s));
}
void put_f64(std::vector<uint8_t>& o, double d) {
    uint64_t v;
    memcpy(&v, &d, 8);
    for (int s = 56; s >= 0; s -= 8) o.push_back((uint8_t)(v >> s));
}

double ring_area(const std::vector<P>& r) {  // r open (first vertex not repeated)
    double a = 0;
    const double ox = r[0].x, oy = r[0].y;
    for (size_t i = 0; i < r.size(); i++) {
        const P& p = r[i];
        const P& q = r[(i + 1) % r.size()];
        a += (p.x - ox) * (q.y - oy) - (q.x - ox) * (p.y - oy);
    }
    return 0.5 * a;
}

bool pip(const std::vector<P>& r, double x, double y) {
    bool in = false;
    for (size_t i = 0, j = r.size() - 1; i < r.size(); j = i++) {
        const P& a = r[j];
        const P& b = r[i];
        if ((a.y > y) != (b.y > y)) {
            const double xc = a.x + (b.x - a.x) * (y - a.y) / (b.y - a.y);
            if (x < xc) in = !in;
        }
    }
    return in;
}

// the ring rotated to start at its smallest vertex, in the given direction
std::vector<P> canonical(const std::vector<P>& r, bool reverse) {
    std::vector<P> v = r;
    if (reverse) std::reverse(v.begin(), v.end());
    size_t k = 0;
    for (size_t i = 1; i < v.size(); i++)
        if (v[i].x < v[k].x || (v[i].x == v[k].x && v[i].y < v[k].y)) k = i;
    std::rotate(v.begin(), v.begin() + (long)k, v.end());
    return v;
}

void put_ring(std::vector<uint8_t>& o, const std::vector<P>& r) {
    put_u32(o, (uint32_t)r.size() + 1);
    for (const P& p : r) put_f64(o, p.x), put_f64(o, p.y);
    put_f64(o, r[0].x);
    put_f64(o, r[0].y);
}

}  // namespace

bool stitch_wkb(const double* edges, size_t n, double snap, std::vector<uint8_t>& out, double* area) {
    out.clear();
    *area = 0.0;
    // 1. nodes
    const double tol = snap;
    const size_t np = 2 * n;
    std::vector<P> pts(np);
    for (size_t i = 0; i < n; i++) {
        pts[2 * i] = {edges[4 * i], edges[4 * i + 1]};
        pts[2 * i + 1] = {edges[4 * i + 2], edges[4 * i + 3]};
    }
    std::vector<uint32_t> order(np), node_of(np);
    for (size_t i = 0; i < np; i++) order[i] = (uint32_t)i;
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        return pts[a].x < pts[b].x || (pts[a].x == pts[b].x && (pts[a].y < pts[b].y || (pts[a].y == pts[b].y && a < b)));
    });
    std::vector<P> nodes;
    std::vector<uint32_t> rep_node(np, ~0u);
    for (size_t q = 0; q < np; q++) {
        const uint32_t k = order[q];
        uint32_t nd = ~0u;
        for (size_t w = q; w-- > 0;) {
            const uint32_t j = order[w];
            if (pts[k].x - pts[j].x > tol) break;
            if (fabs(pts[k].y - pts[j].y) <= tol) {
                nd = node_of[j];
                break;
            }
        }
        if (nd == ~0u) {
            nd = (uint32_t)nodes.size();
            nodes.push_back(pts[k]);
        }
        node_of[k] = nd;
    }
    // nodes by x, for the on-edge queries
    std::vector<uint32_t> nx(nodes.size());
    for (size_t i = 0; i < nodes.size(); i++) nx[i] = (uint32_t)i;
    std::sort(nx.begin(), nx.end(), [&](uint32_t a, uint32_t b) { return nodes[a].x < nodes[b].x; });
    std::vector<double> nxs(nodes.size());
    for (size_t i = 0; i < nodes.size(); i++) nxs[i] = nodes[nx[i]].x;
    // 2. split at nodes on edge interiors; 3. net directed multiplicity per undirected edge
    std::unordered_map<uint64_t, int> net;
    net.reserve(2 * n + 16);
    auto add = [&](uint32_t u, uint32_t v) {
        if (u == v) return;
        if (u < v) net[(uint64_t)u << 32 | v] += 1;
        else net[(uint64_t)v << 32 | u] -= 1;
    };
    std::vector<std::pair<double, uint32_t>> cut;
    for (size_t i = 0; i < n; i++) {
        const uint32_t u = node_of[2 * i], v = node_of[2 * i + 1];
        if (u == v) continue;
        const P a = nodes[u], b = nodes[v];
        const double lo = std::min(a.x, b.x) - tol, hi = std::max(a.x, b.x) + tol;
        const double ylo = std::min(a.y, b.y) - tol, yhi = std::max(a.y, b.y) + tol;
        cut.clear();
        for (size_t q = (size_t)(std::lower_bound(nxs.begin(), nxs.end(), lo) - nxs.begin()); q < nxs.size() && nxs[q] <= hi; q++) {
            const uint32_t w = nx[q];
            if (w == u || w == v || nodes[w].y < ylo || nodes[w].y > yhi) continue;
            double t;
            if (on_interior(a, b, nodes[w], tol, &t)) cut.push_back({t, w});
        }
        std::sort(cut.begin(), cut.end());
        uint32_t prev = u;
        for (const auto& c : cut) {
            add(prev, c.second);
            prev = c.second;
        }
        add(prev, v);
    }
    // 4. outgoing edges, then ring tracing
    struct Out {
        uint32_t to;
        double ang;
        bool used;
    };
    std::vector<std::vector<Out>> outg(nodes.size());
    std::vector<std::pair<uint32_t, uint32_t>> starts;
    for (const auto& kv : net) {
        if (kv.second == 0) continue;
        uint32_t u = (uint32_t)(kv.first >> 32), v = (uint32_t)kv.first;
        if (kv.second < 0) std::swap(u, v);
        for (int m = 0; m < abs(kv.second); m++) {
            outg[u].push_back({v, atan2(nodes[v].y - nodes[u].y, nodes[v].x - nodes[u].x), false});
            starts.push_back({u, v});
        }
    }
    std::sort(starts.begin(), starts.end());
    for (auto& o : outg)
        std::sort(o.begin(), o.end(), [](const Out& a, const Out& b) { return a.to < b.to || (a.to == b.to && a.ang < b.ang); });
    auto take = [&](uint32_t u, uint32_t v) -> bool {
        for (Out& o : outg[u])
            if (o.to == v && !o.used) {
                o.used = true;
                return true;
            }
        return false;
    };
    std::vector<std::vector<P>> shells, holes;
    std::vector<double> shell_area;
    const double kTwoPi = 6.283185307179586;
    for (const auto& s : starts) {
        if (!take(s.first, s.second)) continue;  // (traced already)
        std::vector<uint32_t> ring{s.first};
        uint32_t u = s.first, v = s.second;
        size_t guard = 0;
        while (v != s.first) {
            ring.push_back(v);
            const double back = atan2(nodes[u].y - nodes[v].y, nodes[u].x - nodes[v].x);
            Out* best = nullptr;
            double best_cw = 0;
            for (Out& o : outg[v]) {
                if (o.used) continue;
                double cw = fmod(back - o.ang + 2 * kTwoPi, kTwoPi);
                if (cw <= 0.0) cw = kTwoPi;  // straight back: the last choice
                if (!best || cw < best_cw) best = &o, best_cw = cw;
            }
            if (!best || ++guard > 4 * n + 8) {
                out.clear();
                return false;
            }
            best->used = true;
            u = v;
            v = best->to;
        }
        std::vector<P> r;
        r.reserve(ring.size());
        for (uint32_t k : ring) r.push_back(nodes[k]);
        if (r.size() < 3) continue;
        const double a = ring_area(r);
        double per = 0;
        for (size_t i = 0; i < r.size(); i++) per += hypot(r[(i + 1) % r.size()].x - r[i].x, r[(i + 1) % r.size()].y - r[i].y);
        if (fabs(a) <= tol * per) continue;  // a sliver between near-coincident edges
        if (a > 0) {
            shells.push_back(r);
            shell_area.push_back(a);
        } else {
            holes.push_back(r);
        }
    }
    // holes to their shells
    std::vector<std::vector<size_t>> shell_holes(shells.size());
    for (size_t h = 0; h < holes.size(); h++) {
        const std::vector<P>& r = holes[h];
        // a point just left of the hole's longest edge: inside the result, next to the hole
        size_t k = 0;
        double best = -1;
        for (size_t i = 0; i < r.size(); i++) {
            const P& a = r[i];
            const P& b = r[(i + 1) % r.size()];
            const double l = hypot(b.x - a.x, b.y - a.y);
            if (l > best) best = l, k = i;
        }
        const P& a = r[k];
        const P& b = r[(k + 1) % r.size()];
        const double f = 1e-4;
        const double px = 0.5 * (a.x + b.x) - f * (b.y - a.y), py = 0.5 * (a.y + b.y) + f * (b.x - a.x);
        size_t owner = (size_t)-1;
        for (size_t s = 0; s < shells.size(); s++)
            if (pip(shells[s], px, py) && (owner == (size_t)-1 || shell_area[s] < shell_area[owner])) owner = s;
        if (owner == (size_t)-1) {
            out.clear();
            return false;
        }
        shell_holes[owner].push_back(h);
    }
    // 5. WKB
    std::vector<std::vector<std::vector<P>>> polys(shells.size());
    for (size_t s = 0; s < shells.size(); s++) {
        polys[s].push_back(canonical(shells[s], true));
        std::vector<std::vector<P>> hs;
        for (size_t h : shell_holes[s]) hs.push_back(canonical(holes[h], true));
        std::sort(hs.begin(), hs.end(), [](const std::vector<P>& a, const std::vector<P>& b) {
            return a[0].x < b[0].x || (a[0].x == b[0].x && a[0].y < b[0].y);
        });
        for (auto& h : hs) polys[s].push_back(std::move(h));
        double ar = shell_area[s];
        for (size_t h : shell_holes[s]) ar += ring_area(holes[h]);
        *area += ar;
    }
    std::sort(polys.begin(), polys.end(), [](const std::vector<std::vector<P>>& a, const std::vector<std::vector<P>>& b) {
        return a[0][0].x < b[0][0].x || (a[0][0].x == b[0][0].x && a[0][0].y < b[0][0].y);
    });
    auto put_polygon = [&](const std::vector<std::vector<P>>& p) {
        put_u8(out, 0);
        put_u32(out, 3);
        put_u32(out, (uint32_t)p.size());
        for (const auto& r : p) put_ring(out, r);
    };
    if (polys.size() == 1) {
        put_polygon(polys[0]);
    } else if (polys.empty()) {
        put_u8(out, 0);
        put_u32(out, 3);
        put_u32(out, 0);  // POLYGON EMPTY (the aggregation buffer's initial value)
    } else {
        put_u8(out, 0);
        put_u32(out, 6);
        put_u32(out, (uint32_t)polys.size());
        for (const auto& p : polys) put_polygon(p);
    }
    return true;
}

}  // namespace isect_geom
}  // namespace mosaic
