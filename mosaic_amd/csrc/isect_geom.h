// Host stitching of st_intersection_aggregate's geometry (isect_geom.cpp): the directed boundary
// edges of a group's per-cell overlays (overlay.h, k_isect_overlay) -> the group's polygons as the
// WKB JTS writes (big-endian 2D Polygon / MultiPolygon; POLYGON EMPTY for an empty result).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace mosaic {
namespace isect_geom {

// edges: n x (x0, y0, x1, y1), interior on the left, in any order; the union of the cells' pieces is
// dissolved (shared cell sides cancel), rings are traced as minimal rings, holes assigned to the
// smallest shell holding them.  Shells are written clockwise, holes counter-clockwise, each ring
// starting at its smallest vertex, polygons ordered by that vertex (deterministic output).
// Returns false (out cleared) when the edges do not close into rings (a noding failure).
// snap: the node tolerance (coordinate units); pieces of adjacent cells computed from different
// cells' arithmetic meet within it (see isect_geom.cpp).
bool stitch_wkb(const double* edges, size_t n, double snap, std::vector<uint8_t>& out, double* area);

}  // namespace isect_geom
}  // namespace mosaic
