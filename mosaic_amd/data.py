"""Polygon fixtures and synthetic point sets for the BASELINE configs (host side, not the hot path).

Polygon sets are the reference's own data files converted by tests/golden/make_fixtures.py
(NYC taxi zones: notebooks/data/NYC_Taxi_Zones.geojson; London postcodes:
notebooks/data/London_Postcode_Zones.geojson).  Point generators follow BASELINE.md section 3:
seeds 20250117 + config number; uniform over the zone bbox (C2), or the Quickstart mixture
(80 % Gaussian around 32 seeded zone centres, 20 % uniform, rounded to 1e-6 degrees; C1 / C3).
"""
import os

import numpy as np

from . import wkb as W

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(_ROOT, "tests", "golden")
SEED_BASE = 20250117


class PolygonSet:
    """Geometries as flat arrays: xy[V,2], ring_offsets[R+1], part_rings[P+1], geom_parts[G+1]."""

    def __init__(self, xy, ring_offsets, part_rings, geom_parts, names=None):
        self.xy = np.ascontiguousarray(xy, np.float64)
        self.ring_offsets = np.ascontiguousarray(ring_offsets, np.int64)
        self.part_rings = np.ascontiguousarray(part_rings, np.int64)
        self.geom_parts = np.ascontiguousarray(geom_parts, np.int64)
        self.names = names

    @classmethod
    def load(cls, name):
        z = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
        return cls(z["xy"], z["ring_offsets"], z["part_rings"], z["geom_parts"], z["names"])

    def __len__(self):
        return len(self.geom_parts) - 1

    def parts(self, g):
        """Geometry g as a list of parts, each a list of rings of (x, y)."""
        out = []
        for p in range(self.geom_parts[g], self.geom_parts[g + 1]):
            rings = []
            for r in range(self.part_rings[p], self.part_rings[p + 1]):
                a, b = self.ring_offsets[r], self.ring_offsets[r + 1]
                rings.append([tuple(v) for v in self.xy[a:b]])
            out.append(rings)
        return out

    def wkb(self, g, big_endian=True):
        return W.geometry_wkb(self.parts(g), big_endian)

    def subset(self, idx):
        xy, ro, pr, gp = [], [0], [0], [0]
        for g in idx:
            for rings in self.parts(g):
                for ring in rings:
                    xy.extend(ring)
                    ro.append(len(xy))
                pr.append(len(ro) - 1)
            gp.append(len(pr) - 1)
        names = None if self.names is None else self.names[list(idx)]
        return PolygonSet(np.asarray(xy), ro, pr, gp, names)

    def bbox(self):
        return (float(self.xy[:, 0].min()), float(self.xy[:, 1].min()), float(self.xy[:, 0].max()),
                float(self.xy[:, 1].max()))

    def geom_bbox(self, g):
        a = self.ring_offsets[self.part_rings[self.geom_parts[g]]]
        b = self.ring_offsets[self.part_rings[self.geom_parts[g + 1]]]
        v = self.xy[a:b]
        return float(v[:, 0].min()), float(v[:, 1].min()), float(v[:, 0].max()), float(v[:, 1].max())

    def shell_centroid(self, g):
        """Mean of the first shell's vertices (cheap 'zone centre' for the mixture generator)."""
        r = self.part_rings[self.geom_parts[g]]
        v = self.xy[self.ring_offsets[r]:self.ring_offsets[r + 1]]
        return float(v[:, 0].mean()), float(v[:, 1].mean())


def quickstart_points(zones, n, config=1, sigma=0.005, seed=None, round_1e6=True):
    """C1 / C3 mixture on the host (numpy PCG64)."""
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + config if seed is None else seed))
    x0, y0, x1, y1 = zones.bbox()
    k = min(32, len(zones))  # 32 mixture centres (fewer for small zone sets)
    centres = np.array([zones.shell_centroid(g) for g in rng.choice(len(zones), k, replace=False)])
    n_mix = int(0.8 * n)
    c = centres[rng.integers(0, k, n_mix)]
    pts = np.empty((n, 2))
    pts[:n_mix] = c + rng.normal(0.0, sigma, (n_mix, 2))
    pts[n_mix:, 0] = rng.uniform(x0, x1, n - n_mix)
    pts[n_mix:, 1] = rng.uniform(y0, y1, n - n_mix)
    rng.shuffle(pts)
    if round_1e6:
        pts = np.round(pts * 1e6) / 1e6
    return np.ascontiguousarray(pts[:, 0]), np.ascontiguousarray(pts[:, 1])


def uniform_points(bbox, n, config=2, seed=None):
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + config if seed is None else seed))
    x0, y0, x1, y1 = bbox
    return rng.uniform(x0, x1, n), rng.uniform(y0, y1, n)


def uniform_points_device(bbox, n, seed, device="cuda"):
    """Device-side uniform points (torch Philox): the 1e9-point configs never cross PCIe."""
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    x0, y0, x1, y1 = bbox
    x = torch.rand(n, generator=g, device=device, dtype=torch.float64).mul_(x1 - x0).add_(x0)
    y = torch.rand(n, generator=g, device=device, dtype=torch.float64).mul_(y1 - y0).add_(y0)
    return x, y


def clustered_points_device(zones, n, seed, sigma=0.002, device="cuda", chunk=1 << 27):
    """C3 mixture on the device (torch Philox): 80 % Gaussian around 32 zone centres (sigma in
    degrees), 20 % uniform over the zones' bbox, in random order.  Built in chunks so the 1e9-point
    shards fit beside the output without large temporaries."""
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    rng = np.random.Generator(np.random.PCG64(seed))
    centres = np.array([zones.shell_centroid(k) for k in rng.choice(len(zones), 32, replace=False)])
    ct = torch.tensor(centres, dtype=torch.float64, device=device)
    x0, y0, x1, y1 = zones.bbox()
    x = torch.empty(n, dtype=torch.float64, device=device)
    y = torch.empty(n, dtype=torch.float64, device=device)
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        pick = torch.randint(0, 32, (m,), generator=g, device=device)
        gx = torch.randn(m, generator=g, device=device, dtype=torch.float64).mul_(sigma).add_(ct[pick, 0])
        gy = torch.randn(m, generator=g, device=device, dtype=torch.float64).mul_(sigma).add_(ct[pick, 1])
        uni = torch.rand(m, generator=g, device=device, dtype=torch.float64) < 0.2
        ux = torch.rand(m, generator=g, device=device, dtype=torch.float64).mul_(x1 - x0).add_(x0)
        uy = torch.rand(m, generator=g, device=device, dtype=torch.float64).mul_(y1 - y0).add_(y0)
        x[s:s + m] = torch.where(uni, ux, gx)
        y[s:s + m] = torch.where(uni, uy, gy)
        del pick, gx, gy, uni, ux, uy
    return x, y


NYC_BBOX = (-74.25559136315209, 40.496115395170364, -73.7000090639354, 40.91553277700258)


def synthetic_buildings(n, seed=SEED_BASE + 4, bbox=NYC_BBOX, n_centres=None, sigma=0.004):
    """C4 build side: n OSM-style building footprints -- rotated rectangles (4 vertices) and
    L-shapes (6 vertices), sides 8-40 m, centres clustered (Gaussian, sigma degrees, around
    n_centres seeded centres; default one per 500 buildings, so clusters stay city-like and
    footprints rarely overlap) over the bbox.  One closed shell per geometry, counter-clockwise."""
    rng = np.random.Generator(np.random.PCG64(seed))
    if n_centres is None:
        n_centres = max(16, n // 500)
    x0, y0, x1, y1 = bbox
    cc = np.column_stack([rng.uniform(x0, x1, n_centres), rng.uniform(y0, y1, n_centres)])
    c = cc[rng.integers(0, n_centres, n)] + rng.normal(0.0, sigma, (n, 2))
    c[:, 0] = np.clip(c[:, 0], x0, x1)
    c[:, 1] = np.clip(c[:, 1], y0, y1)
    w, h = rng.uniform(8.0, 40.0, n), rng.uniform(8.0, 40.0, n)
    theta = rng.uniform(0.0, 2.0 * np.pi, n)
    is_l = rng.random(n) < 0.5
    fa, fb = rng.uniform(0.3, 0.7, n), rng.uniform(0.3, 0.7, n)
    # local shells in metres, centred
    rect = np.stack([np.column_stack([-w, -h]), np.column_stack([w, -h]), np.column_stack([w, h]),
                     np.column_stack([-w, h])], axis=1) * 0.5
    lsh = np.stack([np.column_stack([-w, -h]) * 0.5, np.column_stack([w, -h]) * 0.5,
                    np.column_stack([w * 0.5, -h * 0.5 + fb * h]),
                    np.column_stack([-w * 0.5 + fa * w, -h * 0.5 + fb * h]),
                    np.column_stack([-w * 0.5 + fa * w, h * 0.5]), np.column_stack([-w, h]) * 0.5], axis=1)
    ct, st = np.cos(theta)[:, None], np.sin(theta)[:, None]
    mlon = 1.0 / (111320.0 * np.cos(np.radians(c[:, 1])))[:, None]
    mlat = 1.0 / 110540.0

    def place(loc, idx):
        px = (loc[idx, :, 0] * ct[idx] - loc[idx, :, 1] * st[idx]) * mlon[idx] + c[idx, 0:1]
        py = (loc[idx, :, 0] * st[idx] + loc[idx, :, 1] * ct[idx]) * mlat + c[idx, 1:2]
        ring = np.stack([px, py], axis=2)
        return np.concatenate([ring, ring[:, :1]], axis=1)  # closed

    ri, li = np.nonzero(~is_l)[0], np.nonzero(is_l)[0]
    sizes = np.where(is_l, 7, 5)
    ro = np.zeros(n + 1, np.int64)
    ro[1:] = np.cumsum(sizes)
    xy = np.empty((int(ro[-1]), 2))
    pr, pl = place(rect, ri), place(lsh, li)
    xy[(ro[ri][:, None] + np.arange(5)).ravel()] = pr.reshape(-1, 2)
    xy[(ro[li][:, None] + np.arange(7)).ravel()] = pl.reshape(-1, 2)
    idx = np.arange(n + 1, dtype=np.int64)
    return PolygonSet(xy, ro, idx, idx)


def building_points_device(buildings, n, seed, near=0.7, reach_m=25.0, device="cuda", chunk=1 << 26):
    """C4 probe side on the device: a fraction `near` of the points uniform within reach_m metres
    (per axis) of a random building's first vertex, the rest uniform over the buildings' bbox."""
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    first = torch.tensor(buildings.xy[buildings.ring_offsets[:-1]], dtype=torch.float64, device=device)
    x0, y0, x1, y1 = buildings.bbox()
    dlat = reach_m / 110540.0
    dlon = reach_m / (111320.0 * np.cos(np.radians(0.5 * (y0 + y1))))
    x = torch.empty(n, dtype=torch.float64, device=device)
    y = torch.empty(n, dtype=torch.float64, device=device)
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        pick = torch.randint(0, first.shape[0], (m,), generator=g, device=device)
        nx = torch.rand(m, generator=g, device=device, dtype=torch.float64).mul_(2 * dlon).sub_(dlon).add_(first[pick, 0])
        ny = torch.rand(m, generator=g, device=device, dtype=torch.float64).mul_(2 * dlat).sub_(dlat).add_(first[pick, 1])
        uni = torch.rand(m, generator=g, device=device, dtype=torch.float64) >= near
        ux = torch.rand(m, generator=g, device=device, dtype=torch.float64).mul_(x1 - x0).add_(x0)
        uy = torch.rand(m, generator=g, device=device, dtype=torch.float64).mul_(y1 - y0).add_(y0)
        x[s:s + m] = torch.where(uni, ux, nx)
        y[s:s + m] = torch.where(uni, uy, ny)
        del pick, nx, ny, uni, ux, uy
    return x, y
