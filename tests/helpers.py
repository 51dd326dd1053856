"""Test helpers: synthetic chip tables and adversarial points (host side)."""
import numpy as np

from mosaic_amd import wkb as W


def synthetic_chips(zones, geom_ids, res, cell_fn, rng, pts_per_zone=400, core_frac=0.3, clip=False):
    """A chip table whose cells are the cells of random points inside each zone's bbox.

    The join's semantics are defined for any chip table, so parity tests do not need real
    tessellation output: every chip gets the zone's full geometry as its wkb (or none when core).
    Returns dict(is_core, index_id, wkb list, polygon_key) with zone position as the key.
    """
    is_core, ids, wkbs, keys = [], [], [], []
    for k, g in enumerate(geom_ids):
        x0, y0, x1, y1 = zones.geom_bbox(g)
        xs = rng.uniform(x0, x1, pts_per_zone)
        ys = rng.uniform(y0, y1, pts_per_zone)
        cells = np.unique(cell_fn(xs, ys, res))
        blob = zones.wkb(g, big_endian=bool(k % 2))
        for c in cells:
            core = rng.random() < core_frac
            is_core.append(1 if core else 0)
            ids.append(int(c))
            wkbs.append(None if core and rng.random() < 0.5 else blob)
            keys.append(k)
    return dict(is_core=np.array(is_core, np.uint8), index_id=np.array(ids, np.int64), wkb=wkbs,
                polygon_key=np.array(keys, np.int32))


def chips_to_oracle(chips):
    lens = np.array([0 if w is None else len(w) for w in chips["wkb"]], np.int64)
    offs = np.zeros(len(lens) + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    data = np.frombuffer(b"".join(b"" if w is None else w for w in chips["wkb"]) or b"\0", np.uint8).copy()
    return dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
                wkb_offsets=offs, wkb=data)


def boundary_points(zones, geom_ids, rng, n_per=40):
    """Points exactly on zone vertices, on exactly representable edge points, and just off them."""
    xs, ys = [], []
    for g in geom_ids:
        for rings in zones.parts(g):
            ring = rings[0]
            for _ in range(n_per):
                i = int(rng.integers(0, len(ring) - 1))
                (ax, ay), (bx, by) = ring[i], ring[i + 1]
                kind = rng.random()
                if kind < 0.4:
                    xs.append(ax)
                    ys.append(ay)
                elif kind < 0.7:
                    t = 0.5
                    xs.append(ax + t * (bx - ax))
                    ys.append(ay + t * (by - ay))
                else:
                    xs.append(np.nextafter(ax, ax + 1))
                    ys.append(ay)
    return np.array(xs), np.array(ys)
