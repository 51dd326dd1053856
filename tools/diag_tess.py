"""Diagnostic (GPU box): tessellated-chip join, H3 cells and every contains strategy vs the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _rss_guard(limit_gb=16.0):
    import threading
    import time

    import psutil

    def run():
        p = psutil.Process()
        while True:
            if p.memory_info().rss > limit_gb * 2**30:
                print("RSS guard: over", limit_gb, "GB", flush=True)
                os._exit(3)
            time.sleep(0.1)

    threading.Thread(target=run, daemon=True).start()


def main():
    _rss_guard()
    import torch  # noqa: F401

    import oracle
    from mosaic_amd import MosaicContext
    from mosaic_amd.context import tessellate
    from mosaic_amd.data import PolygonSet
    from tests.test_gpu_parity import _chip_boundary_points

    import psutil

    def mark(msg):
        print(msg, "rss GB %.2f" % (psutil.Process().memory_info().rss / 2**30), flush=True)

    mark("start")
    z = PolygonSet.load("nyc_taxi_zones_35")
    chips = tessellate("H3", z, 9)
    rng = np.random.default_rng(5)
    x0, y0, x1, y1 = z.bbox()
    bx, by = _chip_boundary_points(chips, rng)
    x = np.concatenate([rng.uniform(x0, x1, 400_000), bx])
    y = np.concatenate([rng.uniform(y0, y1, 400_000), by])
    mark("points")
    ctx = MosaicContext.build("H3")
    mark("ctx")
    cells = ctx.grid_longlatascellid(x, y, 9, raw=True)
    mark("cells")
    want_cells = oracle.h3_point_to_index(x, y, 9)
    bad = np.nonzero(cells != want_cells)[0]
    print("h3 mismatches", len(bad), "of", len(x), "first", [(float(x[i]), float(y[i])) for i in bad[:5]])
    offs, data = chips["wkb"]
    oc = dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
              wkb_offsets=offs, wkb=data)
    want, total = oracle.pip_join(oc, oracle.GRID_H3, 9, x, y, len(z), threads=8)
    _, _, orow, okey = oracle.pip_join(oc, oracle.GRID_H3, 9, x, y, len(z), pairs=True)
    oset = set(zip(orow.tolist(), okey.tolist()))
    for raster, le in ((16, 8), (16, 0), (1, 8)):
        ctx.set_option("raster", raster)
        ctx.set_option("lane_edges", le)
        table = ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 9,
                               n_polygons=len(z))
        for mode in (3, 2, 1, 0):
            ctx.set_option("pip_mode", mode)
            got = ctx.pip_join_count(table, x, y)
            print("mode", mode, "counts done", flush=True)
            rows, keys = ctx.pip_join_pairs(table, x, y, capacity=4 * len(x))
            gset = set(zip(rows.tolist(), keys.tolist()))
            extra = sorted(gset - oset)[:4]
            miss = sorted(oset - gset)[:4]
            print(f"raster {raster} lane {le} mode {mode}: count diff {int(np.abs(got - want).sum())} "
                  f"extra {len(gset - oset)} {[(r, k, float(x[r]), float(y[r])) for r, k in extra]} "
                  f"missing {len(oset - gset)} {[(r, k, float(x[r]), float(y[r])) for r, k in miss]}")
        table.close()


if __name__ == "__main__":
    main()
