"""Kernel-level timing breakdown of the join (GPU box): cell kernel alone, join with every chip
marked core (no contains), full join.  Prints one JSON line per variant.

    python tools/kbench.py [--n 1e8] [--res 9]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=float, default=1e8)
    p.add_argument("--res", type=int, default=9)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--block", type=int, default=256)
    p.add_argument("--bpc", type=int, default=8)
    p.add_argument("--clustered", action="store_true")
    p.add_argument("--rasters", type=int, nargs="*", default=[8, 16, 32])
    p.add_argument("--lane-edges", type=int, nargs="*", default=[0, 4, 8])
    args = p.parse_args()
    import torch

    from mosaic_amd import MosaicContext
    from mosaic_amd.context import tessellate
    from mosaic_amd.data import PolygonSet, uniform_points_device

    zones = PolygonSet.load("nyc_taxi_zones")
    chips = tessellate("H3", zones, args.res)
    ctx = MosaicContext.build("H3")
    ctx.set_option("block", args.block)
    ctx.set_option("blocks_per_cu", args.bpc)
    n = int(args.n)
    x, y = uniform_points_device(zones.bbox(), n, seed=1)
    out = torch.empty(n, dtype=torch.int64, device="cuda")
    counts = torch.zeros(len(zones), dtype=torch.int64, device="cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e))
        return float(np.median(ts))

    from mosaic_amd import _native as N

    def cells():
        N.check(N.lib().mosaic_point_to_cell(ctx.handle, 0, args.res, x.data_ptr(), y.data_ptr(), None, n,
                                             out.data_ptr(), None))

    t_cell = timeit(cells)
    print(json.dumps({"variant": "cell_kernel", "ms": t_cell, "pts_per_s": n / t_cell * 1e3}))
    ctx.set_option("async", 1)
    variants = [("join_all_core", True, 3, 16, 8), ("join_full_coop", False, 1, 16, 8),
                ("join_full_slab", False, 2, 16, 8)]
    for r in args.rasters:
        for le in args.lane_edges:
            variants.append((f"join_raster{r}_lane{le}", False, 3, r, le))
    for name, core, mode, raster, lane_edges in variants:
        ctx.set_option("pip_mode", mode)
        ctx.set_option("raster", raster)
        ctx.set_option("lane_edges", lane_edges)
        is_core = np.ones_like(chips["is_core"]) if core else chips["is_core"]
        table = ctx.chip_table(is_core, chips["index_id"], chips["wkb"], chips["polygon_key"], args.res,
                               n_polygons=len(zones))
        t = timeit(lambda: ctx.pip_join_count(table, x, y, out=counts))
        ctx.set_option("async", 0)
        ctx.pip_join_count(table, x, y, out=counts)
        st = ctx.last_stats()
        ctx.set_option("async", 1)
        print(json.dumps({"variant": name, "ms": t, "pts_per_s": n / t * 1e3, **st, "info": table.info()}))
        table.close()


if __name__ == "__main__":
    main()
