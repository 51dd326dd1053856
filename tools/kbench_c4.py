"""C4-shape chip join timing (GPU box): synthetic OSM-style buildings (mosaic_amd.data.
synthetic_buildings: rectangles / L-shapes, 8-40 m sides, clustered over the NYC bbox) chipped at
H3 res 11 (grid_tessellateexplode on the GPU; --host-tess: the host producer), points 70 % within 25 m of a building and 30 % uniform
(building_points_device).  BASELINE's C4 is 5e6 buildings x 2.5e8 points per GPU; --buildings
scales the build side (host tessellation ~30 us per building).  Prints one JSON line per variant.

    python tools/kbench_c4.py [--buildings 1e6] [--n 2.5e8] [--variants default raster]
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
    p.add_argument("--buildings", type=float, default=1e6)
    p.add_argument("--n", type=float, default=2.5e8)
    p.add_argument("--res", type=int, default=11)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--host-tess", action="store_true", help="host tessellator (default: this context's GPU)")
    p.add_argument("--variants", nargs="*", default=["default"],
                   help="default | tiles0 (generic path) | praster0 (tile path without the point raster)")
    args = p.parse_args()
    import torch

    from mosaic_amd import MosaicContext
    from mosaic_amd.context import tessellate
    from mosaic_amd.data import building_points_device, synthetic_buildings

    nb = int(args.buildings)
    t0 = time.perf_counter()
    b = synthetic_buildings(nb)
    t_gen = time.perf_counter() - t0
    ctx = MosaicContext.build("H3", "JTS")
    t0 = time.perf_counter()
    chips = tessellate("H3", b, args.res, ctx=None if args.host_tess else ctx)
    t_tess = time.perf_counter() - t0
    print(json.dumps({"buildings": nb, "chips": len(chips["index_id"]), "core_chips": int(chips["is_core"].sum()),
                      "generate_s": round(t_gen, 2), "tessellate_s": round(t_tess, 2)}), flush=True)
    n = int(args.n)
    x, y = building_points_device(b, n, seed=9)
    counts = torch.zeros(nb, dtype=torch.int64, device="cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    for v in args.variants:
        ctx.set_option("tiles", 0 if v == "tiles0" else 1)
        ctx.set_option("point_raster", 0 if v == "praster0" else 1)
        for kv in (v.split(",") if "=" in v else []):  # option sets, e.g. raster_min_segments=8
            k_, v_ = kv.split("=")
            ctx.set_option(k_, int(v_))
        t0 = time.perf_counter()
        table = ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], args.res,
                               n_polygons=nb)
        t_build = time.perf_counter() - t0
        ctx.set_option("async", 1)
        ctx.pip_join_count(table, x, y, out=counts)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            ctx.pip_join_count(table, x, y, out=counts)
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e))
        ctx.set_option("async", 0)
        ctx.pip_join_count(table, x, y, out=counts)
        st = ctx.last_stats()
        sorted_rows = ctx.last_binned_rows()
        ms = float(np.median(ts))
        print(json.dumps({"workload": f"C4 shape: {nb} buildings, H3 res {args.res}, {n} points", "variant": v,
                          "ms": ms, "points_per_s": n / ms * 1e3,
                          "contains_tests_per_s": st["contains_tests"] / ms * 1e3,
                          "pairs": int(counts.sum().item()), "contains_tests": st["contains_tests"],
                          "exact_path_rows": st["exact_path_rows"], "binned_rows": sorted_rows,
                          "build_s": round(t_build, 2),
                          "chips": table.info(), "tiles": table.tiles()}), flush=True)
        table.close()


if __name__ == "__main__":
    main()
