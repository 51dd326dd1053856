"""BNG chip join timing (GPU box): the C5 shape -- London postcode zones (EPSG:27700
coordinates in metres, as in tests/test_gpu_parity.py::test_join_bng), BNG res 4 (100 m), uniform
points over the zones' bbox.  Prints one JSON line.

    python tools/kbench_bng.py [--n 1e9] [--res 4]
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
    p.add_argument("--n", type=float, default=1e9)
    p.add_argument("--res", type=int, default=4)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--cells", type=int, default=32, help="sub-cells per border cell side (bng_cell)")
    p.add_argument("--build-opts", default="", help="comma-separated key=value options set before the table build")
    p.add_argument("--sweep", nargs="*", default=[""], help="join option sets to time in turn, e.g. bng_cpt=0 bng_cpt=1")
    args = p.parse_args()
    import torch

    from mosaic_amd import MosaicContext
    from mosaic_amd.context import tessellate
    from mosaic_amd.data import PolygonSet, uniform_points_device

    proj = PolygonSet.load("london_postcodes_bng")  # EPSG:27700 (tests/golden/make_bng_fixture.py)
    t0 = time.perf_counter()
    chips = tessellate("BNG", proj, args.res)
    t_tess = time.perf_counter() - t0
    ctx = MosaicContext.build("BNG")
    ctx.set_option("bng_cell", args.cells)
    for kv in filter(None, args.build_opts.split(",")):
        k, v = kv.split("=")
        ctx.set_option(k, int(v))
    t0 = time.perf_counter()
    table = ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], args.res,
                           n_polygons=len(proj))
    t_build = time.perf_counter() - t0
    n = int(args.n)
    x, y = uniform_points_device(proj.bbox(), n, seed=5)
    counts = torch.zeros(len(proj), dtype=torch.int64, device="cuda")
    for opts in args.sweep:
        for kv in filter(None, opts.split(",")):
            k, v = kv.split("=")
            ctx.set_option(k, int(v))
        ctx.set_stream(torch.cuda.current_stream().cuda_stream)
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
        ctx.set_option("timing", 2)
        for _ in range(args.reps):
            ctx.pip_join_count(table, x, y, out=counts)
        kt = ctx.kernel_times()
        ctx.set_option("timing", 0)
        ctx.pip_join_count(table, x, y, out=counts)
        st = ctx.last_stats()
        ms = float(np.median(ts))
        print(json.dumps({"workload": f"BNG res {args.res}, {len(proj)} London zones (EPSG:27700), {n} uniform points",
                          "build_opts": args.build_opts, "options": opts, "kernel": ctx.last_kernel(), "raster_cell": args.cells,
                          "ms": ms, "stream_ms": round(float(np.median(kt[0::2])), 4), "mixed_ms": round(float(np.median(kt[1::2])), 4),
                          "stream_frac_of_8TBps": round(16.0 * n / (float(np.median(kt[0::2])) * 1e-3) / 8e12, 4),
                          "points_per_s": n / ms * 1e3, "GBps": n * 16 / ms / 1e6, "chips": table.info(),
                          "tiles": table.tiles(), "tessellate_s": round(t_tess, 2), "build_s": round(t_build, 2),
                          "pair_count": int(counts.sum().item()), "exact_path_rows": st["exact_path_rows"],
                          "contains_tests": st["contains_tests"]}))




if __name__ == "__main__":
    main()
