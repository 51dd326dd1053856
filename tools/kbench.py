"""Kernel-level timing breakdown of the join (GPU box): cell kernel alone, join with every chip
marked core (no contains), full join; with and without the H3 tile directory.  Prints one JSON line per variant.

    python tools/kbench.py [--n 1e8] [--res 9]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


DEFAULTS = {"tile_lds": 1, "stream_persistent": 0, "blocks_per_cu": 8, "stream_mode": 0, "stream_block": 512, "probe_mask": 0, "stream_groups": 1, "mixed_rows": 4,
            "mixed_blocks_per_cu": 8}


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
    p.add_argument("--stream-mode", type=int, default=0, help="0 k_join_stream, 1 loader/worker k_join_stream_dec")
    p.add_argument("--groups", type=int, nargs="*", default=[1], help="stream_groups values")
    p.add_argument("--quads", type=int, nargs="*", default=[1], help="raster_quad values (1 default, else entry budget)")
    p.add_argument("--lines", type=int, nargs="*", default=[1], help="raster_lines values")
    p.add_argument("--stream-blocks", type=int, nargs="*", default=[], help="k_join_stream workgroup sizes to time")
    p.add_argument("--sweeps", nargs="*", default=[],
                   help="launch-option sets to time on each table, e.g. tile_lds=0 stream_block=512,probe_mask=8")
    p.add_argument("--modes", type=lambda v: tuple(int(q) for q in v.split(":")), nargs="*",
                   default=[(1, 1), (1, 0), (0, 0)], help="TILES:POINT_RASTER pairs")
    p.add_argument("--point-raster", type=lambda v: tuple(int(q) for q in v.split("x")), nargs="*",
                   default=[(32, 16)], help="point raster sizes SUBxCELL")
    p.add_argument("--stream-probes", type=int, nargs="*", default=[],
                   help="probe_mask values to time k_join_stream with (4 no sub lookups, 16 no counting, 32 no quad)")
    p.add_argument("--mixed-rows", type=int, nargs="*", default=[], help="k_join_mixed rows per lane to time")
    p.add_argument("--mixed-bpc", type=int, nargs="*", default=[], help="k_join_mixed blocks per CU to time")
    p.add_argument("--probe-mixed", action="store_true", help="time k_join_mixed without its chip loop / cell")
    p.add_argument("--all-core", action="store_true", help="also time every chip marked core")
    p.add_argument("--legacy", action="store_true", help="also time the coop / slab strategies")
    args = p.parse_args()
    import torch

    from mosaic_amd import MosaicContext
    from mosaic_amd.context import tessellate
    from mosaic_amd.data import PolygonSet, uniform_points_device

    zones = PolygonSet.load("nyc_taxi_zones")
    chips = tessellate("H3", zones, args.res)
    ctx = MosaicContext.build("H3")
    ctx.set_option("block", args.block)
    ctx.set_option("stream_mode", args.stream_mode)
    ctx.set_option("blocks_per_cu", args.bpc)
    n = int(args.n)
    if args.clustered:
        from mosaic_amd.data import clustered_points_device

        x, y = clustered_points_device(zones, n, seed=1)
    else:
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
    # floor: one core chip far from the points -> every point is outside the raster grid (no lookups)
    far = ctx.grid_longlatascellid(np.array([10.0]), np.array([10.0]), args.res, raw=True)
    ftab = ctx.chip_table(np.ones(1, np.uint8), far.astype(np.int64), [b""], np.zeros(1, np.int32), args.res,
                          n_polygons=len(zones))
    t = timeit(lambda: ctx.pip_join_count(ftab, x, y, out=counts))
    print(json.dumps({"variant": "stream_floor_no_lookups", "ms": t, "GBps": n * 16 / t / 1e6,
                      "raster": ftab.tiles()["raster"]}))
    ftab.close()
    variants = []
    for tiles, praster in args.modes:
        for sub, cell in (args.point_raster if praster else [(32, 16)]):
            for grp in args.groups:
                for quad in (args.quads if praster else [1]):
                    for ln in (args.lines if praster else [1]):
                        tag = f"tiles{tiles}_praster{praster}" + (f"_{sub}x{cell}_g{grp}" if praster else "")
                        tag += (f"_q{quad}" if quad != 1 else "") + ("" if ln else "_nolines")
                        if args.all_core:
                            variants.append((f"join_all_core_{tag}", True, 3, 16, 0, tiles, praster, (sub, cell), grp,
                                             quad, ln))
                        for r in args.rasters:
                            for le in args.lane_edges:
                                variants.append((f"join_raster{r}_lane{le}_{tag}", False, 3, r, le, tiles, praster,
                                                 (sub, cell), grp, quad, ln))
    if args.legacy:
        variants += [("join_full_coop", False, 1, 16, 8, 0, 0, (32, 16), 1, 1, 1),
                     ("join_full_slab", False, 2, 16, 8, 0, 0, (32, 16), 1, 1, 1)]
    for name, core, mode, raster, lane_edges, tiles, praster, (sub, cell), grp, quad, ln in variants:
        ctx.set_option("stream_groups", grp)
        ctx.set_option("raster_quad", quad)
        ctx.set_option("raster_lines", ln)
        ctx.set_option("tiles", tiles)
        ctx.set_option("point_raster", praster)
        ctx.set_option("raster_sub", sub)
        ctx.set_option("raster_cell", cell)
        ctx.set_option("pip_mode", mode)
        ctx.set_option("raster", raster)
        ctx.set_option("lane_edges", lane_edges)
        is_core = np.ones_like(chips["is_core"]) if core else chips["is_core"]
        tb0 = time.perf_counter()
        table = ctx.chip_table(is_core, chips["index_id"], chips["wkb"], chips["polygon_key"], args.res,
                               n_polygons=len(zones))
        build_s = time.perf_counter() - tb0
        t = timeit(lambda: ctx.pip_join_count(table, x, y, out=counts))
        ctx.set_option("timing", 2)
        ctx.pip_join_count(table, x, y, out=counts)
        kt = [round(v, 4) for v in ctx.kernel_times()]
        ctx.set_option("timing", 0)
        ctx.set_option("async", 0)
        ctx.pip_join_count(table, x, y, out=counts)
        st = ctx.last_stats()
        ctx.set_option("async", 1)
        tl = table.tiles()
        probes = {}
        for sb in args.stream_blocks:
            ctx.set_option("stream_block", sb)
            ctx.pip_join_count(table, x, y, out=counts)
            ctx.set_option("timing", 2)
            for _ in range(3):
                ctx.pip_join_count(table, x, y, out=counts)
            kt3 = ctx.kernel_times()
            probes[f"sblock{sb}_ms"] = [round(float(np.median(kt3[0::2])), 4), round(float(np.median(kt3[1::2])), 4)]
            ctx.set_option("timing", 0)
        ctx.set_option("stream_block", 512)
        for sw in args.sweeps:
            kv = [(q.split("=")[0], int(q.split("=")[1])) for q in sw.split(",")]
            for k, v in kv:
                ctx.set_option(k, v)
            ctx.pip_join_count(table, x, y, out=counts)
            ctx.set_option("timing", 2)
            for _ in range(3):
                ctx.pip_join_count(table, x, y, out=counts)
            kt3 = ctx.kernel_times()
            probes[sw] = [round(float(np.median(kt3[0::2])), 4), round(float(np.median(kt3[1::2])), 4)]
            ctx.set_option("timing", 0)
            for k, v in kv:
                ctx.set_option(k, DEFAULTS[k])
        for pm in args.stream_probes:
            ctx.set_option("probe_mask", pm)
            ctx.set_option("timing", 2)
            for _ in range(3):
                ctx.pip_join_count(table, x, y, out=counts)
            probes[f"stream_probe{pm}_ms"] = round(float(np.median(ctx.kernel_times()[0::2])), 4)
            ctx.set_option("timing", 0)
        ctx.set_option("probe_mask", 0)
        for mr in args.mixed_rows:
            ctx.set_option("mixed_rows", mr)
            ctx.set_option("timing", 2)
            for _ in range(3):
                ctx.pip_join_count(table, x, y, out=counts)
            probes[f"mixed_rows{mr}_ms"] = round(float(np.median(ctx.kernel_times()[1::2])), 4)
            ctx.set_option("timing", 0)
        ctx.set_option("mixed_rows", 4)
        for mb in args.mixed_bpc:
            ctx.set_option("mixed_blocks_per_cu", mb)
            ctx.set_option("timing", 2)
            for _ in range(3):
                ctx.pip_join_count(table, x, y, out=counts)
            probes[f"mixed_bpc{mb}_ms"] = round(float(np.median(ctx.kernel_times()[1::2])), 4)
            ctx.set_option("timing", 0)
        ctx.set_option("mixed_blocks_per_cu", 8)
        if args.probe_mixed and praster:
            for pm in (1, 3):
                ctx.set_option("probe_mask", pm)
                ctx.set_option("timing", 2)
                ctx.pip_join_count(table, x, y, out=counts)
                probes[f"mixed_probe{pm}_ms"] = round(float(ctx.kernel_times()[1]), 4)
                ctx.set_option("timing", 0)
            ctx.set_option("probe_mask", 0)
        print(json.dumps({"variant": name, "ms": t, "kernels_ms": kt, **probes, "pts_per_s": n / t * 1e3, **st,
                          "build_s": round(build_s, 2), "raster": {k: tl[k] for k in ("raster", "pure_sub_blocks", "mixed_sub_blocks", "line_sub_blocks", "mixed_cells", "raster_bytes")}}))
        table.close()


if __name__ == "__main__":
    main()
