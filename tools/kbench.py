"""Kernel-level timing of the H3 chip join on one GPU (device-resident points): the stream kernel
and the mixed-row kernel (HIP events on the launch stream), the whole call, the table build, for
the NYC zones at a resolution.  Prints one JSON line per variant.

    python tools/kbench.py [--n 1e9] [--res 9] [--clustered] [--stream-blocks 1024 512]
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
    p.add_argument("--res", type=int, default=9)
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--clustered", action="store_true", help="C3 mixture (sigma 0.002 deg) instead of uniform")
    p.add_argument("--zones", default="nyc_taxi_zones")
    p.add_argument("--stream-blocks", type=int, nargs="*", default=[1024])
    p.add_argument("--point-raster", type=lambda v: tuple(int(q) for q in v.split("x")), nargs="*",
                   default=[(64, 16)], help="point raster sizes SUBxCELL")
    p.add_argument("--quads", type=int, nargs="*", default=[1], help="raster_quad values (1 default, else entry budget)")
    p.add_argument("--modes", type=lambda v: tuple(int(q) for q in v.split(":")), nargs="*", default=[(1, 1)],
                   help="TILES:POINT_RASTER pairs")
    p.add_argument("--sweep", nargs="*", default=[""], help="option sets to time, e.g. stream_pipe=0 stream_pipe=1")
    p.add_argument("--build-opts", nargs="*", default=[""],
                   help="option sets applied before each table build, e.g. raster_quad_records=0")
    p.add_argument("--save-chips", default="", help="write the chip set to this .npz (A/B of chips against code)")
    p.add_argument("--chips", default="", help="join these chips (.npz from --save-chips) instead of tessellating")
    args = p.parse_args()
    import torch

    from mosaic_amd import MosaicContext
    from mosaic_amd.context import tessellate
    from mosaic_amd.data import PolygonSet, clustered_points_device, uniform_points_device

    zones = PolygonSet.load(args.zones)
    t0 = time.perf_counter()
    if args.chips:
        z = np.load(args.chips)
        chips = {"is_core": z["is_core"], "index_id": z["index_id"], "polygon_key": z["polygon_key"],
                 "wkb": (z["wkb_offsets"], z["wkb_data"])}
    else:
        chips = tessellate("H3", zones, args.res)
    if args.save_chips:
        np.savez(args.save_chips, is_core=chips["is_core"], index_id=chips["index_id"], polygon_key=chips["polygon_key"],
                 wkb_offsets=chips["wkb"][0], wkb_data=chips["wkb"][1])
    tess_s = time.perf_counter() - t0
    ctx = MosaicContext.build("H3")
    n = int(args.n)
    if args.clustered:
        x, y = clustered_points_device(zones, n, seed=1)
    else:
        x, y = uniform_points_device(zones.bbox(), n, seed=1)
    counts = torch.zeros(len(zones), dtype=torch.int64, device="cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ref = None
    for sub, cell, quad, bo in [(s_, c_, q_, b_) for s_, c_ in args.point_raster for q_ in args.quads
                                for b_ in args.build_opts]:
        if True:
            for kv in filter(None, bo.split(",")):
                k, v = kv.split("=")
                ctx.set_option(k, int(v))
            ctx.set_option("raster_sub", sub)
            ctx.set_option("raster_cell", cell)
            ctx.set_option("raster_quad", quad)
            t0 = time.perf_counter()
            table = ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], args.res,
                                   n_polygons=len(zones))
            build_s = time.perf_counter() - t0
            tl = table.tiles()
            binfo = table.build_info()
            for tiles, praster in args.modes:
                ctx.set_option("tiles", tiles)
                ctx.set_option("point_raster", praster)
                for sb, sw in [(b, w) for b in args.stream_blocks for w in args.sweep]:
                    ctx.set_option("stream_block", sb)
                    for kv in filter(None, sw.split(",")):
                        k, v = kv.split("=")
                        ctx.set_option(k, int(v))
                    ctx.pip_join_count(table, x, y, out=counts)
                    torch.cuda.synchronize()
                    ctx.set_option("timing", 2)
                    ts = []
                    for _ in range(args.reps):
                        s = torch.cuda.Event(enable_timing=True)
                        e = torch.cuda.Event(enable_timing=True)
                        s.record()
                        ctx.pip_join_count(table, x, y, out=counts)
                        e.record()
                        torch.cuda.synchronize()
                        ts.append(s.elapsed_time(e))
                    kt = ctx.kernel_times()
                    ctx.set_option("timing", 0)
                    got = counts.cpu().numpy()
                    if ref is None:
                        ref = got
                    stats = ctx.last_stats()
                    step = float(np.median(ts))
                    line = {"res": args.res, "clustered": args.clustered, "n": n, "raster": f"{sub}x{cell}",
                            "quad": quad, "build_opts": bo, "build_ms": {k: round(v, 1) for k, v in binfo.items()
                                                                          if k.endswith("_ms")}, "tiles": tiles, "point_raster": praster, "stream_block": sb, "options": sw,
                            "call_ms": round(step, 4), "points_per_s": n / (step * 1e-3),
                            "same_counts": bool(np.array_equal(got, ref)), "pairs": int(got.sum()),
                            "tess_s": round(tess_s, 2), "build_s": round(build_s, 2),
                            "raster_bytes": tl.get("raster_bytes"), "quad_entries": tl.get("quad_entries"),
                            "stats": stats}
                    if tiles and praster and len(kt) >= 2:
                        line["stream_ms"] = round(float(np.median(kt[0::2])), 4)
                        line["mixed_ms"] = round(float(np.median(kt[1::2])), 4)
                        line["stream_frac_of_8TBps"] = round(16.0 * n / (line["stream_ms"] * 1e-3) / 8e12, 4)
                    elif len(kt):
                        line["kernel_ms"] = round(float(np.median(kt)), 4)
                    print(json.dumps(line), flush=True)
            ctx.set_option("tiles", 1)
            ctx.set_option("point_raster", 1)
            table.close()
            for kv in filter(None, bo.split(",")):  # build options back to their defaults
                k, _ = kv.split("=")
                ctx.set_option(k, {"raster_quad_records": 1, "raster_build": 1, "raster_lines": 1}.get(k, 1))


if __name__ == "__main__":
    main()
