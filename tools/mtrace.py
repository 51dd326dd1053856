"""Per-wave phase times of k_join_mixed from a measurement build (-DMOSAIC_MIXED_TRACE, e.g.
abbuild/lib_tr.so via MOSAIC_HIP_LIB): C2 workload (1e9 uniform points, NYC zones, H3 res 9), one
join after a warm-up, then the wave timestamps (wall clock, 100 MHz): start, after the first
iteration's cell chains, after each of its two raster_chips calls, loop end, after the flush.
Usage: MOSAIC_HIP_LIB=abbuild/lib_tr.so python tools/mtrace.py [--n 1e9]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mosaic_amd import MosaicContext  # noqa: E402
from mosaic_amd import _native as N  # noqa: E402
from mosaic_amd.context import tessellate  # noqa: E402
from mosaic_amd.data import PolygonSet, uniform_points_device  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=float, default=1e9)
    args = p.parse_args()
    zones = PolygonSet.load("nyc_taxi_zones")
    chips = tessellate("H3", zones, 9)
    ctx = MosaicContext.build("H3")
    x, y = uniform_points_device(zones.bbox(), int(args.n), seed=1)
    counts = torch.zeros(len(zones), dtype=torch.int64, device="cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    table = ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 9,
                           n_polygons=len(zones))
    ctx.pip_join_count(table, x, y, out=counts)
    torch.cuda.synchronize()
    ctx.set_option("timing", 2)
    ctx.pip_join_count(table, x, y, out=counts)
    torch.cuda.synchronize()
    kt = ctx.kernel_times()
    buf = np.zeros(16384 * 8, np.uint64)
    f = N.lib().mosaic_debug_mtrace
    f.argtypes = [ctypes.c_void_p]
    f.restype = ctypes.c_int
    assert f(buf.ctypes.data) == 0
    t = buf.reshape(-1, 8).astype(np.int64)
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    ticks_us = 0.01  # 100 MHz
    out = {"kernel_ms": [float(v) for v in kt], "waves": int(len(t)), "stats": ctx.last_stats()}
    def pct(v):
        v = v * ticks_us
        return [round(float(np.percentile(v, q)), 1) for q in (0, 50, 90, 99, 100)]
    ran = t[:, 6] > 0
    out["start_us"] = pct(t[:, 0] - t0)
    out["end_us"] = pct(t[:, 5] - t0)
    out["life_us"] = pct(t[:, 5] - t[:, 0])
    out["iters"] = np.bincount(t[:, 6]).tolist()
    out["chains_us"] = pct(t[ran, 1] - t[ran, 0])
    out["raster0_us"] = pct(t[ran, 2] - t[ran, 1])
    out["raster1_us"] = pct(t[ran, 3] - t[ran, 2])
    out["rest_loop_us"] = pct(t[ran, 4] - t[ran, 3])
    out["flush_us"] = pct(t[:, 5] - t[:, 4])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
