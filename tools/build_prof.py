"""Build-side timing (GPU box): tessellation (GPU classification) and chip-table build of the NYC
zones, three times each on a warm context; prints the per-phase times.  Run under
`rocprofv3 --kernel-trace --stats` for the per-kernel split.

    python tools/build_prof.py [--res 9]
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
    p.add_argument("--res", type=int, default=9)
    p.add_argument("--reps", type=int, default=3)
    args = p.parse_args()
    from mosaic_amd import MosaicContext
    from mosaic_amd.data import PolygonSet

    zones = PolygonSet.load("nyc_taxi_zones")
    ctx = MosaicContext.build("H3", "JTS")
    t0 = time.perf_counter()
    ctx.grid_longlatascellid(np.zeros(1), np.zeros(1), args.res, raw=True)
    init_s = time.perf_counter() - t0
    for rep in range(args.reps):
        t0 = time.perf_counter()
        chips = ctx.grid_tessellateexplode(zones, args.res)
        tess_s = time.perf_counter() - t0
        t0 = time.perf_counter()
        table = ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], args.res,
                               n_polygons=len(zones))
        table_s = time.perf_counter() - t0
        print(json.dumps({"rep": rep, "gpu_init_s": round(init_s, 3), "tessellate_ms": round(tess_s * 1e3, 1),
                          "classify_kernel_ms": round(ctx.tess_last_classify_ms(), 2) if hasattr(ctx, "tess_last_classify_ms") else None,
                          "chip_table_ms": round(table_s * 1e3, 1),
                          **{k: (round(v, 1) if k.endswith("_ms") else v) for k, v in table.build_info().items()}}),
              flush=True)
        table.close()


if __name__ == "__main__":
    main()
