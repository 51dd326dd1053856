"""Build-side variance probe: the NYC res-9 chip table built 6 times in one process
(tessellation on the GPU first), each build's phases (mosaic_chip_table_build_info) printed -- a
process whose first builds are slow and later ones fast points at device state (clocks) rather than
at the build's work.  usage: python tools/build_var.py [--sleep S]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--sleep", type=float, default=0.0, help="idle seconds before each build")
    p.add_argument("--reps", type=int, default=6)
    args = p.parse_args()
    from mosaic_amd import MosaicContext
    from mosaic_amd.data import PolygonSet

    zones = PolygonSet.load("nyc_taxi_zones")
    ctx = MosaicContext.build("H3")
    t0 = time.perf_counter()
    chips = ctx.grid_tessellateexplode(zones, 9)
    tess = time.perf_counter() - t0
    for r in range(args.reps):
        if args.sleep:
            time.sleep(args.sleep)
        t0 = time.perf_counter()
        table = ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 9,
                               n_polygons=len(zones))
        wall = time.perf_counter() - t0
        print(json.dumps({"rep": r, "sleep": args.sleep, "tess_s": round(tess, 4), "build_s": round(wall, 4),
                          **{k: round(v, 2) for k, v in table.build_info().items() if k.endswith("_ms")}}), flush=True)
        table.close()


if __name__ == "__main__":
    main()
