"""C4 build side at scale (GPU box): GPU tessellation and chip-table build of the full-size test's
dense building sets (test_gpu_configs.py::test_c4_full_size_five_million_buildings: 320 centres,
sigma 0.02 deg over a 0.25-degree box) at several sizes, with MOSAIC_BUILD_TRACE phase times on
stderr.  One JSON line per size.

    MOSAIC_BUILD_TRACE=1 python tools/c4_build_probe.py [--sizes 2e5 1e6 5e6]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--sizes", type=float, nargs="*", default=[2e5, 1e6, 5e6])
    p.add_argument("--table", type=int, default=1)
    args = p.parse_args()
    import torch

    from mosaic_amd import MosaicContext
    from mosaic_amd.data import synthetic_buildings

    ctx = MosaicContext.build("H3", "JTS")
    for s in args.sizes:
        nb = int(s)
        b = synthetic_buildings(nb, bbox=(-74.05, 40.60, -73.80, 40.85), n_centres=320, sigma=0.02)
        print(f"== {nb} buildings", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        chips = ctx.grid_tessellateexplode(b, 11)
        t_tess = time.perf_counter() - t0
        out = {"buildings": nb, "chips": len(chips["index_id"]), "tessellate_s": round(t_tess, 3)}
        if args.table:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            table = ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 11,
                                   n_polygons=nb)
            out["table_s"] = round(time.perf_counter() - t0, 3)
            out["info"] = table.info()
            table.close()
        print(json.dumps(out), flush=True)
        del chips


if __name__ == "__main__":
    main()
