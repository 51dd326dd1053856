"""Profiling driver (GPU box): runs the res-9 NYC chip join on 1e8 resident uniform points a few
times with one point-raster configuration, nothing else, so PMC passes see only these launches.

    rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -- python tools/joinrun.py 32x16
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from mosaic_amd import MosaicContext
    from mosaic_amd.context import tessellate
    from mosaic_amd.data import PolygonSet, uniform_points_device

    sub, cell = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "32x16").split("x"))
    n = int(float(sys.argv[2])) if len(sys.argv) > 2 else 100_000_000
    zones = PolygonSet.load("nyc_taxi_zones")
    chips = tessellate("H3", zones, 9)
    ctx = MosaicContext.build("H3")
    ctx.set_option("raster_sub", sub)
    ctx.set_option("raster_cell", cell)
    x, y = uniform_points_device(zones.bbox(), n, seed=1)
    counts = torch.zeros(len(zones), dtype=torch.int64, device="cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    table = ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 9,
                           n_polygons=len(zones))
    for _ in range(3):
        ctx.pip_join_count(table, x, y, out=counts)
    torch.cuda.synchronize()
    print("ok", int(counts.sum()), table.tiles())


if __name__ == "__main__":
    main()
