"""Profiling driver (GPU box): runs the H3 cell kernel and the raster join on 1e8 resident points
a few times, nothing else, so PMC passes see only these launches.

    rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace -d ... -- python tools/cellrun.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from mosaic_amd import MosaicContext
    from mosaic_amd import _native as N
    from mosaic_amd.context import tessellate
    from mosaic_amd.data import PolygonSet, uniform_points_device

    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000_000
    zones = PolygonSet.load("nyc_taxi_zones")
    chips = tessellate("H3", zones, 9)
    ctx = MosaicContext.build("H3")
    x, y = uniform_points_device(zones.bbox(), n, seed=1)
    out = torch.empty(n, dtype=torch.int64, device="cuda")
    counts = torch.zeros(len(zones), dtype=torch.int64, device="cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    table = ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 9,
                           n_polygons=len(zones))
    for _ in range(3):
        N.check(N.lib().mosaic_point_to_cell(ctx.handle, 0, 9, x.data_ptr(), y.data_ptr(), None, n,
                                             out.data_ptr(), None))
        ctx.pip_join_count(table, x, y, out=counts)
    torch.cuda.synchronize()
    print("ok", int(counts.sum()))


if __name__ == "__main__":
    main()
