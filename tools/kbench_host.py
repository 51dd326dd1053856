"""PCIe-inclusive join rate (GPU box): the 263 NYC zones at H3 res 9 joined with 2e8 uniform points
that live in host memory (numpy, pageable; and pinned torch tensors), against the same points
resident in HBM.  host_chunk = 0 stages the whole batch before the join; > 0 overlaps each chunk's
copy with the previous chunk's join.  One JSON line per case."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from mosaic_amd import MosaicContext
    from mosaic_amd.context import tessellate
    from mosaic_amd.data import PolygonSet, uniform_points

    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 200_000_000
    zones = PolygonSet.load("nyc_taxi_zones")
    chips = tessellate("H3", zones, 9)
    ctx = MosaicContext.build("H3")
    table = ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 9,
                           n_polygons=len(zones))
    x, y = uniform_points(zones.bbox(), n, config=2, seed=5)

    def run(label, xs, ys, chunk, reps=3):
        ctx.set_option("host_chunk", chunk)
        ref = ctx.pip_join_count(table, xs, ys)
        ref = ref.cpu().numpy() if hasattr(ref, "cpu") else np.array(ref)
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ctx.pip_join_count(table, xs, ys)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        t = float(np.median(ts))
        print(json.dumps({"case": label, "host_chunk": chunk, "points": n, "s": t, "points_per_s": n / t,
                          "GBps_in": 16 * n / t / 1e9, "total_pairs": int(ref.sum())}), flush=True)
        return ref

    base = run("host pageable, staged whole", x, y, 0)
    for chunk in (1 << 24, 1 << 25, 1 << 26):
        assert np.array_equal(run("host pageable, chunked", x, y, chunk), base)
    xp = torch.from_numpy(x).pin_memory()
    yp = torch.from_numpy(y).pin_memory()
    assert np.array_equal(run("host pinned, staged whole", xp, yp, 0), base)
    assert np.array_equal(run("host pinned, chunked", xp, yp, 1 << 25), base)
    xd, yd = xp.cuda(), yp.cuda()
    out = torch.zeros(len(zones), dtype=torch.int64, device="cuda")
    ctx.set_option("host_chunk", 1 << 25)
    ctx.pip_join_count(table, xd, yd, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        ctx.pip_join_count(table, xd, yd, out=out)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / 3
    assert np.array_equal(out.cpu().numpy(), base)
    print(json.dumps({"case": "device resident (HBM)", "points": n, "s": t, "points_per_s": n / t}), flush=True)


if __name__ == "__main__":
    main()
