"""GPU box: k_cell_h3's grid (option cell_blocks_per_cu; 0 = one lane per row group) against its time -- mosaic_point_to_cell on 1e9
resident NYC-bbox points, res 9, HIP events on the context's stream, best and median of 5 calls per
setting.

    python tools/cell_sweep.py [n] [bpc,bpc,...]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from mosaic_amd import MosaicContext
    from mosaic_amd import _native as N
    from mosaic_amd.data import PolygonSet, uniform_points_device

    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
    bpcs = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "8,32,64").split(",")]
    key = os.environ.get("CELL_SWEEP_KEY", "cell_blocks_per_cu")  # (blocks_per_cu before round 6's option)
    zones = PolygonSet.load("nyc_taxi_zones")
    ctx = MosaicContext.build("H3")
    x, y = uniform_points_device(zones.bbox(), n, seed=1)
    out = torch.empty(n, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()
    ctx.set_stream(s.cuda_stream)
    ref = None
    for bpc in bpcs:
        ctx.set_option(key, bpc)
        ts = []
        for _ in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            N.check(N.lib().mosaic_point_to_cell(ctx.handle, 0, 9, x.data_ptr(), y.data_ptr(), None, n,
                                                 out.data_ptr(), None))
            e1.record(s)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts = sorted(ts[1:])
        h = int(out[::9973].sum())
        ref = h if ref is None else ref
        print(f"{key} {bpc:4d}: best {ts[0]:.3f} ms  median {ts[2]:.3f} ms  digest_ok {h == ref}",
              flush=True)


if __name__ == "__main__":
    main()
