"""Point-geometry decode timing (GPU box): a WKT / WKB column of taxi-GPS points resident in HBM
(Arrow utf8 / binary layout, int32 offsets), decoded by k_decode_points (mosaic_point_geom_decode)
and indexed (mosaic_point_geom_to_cell, decode + H3 res 9).  Prints one JSON line per format.

    python tools/kbench_decode.py [--n 1e8] [--reps 5]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=float, default=1e8)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--formats", nargs="*", default=["wkt6", "wkt17", "wkb"])
    args = p.parse_args()
    import torch

    from mosaic_amd import MosaicContext
    from mosaic_amd import _native as N

    n = int(args.n)
    ctx = MosaicContext.build("H3", "JTS")
    rng = np.random.default_rng(5)
    base = 1 << 20  # distinct rows, tiled on the device to n rows
    x = np.round(rng.uniform(-74.25, -73.70, base), 6)
    y = np.round(rng.uniform(40.50, 40.91, base), 6)
    for fmt in args.formats:
        if fmt == "wkt6":
            rows = [("POINT (%.6f %.6f)" % (a, b)).encode() for a, b in zip(x, y)]
        elif fmt == "wkt17":  # JTS WKTWriter-style full precision
            xx, yy = x + rng.uniform(0, 1e-6, base), y + rng.uniform(0, 1e-6, base)
            rows = [("POINT (%r %r)" % (float(a), float(b))).encode() for a, b in zip(xx, yy)]
        else:
            from mosaic_amd.wkb import point_wkb

            rows = [point_wkb(a, b, big_endian=False) for a, b in zip(x, y)]
        lens = np.array([len(r) for r in rows], np.int64)
        reps = n // base
        total = int(lens.sum()) * reps
        if total >= 2 ** 31:
            reps = (2 ** 31 - 1) // int(lens.sum())
        nn = base * reps
        offs = np.zeros(nn + 1, np.int64)
        np.cumsum(np.tile(lens, reps), out=offs[1:])
        data = torch.tensor(np.frombuffer(b"".join(rows), np.uint8), device="cuda").repeat(reps)
        doffs = torch.tensor(offs.astype(np.int32), device="cuda")
        del offs
        f = (N.GEOM_WKB if fmt == "wkb" else N.GEOM_WKT) | N.GEOM_OFFSETS32
        dx = torch.empty(nn, dtype=torch.float64, device="cuda")
        dy = torch.empty_like(dx)
        st = torch.empty(nn, dtype=torch.uint8, device="cuda")
        cells = torch.empty(nn, dtype=torch.int64, device="cuda")
        rp = ctypes.c_int64(0)
        L = N.lib()

        def dec():
            N.check(L.mosaic_point_geom_decode(ctx.handle, f, N.ptr(doffs), N.ptr(data), None, nn, N.ptr(dx), N.ptr(dy),
                                               N.ptr(st), ctypes.byref(rp)))

        def cell():
            N.check(L.mosaic_point_geom_to_cell(ctx.handle, 0, 9, f, N.ptr(doffs), N.ptr(data), None, nn, N.ptr(cells),
                                                N.ptr(st), ctypes.byref(rp)))

        out = {"format": fmt, "rows": nn, "bytes_per_row": float(lens.mean()), "value_bytes": int(lens.sum()) * reps}
        for name, fn in (("decode", dec), ("to_cell", cell)):
            fn()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(args.reps):
                fn()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / args.reps
            out[name + "_ms"] = dt * 1e3
            out[name + "_rows_per_s"] = nn / dt
            # algorithmic bytes: values + offsets in, x / y / status (decode) or cell / status out
            io = out["value_bytes"] + 4 * nn + (17 if name == "decode" else 9) * nn
            out[name + "_GBps"] = io / dt / 1e9
        assert rp.value == 0
        print(json.dumps(out), flush=True)
        del data, doffs, dx, dy, st, cells
        torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main()
