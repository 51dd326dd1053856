"""BNG cell-column kernels on the GPU box: serializeCellId (mosaic_bng_format_column) and
grid_boundaryaswkb (mosaic_cell_boundary_wkb) over 2e8 res-4 ("100m") ids resident in HBM, outputs
in HBM.  One JSON line per kernel (rows/s and output GB/s)."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from mosaic_amd import MosaicContext
    from mosaic_amd import _native as N

    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 200_000_000
    ctx = MosaicContext.build("BNG")
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.rand(n, dtype=torch.float64, device="cuda", generator=g) * 699_999
    y = torch.rand(n, dtype=torch.float64, device="cuda", generator=g) * 1_299_999
    ids = ctx.grid_longlatascellid(x, y, 4, raw=True)
    del x, y
    offs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    chars = torch.empty(93 * n, dtype=torch.uint8, device="cuda")  # serves both outputs
    need = ctypes.c_int64(0)

    def fmt():
        N.check(N.lib().mosaic_bng_format_column(ctx.handle, ids.data_ptr(), None, n, offs.data_ptr(),
                                                 chars.data_ptr(), 16 * n, ctypes.byref(need)))

    def wkb():
        N.check(N.lib().mosaic_cell_boundary_wkb(ctx.handle, N.GRID_BNG, ids.data_ptr(), None, n, chars.data_ptr()))

    for name, fn, out_bytes in (("bng_format_column", fmt, None), ("cell_boundary_wkb", wkb, 93 * n)):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / 5
        ob = out_bytes if out_bytes is not None else need.value + 8 * (n + 1)
        print(json.dumps({"kernel": name, "rows": n, "ms": t * 1e3, "rows_per_s": n / t,
                          "out_GBps": ob / t / 1e9}), flush=True)


if __name__ == "__main__":
    main()
