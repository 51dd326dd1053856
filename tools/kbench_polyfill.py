"""grid_polyfill throughput: mosaic_polyfill (GPU) over the 263 NYC taxi zones (H3 res 9-11) and the
177 London postcode zones in EPSG:27700 (BNG res 3-4), against the CPU oracle (oracle/polyfill.c,
one thread) on the same input.  Reports wall time of the call, device time (HIP events), cells,
and whether the cell lists equal the oracle's (sets; H3 lists in order where the oracle's is
certain).  Usage: python tools/kbench_polyfill.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import oracle  # noqa: E402  (the checker / CPU baseline only)
from mosaic_amd import MosaicContext  # noqa: E402
from mosaic_amd import _native as N  # noqa: E402
from mosaic_amd.data import PolygonSet  # noqa: E402


def run(ctx, ps, res, oracle_fn, name):
    ctx.grid_polyfill(ps, res, raw=True)  # warm-up (module load, allocations)
    t = time.perf_counter()
    rows = ctx.grid_polyfill(ps, res, raw=True)
    wall = time.perf_counter() - t
    dev = N.lib().mosaic_polyfill_last_ms()
    t = time.perf_counter()
    same, ordered = True, 0
    for g in range(len(ps)):
        want, cf = oracle_fn(ps, g, res)
        same &= sorted(rows[g].tolist()) == sorted(want.tolist())
        if cf and rows[g].tolist() == want.tolist():
            ordered += 1
    cpu = time.perf_counter() - t
    n = sum(len(r) for r in rows)
    print(f"{name} res {res}: {len(ps)} geometries -> {n} cells; GPU call {wall * 1e3:.1f} ms (device {dev:.1f} ms), "
          f"{n / wall:.3g} cells/s; CPU oracle (1 thread) {cpu:.2f} s; equal {same}, order-checked rows {ordered}",
          flush=True)


def h3_oracle(ps, g, res):
    parts = [r for r in ps.parts(g) if r and len(r[0])]
    out = [oracle.h3_polyfill_part(r, res) for r in parts]
    cells = np.concatenate([c for c, _ in out]) if out else np.zeros(0, np.int64)
    return cells, all(cf for _, cf in out)


def bng_oracle(ps, g, res):
    return oracle.bng_polyfill(ps.parts(g), res), False


def main():
    h3 = MosaicContext.build("H3", "JTS")
    zones = PolygonSet.load("nyc_taxi_zones")
    for res in (9, 10, 11):
        run(h3, zones, res, h3_oracle, "H3 NYC zones")
    h3.close()
    bng = MosaicContext.build("BNG", "JTS")
    london = PolygonSet.load("london_postcodes_bng")
    for res in (3, 4):
        run(bng, london, res, bng_oracle, "BNG London zones")
    bng.close()


if __name__ == "__main__":
    main()
