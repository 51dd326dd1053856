"""Build-side probe (measurement only): the NYC zones tessellated three times in one context with
MOSAIC_BUILD_TRACE=1, to tell one-time device costs from per-call costs."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MOSAIC_BUILD_TRACE", "1")
import numpy as np  # noqa: E402

from mosaic_amd import MosaicContext  # noqa: E402
from mosaic_amd.data import PolygonSet  # noqa: E402

ctx = MosaicContext.build("H3", "JTS", device=0)
ctx.grid_longlatascellid(np.zeros(1), np.zeros(1), 9, raw=True)
zones = PolygonSet.load("nyc_taxi_zones")
for rep in range(3):
    t0 = time.perf_counter()
    chips = ctx.grid_tessellateexplode(zones, 9)
    print(f"rep {rep}: tessellate {1e3 * (time.perf_counter() - t0):.2f} ms", file=sys.stderr, flush=True)
