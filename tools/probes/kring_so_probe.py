"""GPU probe: mosaic_cell_kring (libmosaic_hip.so) over tools/probes/kring_cells.txt at k: prints
"row count first" per row, as kring_probe does for h3_neighbors.h compiled alone."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mosaic_amd import MosaicContext  # noqa: E402
from mosaic_amd import _native as N  # noqa: E402

cells = np.array([int(v) for v in open(sys.argv[1]).read().split()], np.int64)
k = int(sys.argv[2])
ctx = MosaicContext.build("H3", "JTS")
stride = 1 + 3 * k * (k + 1)
out = np.zeros(len(cells) * stride, np.int64)
cnt = np.zeros(len(cells), np.int32)
N.check(N.lib().mosaic_cell_kring(ctx.handle, N.GRID_H3, N.ptr(cells), None, len(cells), k, 0, N.ptr(out), N.ptr(cnt)))
for i in range(len(cells)):
    print(i, cnt[i], out[i * stride + 1] if cnt[i] > 0 else 0)
