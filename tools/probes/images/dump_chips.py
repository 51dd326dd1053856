"""Probe (not the product): writes the C4 chip set (synthetic_buildings(N) at H3 res 11, host
tessellation) in tests/native's chips.bin format for image_stats.cpp.  usage: dump_chips.py N OUT"""
import struct
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mosaic_amd.context import tessellate  # noqa: E402
from mosaic_amd.data import synthetic_buildings  # noqa: E402

n, out = int(float(sys.argv[1])), sys.argv[2]
chips = tessellate("H3", synthetic_buildings(n), 11)
offs, data = chips["wkb"]
ids, core, keys = chips["index_id"], chips["is_core"], chips["polygon_key"]
offs = np.asarray(offs)
with open(out, "wb") as f:
    f.write(struct.pack("<iI", 11, len(ids)))
    for i in range(len(ids)):
        w = bytes(data[offs[i]:offs[i + 1]])
        f.write(struct.pack("<qBiI", int(ids[i]), int(core[i]), int(keys[i]), len(w)))
        f.write(w)
print(len(ids))
