"""Writes a tessellated chip set in the chips.bin format of tests/native/tiles_selfcheck.cpp
(int32 res, uint32 n, then per chip int64 cell, uint8 is_core, int32 key, uint32 len, wkb)."""
import struct
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mosaic_amd.context import tessellate  # noqa: E402
from mosaic_amd.data import PolygonSet  # noqa: E402


def dump(path, zones_name="nyc_taxi_zones", res=9):
    zones = PolygonSet.load(zones_name)
    chips = tessellate("H3", zones, res)
    offs, data = chips["wkb"]
    with open(path, "wb") as f:
        f.write(struct.pack("<iI", res, len(chips["index_id"])))
        for i in range(len(chips["index_id"])):
            w = bytes(data[offs[i]:offs[i + 1]])
            f.write(struct.pack("<qBiI", int(chips["index_id"][i]), int(chips["is_core"][i]),
                                int(chips["polygon_key"][i]), len(w)))
            f.write(w)
    print(zones.bbox())


if __name__ == "__main__":
    dump(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "nyc_taxi_zones", int(sys.argv[3]) if len(sys.argv) > 3 else 9)
