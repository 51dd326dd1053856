"""CPU-only: the ray-parity raster (mosaic_amd/csrc/raster.h) compiled for the host answers
contains() exactly like the full-ring JTS locate on the one-ring border chips of a real
tessellation, for uniform points and for points on / next to vertices, segments and raster cell
lines, at several raster sizes."""
import os
import struct
import subprocess

import numpy as np
import pytest

from mosaic_amd.context import tessellate
from mosaic_amd.data import PolygonSet
from mosaic_amd.wkb import read_wkb

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = tmp_path_factory.mktemp("raster") / "raster_sc"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-Wno-unknown-pragmas", "-o", str(out),
                    os.path.join(ROOT, "tests", "native", "raster_selfcheck.cpp")], check=True)
    return out


def _rings_file(path, chips, limit):
    offs, data = chips["wkb"]
    rings = []
    for i in np.nonzero(chips["is_core"] == 0)[0]:
        kind, parts = read_wkb(data[offs[i]:offs[i + 1]])
        if kind == "polygon" and len(parts) == 1 and len(parts[0]) == 1:
            rings.append(parts[0][0])
        if len(rings) >= limit:
            break
    with open(path, "wb") as f:
        f.write(struct.pack("<I", len(rings)))
        for r in rings:
            f.write(struct.pack("<I", len(r)))
            f.write(np.asarray(r, np.float64).tobytes())
    return len(rings)


@pytest.mark.parametrize("res,dims", [(9, 16), (9, 5), (8, 32), (7, 1)])
def test_raster_matches_ring_locate(exe, tmp_path, res, dims):
    zones = PolygonSet.load("nyc_taxi_zones_35")
    chips = tessellate("H3", zones, res)
    path = tmp_path / "rings.bin"
    nr = _rings_file(path, chips, 1500)
    assert nr > 50
    out = subprocess.run([str(exe), str(path), str(dims), "400", "7"], check=True, capture_output=True, text=True)
    bad, total, uni, uni_pure, _ = map(int, out.stdout.split())
    assert bad == 0, out.stderr
    assert total > nr * 300
    if dims >= 16:
        assert uni_pure > 0.5 * uni  # most uniform points are decided by the lookup alone
