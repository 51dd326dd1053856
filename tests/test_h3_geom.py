"""H3 cell geometry (h3ToGeo / h3ToGeoBoundary) for grid_boundaryaswkb, indexToGeometry,
getBufferRadius and polyfill (reference H3IndexSystem.scala:73-126; kernel code
mosaic_amd/csrc/h3_geom.h).

The kernel code compiled for the host must equal the oracle (oracle/h3.c: H3 C v3.7 restated with
real x87 long double and the host glibc) bit for bit -- centres and every boundary vertex, for
cells of every resolution around the globe, pentagons and the Class III face-crossing cells with
distortion vertices included.  The oracle itself is checked geometrically (tests below): each
vertex lies on its cell (points just inside map back to the cell), the centre maps to the cell.
Reference-held vectors for H3 boundaries do not exist (docs show only a truncated WKB), so the
restatement of H3's boundary algorithm is parity-unpinned beyond those properties."""
import ctypes
import math
import os
import subprocess

import numpy as np
import pytest

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def host_geom(tmp_path_factory):
    so = tmp_path_factory.mktemp("h3g") / "libh3g.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-Wno-unknown-pragmas", "-shared", "-fPIC",
                    "-I", os.path.join(ROOT, "mosaic_amd", "csrc"), "-o", str(so),
                    os.path.join(ROOT, "tests", "native", "h3_geom_host.cpp")], check=True)
    lib = ctypes.CDLL(str(so))
    for fn in (lib.h3_boundary_host, lib.h3_center_host):
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.c_int64, ctypes.c_void_p]

    def boundary(cell):
        out = np.zeros(20)
        n = lib.h3_boundary_host(int(cell), out.ctypes.data_as(ctypes.c_void_p))
        return [(float(out[2 * i]), float(out[2 * i + 1])) for i in range(n)]

    def center(cell):
        out = np.zeros(2)
        assert lib.h3_center_host(int(cell), out.ctypes.data_as(ctypes.c_void_p)) == 1
        return float(out[0]), float(out[1])
    return boundary, center


def cells_everywhere(n, seed):
    rng = np.random.default_rng(seed)
    lat = np.degrees(np.arcsin(rng.uniform(-1, 1, n)))
    lon = rng.uniform(-180, 180, n)
    res = rng.integers(0, 16, n)
    return [int(oracle.h3_point_to_index(lon[i:i + 1], lat[i:i + 1], int(res[i]))[0]) for i in range(n)]


def pentagons(res):
    # the 12 pentagons: centre children of the pentagon base cells
    out = []
    for bc in (4, 14, 24, 38, 49, 58, 63, 72, 83, 97, 107, 117):
        h = (1 << 59) | (res << 52) | (bc << 45) | ((1 << 45) - 1)
        for r in range(1, res + 1):
            h &= ~(7 << ((15 - r) * 3))
        out.append(h)
    return out


def test_host_kernel_code_equals_oracle(host_geom):
    boundary, center = host_geom
    cells = cells_everywhere(6000, 1) + [p for r in range(16) for p in pentagons(r)]
    nv = {}
    for c in cells:
        assert center(c) == oracle.h3_to_geo(c), hex(c)
        got, want = boundary(c), oracle.h3_to_geo_boundary(c)
        assert got == want, hex(c)
        nv[len(want)] = nv.get(len(want), 0) + 1
    # Class II pentagons have 5 vertices, Class III ones 10 (an edge-crossing vertex per edge);
    # Class III hexagons crossing a face edge 7 or 8
    assert nv.get(5, 0) >= 12 * 8 and nv.get(10, 0) >= 12 * 8 and nv.get(7, 0) + nv.get(8, 0) > 20, nv


def test_nyc_cells_bit_exact(host_geom):
    boundary, center = host_geom
    rng = np.random.default_rng(2)
    for res in range(0, 16):
        lon = rng.uniform(-74.25, -73.70, 50)
        lat = rng.uniform(40.50, 40.91, 50)
        for c in oracle.h3_point_to_index(lon, lat, res).tolist():
            assert boundary(c) == oracle.h3_to_geo_boundary(c)
            assert center(c) == oracle.h3_to_geo(c)


def test_oracle_boundary_geometry():
    # every vertex is a corner of its cell: a point 2% of the way to the centre maps to the cell;
    # the centre maps to the cell (res >= 2, away from the poles' lat/lng interpolation)
    rng = np.random.default_rng(3)
    checked = 0
    for t in range(1500):
        lat = math.degrees(math.asin(rng.uniform(-0.98, 0.98)))
        lon = rng.uniform(-180, 180)
        res = int(rng.integers(2, 16))
        c = int(oracle.h3_point_to_index(np.array([lon]), np.array([lat]), res)[0])
        clat, clon = oracle.h3_to_geo(c)
        assert oracle.h3_geo_to_h3(clat, clon, res) == c
        for vl, vg in oracle.h3_to_geo_boundary(c):
            dl = (clon - vg + math.pi) % (2 * math.pi) - math.pi
            assert oracle.h3_geo_to_h3(vl + 0.02 * (clat - vl), vg + 0.02 * dl, res) == c
            checked += 1
    assert checked > 8000


@pytest.mark.gpu
def test_gpu_h3_geometry_equals_oracle(host_geom):
    """mosaic_h3_cell_geometry on the GPU: centres, boundary vertices and grid_boundaryaswkb bytes
    equal the oracle (degrees via JDK 8 Math.toDegrees), pentagons and distortion cells included;
    invalid ids raise."""
    import struct

    from mosaic_amd import MosaicContext, MosaicError

    def deg(r):
        return r * 180.0 / 3.141592653589793

    h3 = MosaicContext.build("H3", "JTS")
    cells = cells_everywhere(20000, 4) + [p for r in range(16) for p in pentagons(r)]
    cen = h3.grid_cellcenter(cells)
    bnd = h3.grid_boundary(cells)
    wkb = h3.grid_boundaryaswkb(cells)
    for i, c in enumerate(cells):
        lat, lon = oracle.h3_to_geo(c)
        assert (cen[i, 0], cen[i, 1]) == (deg(lon), deg(lat))
        want = [(deg(g), deg(a)) for a, g in oracle.h3_to_geo_boundary(c)]
        assert [tuple(v) for v in bnd[i].tolist()] == want, hex(c)
        ring = want + want[:1]
        assert wkb[i] == struct.pack(">BIII", 0, 3, 1, len(ring)) + b"".join(struct.pack(">dd", x, y) for x, y in ring)
    with pytest.raises(MosaicError):
        h3.grid_boundaryaswkb([cells[0], 12345])
    # mixed waves (tools/probes/early_exit: a bool decided inside a divergent loop was misread by
    # lanes that left it early): 64 cells of every resolution with one digit-7 id at each lane in
    # turn -- its lane leaves the digit check first -- must raise every time, and the valid batch
    # must still equal the oracle
    rng = np.random.default_rng(64)
    lat, lon = np.degrees(np.arcsin(rng.uniform(-1, 1, 64))), rng.uniform(-180, 180, 64)
    wave = [int(oracle.h3_point_to_index(lon[r:r + 1], lat[r:r + 1], 1 + r % 15)[0]) for r in range(64)]
    for lane in range(64):
        bad = list(wave)
        c = bad[lane]
        res = (c >> 52) & 15
        bad[lane] = c | (7 << (3 * (15 - max(1, res // 2))))  # digit res / 2 (>= 1) set to 7
        with pytest.raises(MosaicError):
            h3.grid_cellcenter(bad)
    cen = h3.grid_cellcenter(wave)
    for i, c in enumerate(wave):
        lat, lon = oracle.h3_to_geo(c)
        assert (cen[i, 0], cen[i, 1]) == (deg(lon), deg(lat))
    h3.close()
