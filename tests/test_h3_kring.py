"""grid_cellkring / grid_cellkloop over H3 cells (reference H3IndexSystem.kRing / kLoop =
h3-java kRing / hexRing, core/index/H3IndexSystem.scala:154-177; kernel mosaic_amd/csrc/
h3_neighbors.h, H3 v3.7's h3NeighborRotations / hexRangeDistances / hexRing / _kRingInternal).

The oracle (oracle/h3.c oracle_h3_kring_set) finds the k-ring on the sphere -- a cell's neighbours
are the cells geoToH3 gives just beyond the midpoints of its boundary edges (h3ToGeoBoundary),
closed breadth-first -- so it checks the kernel's walk independently of H3's neighbour tables:
same set, same ring distance per cell (hexRange emits ring by ring), kLoop = the ring-k cells.
Order pin: the reference's documented kring of 613177664827555839 starts [613177664827555839,
613177664825458687, ...] (docs/source/api/spatial-indexing.rst:648-653).  Near the 12 pentagons
H3 falls back to _kRingInternal (kRing: its hash table in slot order, as h3-java returns it) and
the reference's kLoop to kRing(k).toSet diff kRing(k - 1).toSet (Scala HashSet order): sets are
checked against the oracle and against shared-edge adjacency of the cells' boundaries; those
orders follow H3's / Scala's published algorithms and no reference fixture pins them ("order
unpinned")."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOC_CELL, DOC_SECOND = 613177664827555839, 613177664825458687


@pytest.fixture(scope="module")
def host_lib(tmp_path_factory):
    so = tmp_path_factory.mktemp("h3k") / "libh3k.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-Wno-unknown-pragmas", "-shared", "-fPIC",
                    "-I", os.path.join(ROOT, "mosaic_amd", "csrc"), "-o", str(so),
                    os.path.join(ROOT, "tests", "native", "h3_kring_host.cpp")], check=True)
    lib = ctypes.CDLL(str(so))
    lib.h3_kring_host.restype = ctypes.c_int
    lib.h3_kring_host.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    lib.h3_neighbor_host.restype = ctypes.c_int64
    lib.h3_neighbor_host.argtypes = [ctypes.c_int64, ctypes.c_int]
    return lib


@pytest.fixture(scope="module")
def host_kring(host_lib):
    def run(cell, k, loop, want_slow=False):
        out = np.zeros(max(1 + 3 * k * (k + 1), 1), np.int64)
        slow = ctypes.c_int(0)
        n = host_lib.h3_kring_host(int(cell), k, loop, out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(slow))
        r = None if n < 0 else out[:n].tolist()
        return (r, bool(slow.value)) if want_slow else r
    return run


def random_cells(n, seed, res_list):
    rng = np.random.default_rng(seed)
    lat = np.degrees(np.arcsin(rng.uniform(-1, 1, n)))
    lon = rng.uniform(-180, 180, n)
    res = rng.choice(res_list, n)
    return [int(oracle.h3_point_to_index(lon[i:i + 1], lat[i:i + 1], int(res[i]))[0]) for i in range(n)]


PENTAGON_BASE_CELLS = (4, 14, 24, 38, 49, 58, 63, 72, 83, 97, 107, 117)


def pentagon_cell(bc, res):
    h = (1 << 59) | (res << 52) | (bc << 45)
    for r in range(res + 1, 16):
        h |= 7 << (3 * (15 - r))
    return h


def check(run, cell, k):
    """the row against the oracle; True when H3's fast walk served it (False: its fallback)"""
    (ring, slow) = run(cell, k, 0, want_slow=True)
    want = oracle.h3_kring_set(cell, k)
    assert ring is not None
    assert len(ring) == len(set(ring)) and set(ring) == set(want), (cell, k)
    loop = run(cell, k, 1)
    assert loop is not None and set(loop) == {c for c, d in want.items() if d == k}, (cell, k)
    if slow:
        return False
    assert len(ring) == 1 + 3 * k * (k + 1)
    # hexRange emits ring by ring
    assert [want[c] for c in ring] == sorted(want[c] for c in ring)
    assert len(loop) == (6 * k if k else 1)
    if k:  # hexRing starts at the ring's start cell, which hexRange emits last in that ring
        seg = ring[1 + 3 * (k - 1) * k:]
        assert loop == [seg[-1]] + seg[:-1]
    return True


def test_documented_kring_order(host_kring):
    ring = host_kring(DOC_CELL, 2, 0)
    assert ring[:2] == [DOC_CELL, DOC_SECOND] and len(ring) == 19
    assert check(host_kring, DOC_CELL, 2)


def test_nyc_cells_all_resolutions(host_kring):
    rng = np.random.default_rng(11)
    for res in range(1, 16):
        lon = rng.uniform(-74.25, -73.70, 12)
        lat = rng.uniform(40.50, 40.91, 12)
        for c in oracle.h3_point_to_index(lon, lat, res).tolist():
            for k in (0, 1, 2, 3):
                check(host_kring, c, k)


def test_global_cells(host_kring):
    cells = random_cells(400, 5, list(range(1, 16)))
    fast = sum(check(host_kring, c, (0, 1, 2, 4)[i % 4]) for i, c in enumerate(cells))
    assert fast > 300


def test_pentagon_neighbourhoods(host_kring, host_lib):
    """Every cell within two rings of each of the 12 pentagons (res 1-10): kRing / kLoop sets equal
    the oracle's (H3's fallback runs), and every h3NeighborRotations step lands on a cell sharing
    a boundary edge with its origin (the base-cell neighbour tables, tools/h3gen_neighbors.py)."""
    import math

    def unit(lat, lng):
        return np.array([math.cos(lat) * math.cos(lng), math.cos(lat) * math.sin(lng), math.sin(lat)])

    def edge_neighbours(c, pool):
        vc = [unit(*v) for v in oracle.h3_to_geo_boundary(c)]
        tol = 1e-3 * 0.378 ** ((c >> 52) & 15)
        out = set()
        for d in pool:
            if d == c:
                continue
            vd = [unit(*v) for v in oracle.h3_to_geo_boundary(d)]
            if sum(any(np.linalg.norm(p - q) < tol for q in vd) for p in vc) >= 2:
                out.add(d)
        return out

    slow = 0
    for bc in PENTAGON_BASE_CELLS:
        for res in (1, 2, 3, 6, 8, 10):
            p = pentagon_cell(bc, res)
            around = sorted(oracle.h3_kring_set(p, 2))
            pool = set(oracle.h3_kring_set(p, 3))
            for c in around:
                for k in (1, 2, 3):
                    slow += not check(host_kring, c, k)
                if res <= 3:
                    nbs = {host_lib.h3_neighbor_host(c, d) for d in range(1, 7)} - {0}
                    assert nbs == edge_neighbours(c, pool), (bc, res, c)
    assert slow > 500


K_BIG = 100


def test_pentagon_large_k(host_kring):
    """k = 100 around all 12 pentagons (the k > 60 limit lifted): H3's _kRingInternal
    search with its depth-first stack in scratch; kRing / kLoop sets equal the oracle's sphere
    search (1 + 5 k (k + 1) / 2 cells around a pentagon)."""
    for i, bc in enumerate(PENTAGON_BASE_CELLS):
        p = pentagon_cell(bc, 7 + i % 4)
        ring, slow = host_kring(p, K_BIG, 0, want_slow=True)
        want = oracle.h3_kring_set(p, K_BIG)
        assert slow and len(ring) == len(set(ring)) == 1 + 5 * K_BIG * (K_BIG + 1) // 2
        assert set(ring) == set(want), bc
        loop = host_kring(p, K_BIG, 1)
        assert set(loop) == {c for c, d in want.items() if d == K_BIG} and len(loop) == 5 * K_BIG


def test_pentagon_cell_itself(host_kring):
    # a pentagon's ring: 5 neighbours (H3's fallback table of 7 slots, 6 filled)
    for bc in PENTAGON_BASE_CELLS:
        for res in (0, 1, 5, 9):
            p = pentagon_cell(bc, res)
            ring, slow = host_kring(p, 1, 0, want_slow=True)
            assert slow and len(ring) == 6 and set(ring) == set(oracle.h3_kring_set(p, 1))
            assert host_kring(p, 0, 1) == [p]
            assert set(host_kring(p, 1, 1)) == set(ring) - {p}


def test_invalid_cells(host_kring):
    assert host_kring(0, 1, 0) is None
    bad_pent = pentagon_cell(4, 2) & ~(7 << (3 * 14)) | (1 << (3 * 14))  # leading k digit
    assert host_kring(bad_pent, 1, 0) is None


@pytest.mark.gpu
def test_gpu_kring_pentagons_large_k(host_kring):
    """k = 100 around all 12 pentagons on the GPU (k_h3_kring_slow, one row per wave, stack in
    scratch): element for element the host build, sets equal the oracle's."""
    from mosaic_amd import MosaicContext

    h3 = MosaicContext.build("H3", "JTS")
    pents = [pentagon_cell(bc, 7 + i % 4) for i, bc in enumerate(PENTAGON_BASE_CELLS)]
    for loop in (0, 1):
        got = (h3.grid_cellkloop if loop else h3.grid_cellkring)(pents, K_BIG)
        for p, g in zip(pents, got):
            assert g.tolist() == host_kring(p, K_BIG, loop), (p, loop)
    for p, g in zip(pents[:3], h3.grid_cellkring(pents[:3], K_BIG)):
        assert set(g.tolist()) == set(oracle.h3_kring_set(p, K_BIG))
    h3.close()


def _digest(cells):
    m = (1 << 64) - 1
    cells = [int(c) & m for c in cells]
    s = x = q = 0
    for c in cells:
        s, x, q = (s + c) & m, x ^ c, (q + c * c) & m
    return dict(n=len(cells), sum=s, xor=x, sumsq=q)


@pytest.mark.gpu
def test_gpu_kring_pentagons_k200(host_kring):
    """k = 200 around all 12 pentagons -- past the device search's k <= 128, answered
    by the same H3 _kRingInternal code on host threads inside mosaic_cell_kring (no -4 / row path any
    more): kRing and kLoop sets equal the oracle's sphere search (order-free digests committed by
    tests/golden/make_kring_k200.py), in a batch with a row H3's fast walk serves; the element order
    equals the host build of the device code on two pentagons."""
    import json
    import os

    from mosaic_amd import MosaicContext

    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kring_k200_pentagons.json")))
    k = fx["k"]
    h3 = MosaicContext.build("H3", "JTS")
    cells = [DOC_CELL] + [r["cell"] for r in fx["rows"]]
    for loop, name in ((0, "ring"), (1, "loop")):
        got = (h3.grid_cellkloop if loop else h3.grid_cellkring)(cells, k)
        assert len(got[0]) == (6 * k if loop else 1 + 3 * k * (k + 1))  # the hexagon row: H3's walk
        for r, g in zip(fx["rows"], got[1:]):
            assert len(set(g.tolist())) == len(g)
            assert _digest(g.tolist()) == r[name], (hex(r["cell"]), name)
        for r, g in zip(fx["rows"][:2], got[1:3]):
            assert g.tolist() == host_kring(r["cell"], k, loop)
    h3.close()


@pytest.mark.gpu
def test_gpu_kring_equals_host_and_oracle(host_kring):
    """mosaic_cell_kring (H3) on the GPU through the MosaicContext mirror: element for element the
    host build's order (fast walk and pentagon fallback alike), the oracle's sets; invalid ids
    raise."""
    from mosaic_amd import MosaicContext, MosaicError

    h3 = MosaicContext.build("H3", "JTS")
    rng = np.random.default_rng(17)
    cells = []
    for res in range(1, 16):
        lon = rng.uniform(-74.25, -73.70, 40)
        lat = rng.uniform(40.50, 40.91, 40)
        cells += oracle.h3_point_to_index(lon, lat, res).tolist()
    cells += random_cells(300, 23, list(range(1, 16)))
    for bc in PENTAGON_BASE_CELLS:  # pentagon neighbourhoods: H3's fallback
        for res in (1, 3, 7):
            cells += sorted(oracle.h3_kring_set(pentagon_cell(bc, res), 2))
    for k in (0, 1, 2, 5):
        for loop in (0, 1):
            got = (h3.grid_cellkloop if loop else h3.grid_cellkring)(cells, k)
            for c, g in zip(cells, got):
                assert g.tolist() == host_kring(c, k, loop), (c, k, loop)
        for c in cells[::37]:
            assert set(h3.grid_cellkring([c], k)[0].tolist()) == set(oracle.h3_kring_set(c, k))
    ring = h3.grid_cellkring([DOC_CELL], 2)[0].tolist()
    assert ring[:2] == [DOC_CELL, DOC_SECOND]
    with pytest.raises(MosaicError, match="not a valid"):
        h3.grid_cellkring([DOC_CELL, 0], 2)
    h3.close()


def test_base_cell_tables_round_trip():
    """geoToH3(h3ToGeo(h)) == h for every cell of resolutions 0-3 under all 122 base cells (the
    pentagons' deleted k sub-sequence skipped): checks the faceIjkBaseCells rotations the ring walk
    and the oracle share (tools/h3gen.py), the ten cw-offset pentagons included."""
    import math
    cells = []
    for bc in range(122):
        pent = bc in PENTAGON_BASE_CELLS
        for res in range(4):
            for digits in np.ndindex(*([7] * res)):
                lead = next((d for d in digits if d), 0)
                if pent and lead == 1:
                    continue
                h = (1 << 59) | (res << 52) | (bc << 45)
                for r in range(1, 16):
                    h |= (digits[r - 1] if r <= res else 7) << (3 * (15 - r))
                cells.append(h)
    lat, lon = zip(*(oracle.h3_to_geo(c) for c in cells))
    res = np.array([(c >> 52) & 15 for c in cells])
    lon_d = np.degrees(np.array(lon))
    lat_d = np.degrees(np.array(lat))
    bad = []
    for r in range(4):
        m = res == r
        got = oracle.h3_point_to_index(lon_d[m], lat_d[m], r)
        want = np.array(cells)[m]
        bad += [int(c) for c in want[got != want]]
    assert len(cells) > 40_000 and bad == []
