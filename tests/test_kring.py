"""grid_cellkring / grid_cellkloop over BNG cells (§8(f) row 4, the grid rings of KNN).

Reference: BNGIndexSystem.kRing / kLoop / isValid (core/index/BNGIndexSystem.scala:216-263),
reached from CellKRing / CellKLoop.nullSafeEval (expressions/index/CellKRing.scala:66-70).
The oracle (oracle/bng.c) is pinned by the reference's golden vectors
(TestBNGIndexSystem.scala:92-161: k-loops 1..3 around "TQ3879SE" (res -4) and "TQ3879" (res 3),
k-rings = the cell and its loops, isValid); the GPU path (mosaic_cell_kring through the C ABI,
marked gpu) must equal the oracle element for element, order included.  H3 k-rings:
tests/test_h3_kring.py."""
import numpy as np
import pytest

import oracle

NEG = 1050138794  # "TQ3879SE", res -4
POS = 1050138790  # "TQ3879", res 3
GOLD_NEG = {
    1: ["TQ3878NW", "TQ3878NE", "TQ3978NW", "TQ3979SW", "TQ3979NW", "TQ3879NE", "TQ3879NW", "TQ3879SW"],
    2: ["TQ3778SE", "TQ3878SW", "TQ3878SE", "TQ3978SW", "TQ3978SE", "TQ3978NE", "TQ3979SE", "TQ3979NE",
        "TQ3980SE", "TQ3980SW", "TQ3880SE", "TQ3880SW", "TQ3780SE", "TQ3779NE", "TQ3779SE", "TQ3778NE"],
    3: ["TQ3777NW", "TQ3777NE", "TQ3877NW", "TQ3877NE", "TQ3977NW", "TQ3977NE", "TQ4077NW", "TQ4078SW",
        "TQ4078NW", "TQ4079SW", "TQ4079NW", "TQ4080SW", "TQ4080NW", "TQ3980NE", "TQ3980NW", "TQ3880NE",
        "TQ3880NW", "TQ3780NE", "TQ3780NW", "TQ3780SW", "TQ3779NW", "TQ3779SW", "TQ3778NW", "TQ3778SW"],
}
GOLD_POS = {
    1: ["TQ3778", "TQ3779", "TQ3780", "TQ3878", "TQ3880", "TQ3978", "TQ3979", "TQ3980"],
    2: ["TQ3677", "TQ3777", "TQ3877", "TQ3977", "TQ4077", "TQ4078", "TQ4079", "TQ4080", "TQ4081", "TQ3981",
        "TQ3881", "TQ3781", "TQ3681", "TQ3680", "TQ3679", "TQ3678"],
    3: ["TQ3576", "TQ3676", "TQ3776", "TQ3876", "TQ3976", "TQ4076", "TQ4176", "TQ4177", "TQ4178", "TQ4179",
        "TQ4180", "TQ4181", "TQ4182", "TQ4082", "TQ3982", "TQ3882", "TQ3782", "TQ3682", "TQ3582", "TQ3581",
        "TQ3580", "TQ3579", "TQ3578", "TQ3577"],
}


def _fmt(cells):
    return [oracle.bng_format(int(c)) for c in cells]


@pytest.mark.parametrize("cell,gold", [(NEG, GOLD_NEG), (POS, GOLD_POS)])
def test_oracle_kloop_matches_reference_goldens(oracle_lib, cell, gold):
    for k, want in gold.items():
        assert sorted(_fmt(oracle.bng_kloop(cell, k))) == sorted(want)


def test_oracle_kring_is_cell_plus_loops(oracle_lib):
    for k in (1, 2, 3):
        want = [oracle.bng_format(POS)] + [s for j in range(1, k + 1) for s in GOLD_POS[j]]
        assert sorted(_fmt(oracle.bng_kring(POS, k))) == sorted(want)


def test_oracle_is_valid_reference_cases(oracle_lib):
    # TestBNGIndexSystem.scala:156-161
    assert not oracle.bng_is_valid(oracle.bng_point_to_index(-50000.0, 50.0, 3))
    assert not oracle.bng_is_valid(oracle.bng_point_to_index(50.0, 500000000.0, 4))
    assert oracle.bng_is_valid(POS) and oracle.bng_is_valid(NEG)


def _cells(n, seed=5):
    """Cells at every resolution over (and just outside) the grid, incl. its edges (filtered)."""
    rng = np.random.default_rng(seed)
    out = []
    for res in (-1, 1, -2, 2, -3, 3, -4, 4, -5, 5, -6, 6):
        e = rng.uniform(-20000, 720000, n)
        nn = rng.uniform(-20000, 1320000, n)
        e[: n // 8] = rng.uniform(0, 3000, n // 8)  # along the west edge
        nn[n // 8: n // 4] = rng.uniform(1297000, 1300000, n // 4 - n // 8)  # along the north edge
        for x, y in zip(e, nn):
            c = oracle.bng_point_to_index(float(x), float(y), res)
            if oracle.bng_is_valid(c):
                out.append(int(c))
    return np.array(out, np.int64)


@pytest.mark.gpu
@pytest.mark.parametrize("loop", [0, 1])
def test_gpu_kring_matches_oracle(loop):
    from mosaic_amd import MosaicContext

    ctx = MosaicContext.build("BNG")
    cells = _cells(300)
    assert len(cells) > 1000
    for k in (0, 1, 2, 3, 7):
        got = ctx._kring(cells, k, bool(loop), raw=True)
        for c, g in zip(cells, got):
            want = oracle.bng_kloop(c, k) if loop else oracle.bng_kring(c, k)
            assert np.array_equal(g, want), (int(c), k)
    # the reference's goldens through the GPU, as strings
    for k, want in GOLD_POS.items():
        assert sorted(ctx.grid_cellkloop([POS], k)[0]) == sorted(want)
    for k, want in GOLD_NEG.items():
        assert sorted(ctx.grid_cellkloop(["TQ3879SE"], k)[0]) == sorted(want)
    # the explode variants: one row per (input row, cell), same cells in the same order
    idx, cells_out = ctx.grid_cellkringexplode([POS, NEG], 2)
    rings = ctx.grid_cellkring([POS, NEG], 2)
    assert list(idx) == [0] * len(rings[0]) + [1] * len(rings[1])
    assert list(cells_out) == rings[0] + rings[1]
    ctx.close()


def test_device_code_on_host_matches_oracle(oracle_lib, tmp_path):
    """bng_device.h's kring (the kernel's code) compiled for the host == the oracle, order included."""
    import os
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = tmp_path / "kr"
    lib = os.path.join(root, "oracle", "liboracle.so")
    subprocess.run(["g++", "-O1", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(root, "mosaic_amd", "csrc"),
                    "-o", str(exe), os.path.join(root, "tests", "native", "bng_kring_selfcheck.cpp"), lib,
                    f"-Wl,-rpath,{os.path.dirname(lib)}"], check=True)
    tot, bad = map(int, subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split())
    assert tot == 100000 and bad == 0
