"""serializeCellId for BNG on the GPU (§8(a) row a8: BNG ids default to StringType).

Reference: IndexSystem.serializeCellId (core/index/IndexSystem.scala:37-46) ->
BNGIndexSystem.format (core/index/BNGIndexSystem.scala:114-129; letterMap :84-99 with its row-10
"SZ" quirk).  The oracle's format (oracle/bng.c) is pinned by the reference's 12 golden strings
(tests/test_oracle.py); here the GPU formatter's code compiled for the host equals it on 60,010
ids (tests/native/bng_format_selfcheck.cpp), and the GPU column (mosaic_bng_format_column, Arrow
utf8 layout) equals it on ids of every resolution, with null rows and an unformattable id."""
import os
import subprocess

import numpy as np
import pytest

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_device_formatter_on_host_matches_oracle(oracle_lib, tmp_path):
    exe = tmp_path / "fmt"
    lib = os.path.join(ROOT, "oracle", "liboracle.so")
    subprocess.run(["g++", "-O1", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(ROOT, "mosaic_amd", "csrc"),
                    "-o", str(exe), os.path.join(ROOT, "tests", "native", "bng_format_selfcheck.cpp"), lib,
                    f"-Wl,-rpath,{os.path.dirname(lib)}"], check=True)
    tot, bad = map(int, subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split())
    assert tot == 60010 and bad == 0


def _ids(n, seed=9):
    rng = np.random.default_rng(seed)
    out = []
    for res in (-1, 1, -2, 2, -3, 3, -4, 4, -5, 5, -6, 6):
        for x, y in zip(rng.uniform(-10000, 710000, n), rng.uniform(-10000, 1310000, n)):
            c = oracle.bng_point_to_index(float(x), float(y), res)
            try:  # ids of points far outside the grid have letter digits the reference cannot format
                oracle.bng_format(int(c))
            except ValueError:
                continue
            out.append(c)
    return np.array(out, np.int64)


@pytest.mark.gpu
def test_gpu_format_column_matches_oracle():
    from mosaic_amd import MosaicContext, MosaicError

    ctx = MosaicContext.build("BNG")
    ids = _ids(2000)
    assert len(ids) > 20000
    valid = np.ones(len(ids), np.uint8)
    valid[::97] = 0
    offs, chars = ctx.bng_format_column(ids, valid)
    assert offs[0] == 0 and len(chars) == offs[-1]
    for i, c in enumerate(ids):
        s = chars[offs[i]:offs[i + 1]].decode()
        assert s == ("" if not valid[i] else oracle.bng_format(int(c))), i
    # the reference's own ids (TestBNGIndexSystem.scala:29-34, 60-65)
    assert ctx.grid_longlatascellid(np.array([538825.0]), np.array([179111.0]), 4) == ["TQ388791"]
    with pytest.raises(MosaicError):
        ctx.bng_format_column(np.array([1050138790, 123], np.int64))
    ctx.close()
