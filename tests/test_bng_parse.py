"""BNG string cell ids back to long ids (§8(a) row a9: BNG chips carry StringType index_id by
default, BNGIndexSystem.scala:28; the join needs the long id).

Reference: BNGIndexSystem.parse (core/index/BNGIndexSystem.scala:391-413) + encode (:528-541),
letterMap :84-99 (row 10 repeats "SZ"; find() takes row 0).  The oracle's parse (oracle/bng.c) is
pinned by the reference's 12 golden (string, id) pairs (TestBNGIndexSystem.scala:10-90, in
tests/golden/reference_vectors.json); the engine's restatement (bng_device.h, shared by the host
ABI mosaic_bng_parse and the GPU column kernel k_bng_parse) equals it on formatted ids of every
resolution and on strings the reference treats oddly (signs inside the bins, odd digit counts whose
halves overlap, quadrant-like suffixes of short ids, Int overflow, unknown letters)."""
import ctypes
import json
import os

import numpy as np
import pytest

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_vectors.json")))


def corpus(n=600, seed=3):
    rng = np.random.default_rng(seed)
    out = []
    for res in (-1, 1, -2, 2, -3, 3, -4, 4, -5, 5, -6, 6):
        for x, y in zip(rng.uniform(0, 700000, n), rng.uniform(0, 1300000, n)):
            c = oracle.bng_point_to_index(float(x), float(y), res)
            try:
                out.append(oracle.bng_format(int(c)))
            except ValueError:
                pass
    out += [r["fmt"] for r in GOLD["bng_point_to_index"]]
    odd = ["SW", "SE", "NW", "NE", "SZ", "SZ12", "HY", "T", "S", "N", "H", "J", "O", "X", "", "V", "tq", "TQ",
           "TQ1", "TQ123", "TQ12345", "TQ-1-1", "TQ+1+1", "TQ1-2", "TQ--", "TQ99999999999", "TQ2147483647",
           "TQ21474836472147483647", "TQ21474836482147483648", "TQ12SW", "TQ1SW", "TQSW", "TQ NE", "TQ12 3",
           "TQ3879SE", "TQ3879XX", "TQ38798SE", "SWSW", "SSW", "ZZ12", "TQ0000", "TQ00000000000000"]
    return out + odd


def test_oracle_parse_pinned_by_reference_goldens(oracle_lib):
    for r in GOLD["bng_point_to_index"]:
        assert oracle.bng_parse(r["fmt"]) == r["id"], r


def test_host_abi_parse_matches_oracle(oracle_lib):
    from mosaic_amd import _native as N

    lib = N.lib()
    bad = []
    for s in corpus():
        out = ctypes.c_int64(0)
        rc = lib.mosaic_bng_parse(s.encode(), ctypes.byref(out))
        want = oracle.bng_parse(s)
        got = out.value if rc == 0 else None
        if got != want:
            bad.append((s, got, want))
    assert not bad, bad[:10]


@pytest.mark.gpu
def test_gpu_parse_column_matches_oracle(oracle_lib):
    from mosaic_amd import BNGIndexSystem, MosaicContext, MosaicError

    ctx = MosaicContext.build("BNG", "JTS")
    try:
        strs = corpus(2000)
        good = [s for s in strs if oracle.bng_parse(s) is not None]
        want = np.array([oracle.bng_parse(s) for s in good], np.int64)
        assert np.array_equal(ctx.bng_parse_column(good), want)
        # null rows, int64 (large_utf8) offsets
        vals = [None if i % 7 == 3 else s for i, s in enumerate(good)]
        got = ctx.bng_parse_column(vals)
        exp = np.array([0 if v is None else oracle.bng_parse(v) for v in vals], np.int64)
        assert np.array_equal(got, exp)
        enc = [s.encode() for s in good]
        offs = np.zeros(len(enc) + 1, np.int64)
        np.cumsum([len(e) for e in enc], out=offs[1:])
        assert np.array_equal(ctx.bng_parse_column((offs, b"".join(enc))), want)
        # a row the reference cannot parse: an error naming it
        bad_rows = [s for s in strs if oracle.bng_parse(s) is None]
        assert bad_rows
        with pytest.raises(MosaicError, match="row 2"):
            ctx.bng_parse_column(good[:2] + [bad_rows[0]] + good[2:5])
    finally:
        ctx.close()


@pytest.mark.gpu
def test_bng_string_chip_ids_join(oracle_lib):
    """A BNG chip table whose index_id column holds the reference's default StringType ids joins
    exactly like the same table with long ids."""
    from mosaic_amd import MosaicContext
    from mosaic_amd.context import tessellate
    from mosaic_amd.data import PolygonSet, uniform_points

    ctx = MosaicContext.build("BNG", "JTS")
    try:
        zones = PolygonSet.load("london_postcodes_bng")
        chips = tessellate("BNG", zones, 3)
        strs = [oracle.bng_format(int(c)) for c in chips["index_id"]]
        t_long = ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 3,
                                n_polygons=len(zones))
        t_str = ctx.chip_table(chips["is_core"], strs, chips["wkb"], chips["polygon_key"], 3, n_polygons=len(zones))
        offs, data = chips["wkb"]
        t_o32 = ctx.chip_table(chips["is_core"], strs, (offs.astype(np.int32), data), chips["polygon_key"], 3,
                               n_polygons=len(zones))
        x, y = uniform_points(zones.bbox(), 300_000, seed=5)
        want = ctx.pip_join_count(t_long, x, y)
        assert want.sum() > 1000
        assert np.array_equal(ctx.pip_join_count(t_str, x, y), want)
        assert np.array_equal(ctx.pip_join_count(t_o32, x, y), want)
        for t in (t_long, t_str, t_o32):
            t.close()
    finally:
        ctx.close()
