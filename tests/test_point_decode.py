"""CPU-only: the device point decoder (mosaic_amd/csrc/point_decode.h, compiled for the host)
against the oracle restatement (oracle/point_decode.py) on the corpus of tests/helpers.point_rows:
identical decode / row-path split, and bit-identical x / y (correct rounding of decimal strings
like Double.parseDouble, WKB byte orders and EWKB / ISO dimension flags, hex WKB)."""
import os
import struct
import subprocess

import numpy as np

from oracle import point_decode as PD
from tests.helpers import point_rows

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bits(v):
    return struct.unpack("<Q", struct.pack("<d", v))[0]


def test_oracle_on_reference_fixtures():
    # test/package.scala:70, 91: the reference's WKT point mocks; Python float == parseDouble
    assert PD.wkt_point("POINT (-75.78033 35.18937)") == ("ok", -75.78033, 35.18937)
    assert PD.wkt_point("POINT (75780 35189)") == ("ok", 75780.0, 35189.0)
    assert PD.wkt_point("POLYGON EMPTY")[0] == "rowpath"  # PointIndexBehaviors.scala:133-135 throws
    assert PD.hex_point("0101000000000000000000F03F0000000000000040") == ("ok", 1.0, 2.0)


def test_device_decoder_on_host_matches_oracle(tmp_path):
    exe = tmp_path / "decsc"
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), os.path.join(ROOT, "tests", "native", "decode_selfcheck.cpp")],
                   check=True)
    rows = point_rows(np.random.default_rng(31))
    n_ok = 0
    for fmt in (0, 1, 2):
        sel = [r for f, r in rows if f == fmt]
        out = subprocess.run([str(exe), str(fmt)], input="".join(r.hex() + "\n" for r in sel), check=True,
                             capture_output=True, text=True).stdout.splitlines()
        assert len(out) == len(sel)
        for r, line in zip(sel, out):
            st, bx, by = line.split()
            want = PD.decode(fmt, r)
            if want[0] == "ok":
                assert st == "0", (fmt, r, line)
                assert (int(bx, 16), int(by, 16)) == (_bits(want[1]), _bits(want[2])), (fmt, r, line, want)
                n_ok += 1
            else:
                assert st != "0", (fmt, r, line, want)
    assert n_ok > 2500
