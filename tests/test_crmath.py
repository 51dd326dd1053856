"""CPU-only: crmath.h (the GPU exact path's sin / cos / tan / acos / atan2) is correctly rounded,
checked against mpmath at 250 bits; its disagreement with glibc is glibc's own rounding error."""
import ctypes
import math
import os
import subprocess

import numpy as np
import pytest

mpmath = pytest.importorskip("mpmath")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def crm(tmp_path_factory):
    so = tmp_path_factory.mktemp("crm") / "libcrm.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-shared", "-fPIC", "-o", str(so),
                    os.path.join(ROOT, "tests", "native", "crmath_host.cpp")], check=True)
    lib = ctypes.CDLL(str(so))

    def ev(fn, a, b=None):
        a = np.ascontiguousarray(a, np.float64)
        b = np.ascontiguousarray(a if b is None else b, np.float64)
        out = np.empty_like(a)
        vp = ctypes.c_void_p
        lib.crm_eval(ctypes.c_int(fn), vp(a.ctypes.data), vp(b.ctypes.data), ctypes.c_long(len(a)), vp(out.ctypes.data))
        return out

    return ev


CASES = [(0, "sin", mpmath.sin, (-7, 7)), (1, "cos", mpmath.cos, (-7, 7)), (2, "tan", mpmath.tan, (0, 1.2)),
         (3, "acos", mpmath.acos, (-1, 1)), (4, "atan2", mpmath.atan2, (-1, 1))]


@pytest.mark.parametrize("fn,name,ref,rng_", CASES, ids=[c[1] for c in CASES])
def test_correctly_rounded(crm, fn, name, ref, rng_):
    mpmath.mp.prec = 250
    rng = np.random.default_rng(fn)
    n = 4000
    a = rng.uniform(*rng_, n)
    if name == "acos":
        a[: n // 2] = 1 - rng.uniform(0, 0.3, n // 2) ** 2  # H3's acos(1 - sqd/2) range
    b = rng.uniform(-1, 1, n) if name == "atan2" else None
    got = crm(fn, a, b)
    for i in range(n):
        args = (a[i],) if b is None else (a[i], b[i])
        want = float(ref(*[mpmath.mpf(float(v)) for v in args]))
        assert got[i] == want, (name, args)


def test_glibc_is_within_one_ulp(crm):
    rng = np.random.default_rng(9)
    a = rng.uniform(-7, 7, 20000)
    got = crm(0, a)
    ref = np.array([math.sin(v) for v in a])
    diff = np.abs(got - ref) / np.spacing(np.abs(ref))
    assert diff.max() <= 1.0
    assert (got != ref).mean() < 0.01
