"""GPU: H3's exact path (h3_exact + the glibc 2.35 restatement glibc_math.h) against the oracle.

The oracle is H3 C v3.7 compiled by gcc against this host's glibc -- the libm the reference's H3
JNI library reaches -- so every comparison here is bit for bit, with no tolerance and no excluded
rows: the device's sincos / tan / acos / atan2 on ~10^7 arguments, and cells from the exact path
alone (mosaic_point_to_cell_exact, no fast-path certification) on uniform points and on points
within an ulp of the reference's own cell boundaries at coarse to fine resolutions."""
import numpy as np
import pytest

import oracle
from mosaic_amd import MosaicContext
from mosaic_amd import _native as N

from .helpers import h3_cell_boundary_points

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = MosaicContext.build("H3", "JTS")
    yield c
    c.close()


def _device_libm(ctx, fn, a, b=None):
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(a if b is None else b, np.float64)
    out = np.empty_like(a)
    N.check(N.lib().mosaic_diag_libm(ctx.handle, fn, N.ptr(a), N.ptr(b), len(a), N.ptr(out)))
    return out


def _same_bits(got, want):
    return (got.view(np.int64) == want.view(np.int64)) | (np.isnan(got) & np.isnan(want))


def _args(rng, fn, n):
    sgn = np.where(rng.random(n) < 0.5, -1.0, 1.0)
    logu = lambda lo, hi: np.exp(rng.uniform(np.log(lo), np.log(hi), n))  # noqa: E731
    rbits = rng.integers(0, 2**63, n, dtype=np.int64).view(np.float64) * sgn
    rbits[~np.isfinite(rbits)] = 1.0
    if fn in (0, 1):
        parts = [rng.uniform(-np.pi, np.pi, n), rng.uniform(-10, 10, n), sgn * logu(1e-12, 1e9), sgn * logu(1e8, 1e300),
                 np.round(rng.uniform(-100, 100, n)) * (np.pi / 2) + rng.uniform(-1e-6, 1e-6, n), rbits]
    elif fn == 2:
        parts = [rng.uniform(0, 0.6525, n), sgn * logu(1e-12, 0.787)]
    elif fn == 3:
        parts = [1 - rng.uniform(0, 0.2054, n), rng.uniform(-1, 1, n), sgn * (1 - logu(1e-17, 0.04)), sgn * logu(1e-20, 0.5)]
    else:
        parts = [rng.uniform(-1, 1, n), sgn * logu(1e-300, 1e300), sgn * rng.uniform(0, 0.07, n), rbits]
    return np.concatenate(parts)


@pytest.mark.parametrize("fn,name", [(0, "sin"), (1, "cos"), (2, "tan"), (3, "acos"), (4, "atan2")])
def test_glibc_math_device(ctx, fn, name):
    rng = np.random.default_rng(70 + fn)
    a = _args(rng, fn, 400_000)
    b = None
    if fn == 4:
        b = _args(np.random.default_rng(90), fn, 400_000)
        sp = np.array([0.0, -0.0, np.inf, -np.inf, 1.0, -1.0, 1e-310, -1e-310, np.nan])
        a = np.concatenate([a, np.repeat(sp, len(sp))])
        b = np.concatenate([b, np.tile(sp, len(sp))])
    got = _device_libm(ctx, fn, a, b)
    want = oracle.libm_eval(fn, a, b)
    ok = _same_bits(got, want)
    bad = np.nonzero(~ok)[0]
    assert len(bad) == 0, (name, len(bad), [(a[i], None if b is None else b[i], got[i], want[i]) for i in bad[:5]])


def _exact_cells(ctx, lon, lat, res):
    lon = np.ascontiguousarray(lon, np.float64)
    lat = np.ascontiguousarray(lat, np.float64)
    out = np.empty(len(lon), np.int64)
    N.check(N.lib().mosaic_point_to_cell_exact(ctx.handle, res, N.ptr(lon), N.ptr(lat), len(lon), N.ptr(out)))
    return out


@pytest.mark.parametrize("res", list(range(16)))
def test_exact_path_every_row_global(ctx, res):
    rng = np.random.default_rng(300 + res)
    lon = rng.uniform(-180, 180, 300_000)
    lat = np.degrees(np.arcsin(rng.uniform(-1, 1, 300_000)))
    got = _exact_cells(ctx, lon, lat, res)
    want = oracle.h3_point_to_index(lon, lat, res)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, [(lon[i], lat[i], hex(got[i]), hex(want[i])) for i in bad[:5]]


@pytest.mark.parametrize("res", [0, 2, 5, 9, 10, 11, 13, 15])
def test_exact_path_on_cell_boundaries(ctx, res):
    """Points within an ulp of the reference's cell boundaries (global, and in the NYC bbox the
    bench uses): the exact path and the full path (fast + exact) both equal the oracle."""
    rng = np.random.default_rng(500 + res)
    gx, gy = h3_cell_boundary_points(rng, 20_000, res)
    nx, ny = h3_cell_boundary_points(rng, 20_000, res, (-74.26, -73.70), (40.49, 40.92))
    lon, lat = np.concatenate([gx, nx]), np.concatenate([gy, ny])
    assert len(lon) > 20_000
    want = oracle.h3_point_to_index(lon, lat, res)
    for path in ("exact", "full"):
        if path == "exact":
            got = _exact_cells(ctx, lon, lat, res)
        else:
            got = ctx.grid_longlatascellid(lon, lat, res, raw=True)
        bad = np.nonzero(got != want)[0]
        assert len(bad) == 0, (path, [(lon[i], lat[i], hex(got[i]), hex(want[i])) for i in bad[:5]])
    # the boundary points do reach the exact path
    assert ctx.last_stats()["exact_path_rows"] > 0
