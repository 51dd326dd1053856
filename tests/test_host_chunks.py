"""Host-resident coordinates (the boundary's Arrow-buffer case): mosaic_pip_join_count joins them in
chunks whose PCIe copies overlap the previous chunk's join (context option host_chunk).  The
chunked path must give the same counts as staging the whole batch (host_chunk = 0) and as the
oracle, keep the reference's NaN error for BNG wherever the NaN row falls, and report its stats."""
import numpy as np
import pytest

import oracle
from mosaic_amd import IllegalStateException, MosaicContext
from mosaic_amd.context import tessellate
from mosaic_amd.data import PolygonSet, uniform_points

pytestmark = pytest.mark.gpu


def test_chunked_counts_match_whole_batch_and_oracle():
    zones = PolygonSet.load("nyc_taxi_zones")
    chips = tessellate("H3", zones, 9)
    ctx = MosaicContext.build("H3")
    table = ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 9,
                           n_polygons=len(zones))
    x, y = uniform_points(zones.bbox(), 1_000_003, config=2, seed=77)
    ctx.set_option("host_chunk", 0)
    whole = ctx.pip_join_count(table, x, y).copy()
    offs, data = chips["wkb"]
    oc = dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
              wkb_offsets=offs, wkb=data)
    want, _ = oracle.pip_join(oc, oracle.GRID_H3, 9, x, y, len(zones), threads=8)
    assert np.array_equal(whole, want)
    for chunk in (1 << 17, 333_333, 999_999):
        ctx.set_option("host_chunk", chunk)
        got = ctx.pip_join_count(table, x, y)
        assert np.array_equal(got, want), chunk
        assert ctx.last_stats()["contains_tests"] >= 0
    ctx.set_option("host_chunk", 1 << 25)
    ctx.close()


def test_chunked_bng_nan_in_a_later_chunk_raises():
    ctx = MosaicContext.build("BNG")
    x0, y0 = 530000.0, 180000.0
    sq = [[[(x0, y0), (x0 + 900, y0), (x0 + 900, y0 + 900), (x0, y0 + 900), (x0, y0)]]]
    zones = PolygonSet(np.array(sq[0][0]), [0, 5], [0, 1], [0, 1])
    chips = tessellate("BNG", zones, 3)
    table = ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 3, n_polygons=1)
    rng = np.random.default_rng(3)
    x = x0 + rng.random(500_000) * 1000
    y = y0 + rng.random(500_000) * 1000
    ctx.set_option("host_chunk", 100_000)
    good = ctx.pip_join_count(table, x, y).copy()
    ctx.set_option("host_chunk", 0)
    assert np.array_equal(ctx.pip_join_count(table, x, y), good)
    x[400_123] = np.nan
    ctx.set_option("host_chunk", 100_000)
    with pytest.raises(IllegalStateException, match="NaN coordinates are not supported."):
        ctx.pip_join_count(table, x, y)
    ctx.close()
