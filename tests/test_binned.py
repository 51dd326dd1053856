"""GPU: the binned chip join (join_binned.hip) -- points sorted by tile before the chip loop, for
tile-directory tables without a usable point raster (the border-chip-heavy C4 shape, SURVEY.md
§7.3-4).  Checked against the oracle's pairs and counts (QuickstartNotebook.py:205-219 join +
filter) and against the unbinned tiled join on the same inputs: LDS counts (few polygons), the
per-wave count hash (many polygons), pairs (source rows carried through the sort), several sort
chunks (the exact-H3 queue drained per chunk), and points on / next to chip vertices and segments
(the exact-H3 path reading sorted records)."""
import numpy as np
import pytest

import oracle
from mosaic_amd.context import tessellate
from mosaic_amd.data import PolygonSet, synthetic_buildings
from tests.test_gpu_parity import _chip_boundary_points

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def h3ctx():
    from mosaic_amd import MosaicContext

    ctx = MosaicContext.build("H3", "JTS")
    yield ctx
    ctx.close()


def _oracle_chips(chips):
    offs, data = chips["wkb"]
    return dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
                wkb_offsets=offs, wkb=data)


def _set(ctx, **kw):
    for k, v in kw.items():
        ctx.set_option(k, v)


def test_binned_zones_pairs_counts_chunks(h3ctx):
    zones = PolygonSet.load("nyc_taxi_zones_35")
    chips = tessellate("H3", zones, 9)
    rng = np.random.default_rng(17)
    x0, y0, x1, y1 = zones.bbox()
    bx, by = _chip_boundary_points(chips, rng)
    # widened bbox: some points fall in kSkip tiles and outside the tile grid
    x = np.concatenate([rng.uniform(x0 - 0.05, x1 + 0.05, 600_000), bx])
    y = np.concatenate([rng.uniform(y0 - 0.05, y1 + 0.05, 600_000), by])
    perm = rng.permutation(len(x))
    x, y = x[perm], y[perm]
    oc = _oracle_chips(chips)
    _, total, orow, okey = oracle.pip_join(oc, oracle.GRID_H3, 9, x, y, len(zones), pairs=True)
    want_pairs = set(zip(orow.tolist(), okey.tolist()))
    want = np.bincount(okey, minlength=len(zones))
    assert total > 10_000
    tables = []
    try:
        for images in (1, 2):  # 1: no images (the table has a point raster); 2: per-tile LDS images
            _set(h3ctx, tile_images=images)
            table = h3ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 9,
                                     n_polygons=len(zones))
            tables.append(table)
            t = table.tiles()
            assert (t["image_records"] > 0) == (images == 2), t
            _set(h3ctx, point_raster=0)
            for bins, chunk in ((0, 1 << 28), (1, 1 << 28), (1, 100_003), (1, 1024)):
                _set(h3ctx, bin_points=bins, bin_chunk=chunk)
                counts = h3ctx.pip_join_count(table, x, y)
                kern = ("k_join_tiles" if images == 2 else "k_join_binned") if bins else "k_join_tiled"
                assert h3ctx.last_kernel() == kern
                assert np.array_equal(counts, want), (images, bins, chunk)
                assert h3ctx.last_stats()["exact_path_rows"] > 0  # the boundary points reach the exact pass
                rows, keys = h3ctx.pip_join_pairs(table, x, y)
                assert set(zip(rows.tolist(), keys.tolist())) == want_pairs, (images, bins, chunk)
                assert len(rows) == total
            _set(h3ctx, point_raster=1, bin_points=1, bin_chunk=1 << 28)
    finally:
        _set(h3ctx, point_raster=1, bin_points=1, bin_chunk=1 << 28, tile_images=1)
        for t in tables:
            t.close()


def test_binned_host_chunked_exact_queue_overflow(h3ctx):
    """Host-resident points through the binned join in async chunks (join_count_host_chunked): a
    chunk whose exact-H3 rows exceed the queue (option exact_cap, tiny here) must be rerun, not
    returned short; the chunks' exact rows must reach last_stats."""
    zones = PolygonSet.load("nyc_taxi_zones_35")
    chips = tessellate("H3", zones, 9)
    rng = np.random.default_rng(23)
    x0, y0, x1, y1 = zones.bbox()
    bx, by = _chip_boundary_points(chips, rng)
    x = np.concatenate([rng.uniform(x0, x1, 300_000), bx])
    y = np.concatenate([rng.uniform(y0, y1, 300_000), by])
    perm = rng.permutation(len(x))
    x, y = np.ascontiguousarray(x[perm]), np.ascontiguousarray(y[perm])
    want, _ = oracle.pip_join(_oracle_chips(chips), oracle.GRID_H3, 9, x, y, len(zones))
    _set(h3ctx, tile_images=2)
    table = h3ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 9,
                             n_polygons=len(zones))
    try:
        _set(h3ctx, point_raster=0, bin_points=1, bin_min_rows=0, host_chunk=100_000)
        got = h3ctx.pip_join_count(table, x, y)
        assert h3ctx.last_kernel() == "k_join_tiles"
        assert np.array_equal(got, want)
        assert h3ctx.last_stats()["exact_path_rows"] > 0
        for cap in (1, 3):
            _set(h3ctx, exact_cap=cap)
            assert np.array_equal(h3ctx.pip_join_count(table, x, y), want), cap
    finally:
        _set(h3ctx, point_raster=1, bin_points=1, bin_min_rows=1 << 18, host_chunk=1 << 25, tile_images=1,
             exact_cap=0)
        table.close()


def test_binned_many_polygons_wave_hash(h3ctx):
    """60k building footprints at res 11 (n_polygons above the LDS count array: the per-wave hash
    of (key, count)), device points near the buildings."""
    import torch

    from mosaic_amd.data import building_points_device

    nb = 60_000
    b = synthetic_buildings(nb, bbox=(-74.02, 40.70, -73.95, 40.77), n_centres=12, sigma=0.01)
    chips = h3ctx.grid_tessellateexplode(b, 11)
    table = h3ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 11,
                             n_polygons=nb)
    t = table.tiles()
    assert t["built"] == 1 and t["raster"] == 0 and t["image_records"] > 0.5 * t["records"], t  # (dense tiles past the LDS cap run the generic loop)
    xd, yd = building_points_device(b, 3_000_000, seed=5)
    try:
        got = {}
        for bins, images, kern in ((1, 1, "k_join_tiles"), (1, 0, "k_join_binned"), (0, 1, "k_join_tiled")):
            _set(h3ctx, bin_points=bins, tile_images=images)
            got[kern] = h3ctx.pip_join_count(table, xd, yd).cpu().numpy()
            assert h3ctx.last_kernel() == kern
        _set(h3ctx, tile_images=1)
        x, y = xd.cpu().numpy(), yd.cpu().numpy()
        want, total = oracle.pip_join(_oracle_chips(chips), oracle.GRID_H3, 11, x, y, nb, threads=16)
        assert total > 500_000
        for kern, g in got.items():
            assert np.array_equal(g, want), kern
        # pairs through the binned path (source rows from the sorted records)
        _set(h3ctx, bin_points=1)
        rows, keys = h3ctx.pip_join_pairs(table, xd, yd)
        rows = rows.cpu().numpy() if hasattr(rows, "cpu") else rows
        keys = keys.cpu().numpy() if hasattr(keys, "cpu") else keys
        assert np.array_equal(np.bincount(keys, minlength=nb), want)
        assert len(np.unique(rows.astype(np.int64) * nb + keys)) == len(rows)
    finally:
        _set(h3ctx, bin_points=1, tile_images=1)
        del xd, yd
        torch.cuda.empty_cache()
        table.close()



def test_binned_lookback_fallback(h3ctx):
    """k_bin_cover's compaction takes ordered tickets; its bounded wait's fallback (rerun in place,
    dropped rows keyed kSkip) is forced with bin_spin_cap < 0 and must give the same counts and pairs
    (every row then goes through the sort: last_binned_rows == n)."""
    zones = PolygonSet.load("nyc_taxi_zones_35")
    chips = tessellate("H3", zones, 9)
    rng = np.random.default_rng(31)
    x0, y0, x1, y1 = zones.bbox()
    x = rng.uniform(x0 - 0.05, x1 + 0.05, 700_001)
    y = rng.uniform(y0 - 0.05, y1 + 0.05, 700_001)
    want, total = oracle.pip_join(_oracle_chips(chips), oracle.GRID_H3, 9, x, y, len(zones))
    _set(h3ctx, tile_images=2)
    table = h3ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 9,
                             n_polygons=len(zones))
    try:
        _set(h3ctx, point_raster=0, bin_points=1)
        kept = None
        for cap in (1 << 20, -1):
            _set(h3ctx, bin_spin_cap=cap)
            assert np.array_equal(h3ctx.pip_join_count(table, x, y), want), cap
            assert h3ctx.last_kernel() == "k_join_tiles"
            rows = h3ctx.last_binned_rows()
            if cap > 0:
                kept = rows
                assert 0 < kept < len(x)
            else:
                assert rows == len(x)
            r, k = h3ctx.pip_join_pairs(table, x, y)
            assert len(r) == total and np.array_equal(np.bincount(k, minlength=len(zones)), want)
    finally:
        _set(h3ctx, point_raster=1, bin_points=1, tile_images=1, bin_spin_cap=1 << 20)
        table.close()
