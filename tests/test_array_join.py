"""The array form of the chip join: PointInPolygonJoin.joinArrayRows
(sql/join/PointInPolygonJoin.scala:39-66) over grid_tessellate chip arrays, one array per polygon
row -- a point joins a row when array_contains(chips.index_id, cell), and the row's chip at
array_position (the FIRST chip with the cell) decides: is_core || st_contains(wkb, point).  Checked
against a literal restatement of those three Spark functions in Python (below), on tessellated NYC
zones with a duplicated cell appended to some rows (a later chip the array form must ignore, the
exploded form would count)."""
import numpy as np
import pytest

import oracle
from mosaic_amd.context import tessellate
from mosaic_amd.data import PolygonSet, quickstart_points


def _arrays(chips, n_rows, rng, n_dup):
    """chip rows grouped per polygon row (the array column), with n_dup rows given an appended
    duplicate of one of their cells (is_core = 1: it would accept every point of the cell)"""
    key = chips["polygon_key"]
    offs, data = chips["wkb"]
    rows = [[] for _ in range(n_rows)]
    for i in np.argsort(key, kind="stable"):
        rows[key[i]].append((int(chips["is_core"][i]), int(chips["index_id"][i]), bytes(data[offs[i]:offs[i + 1]])))
    for r in rng.choice(n_rows, n_dup, replace=False):
        border = [c for c in rows[r] if c[0] == 0]
        if border:
            rows[r].append((1, border[0][1], b""))
    chip_offsets = np.zeros(n_rows + 1, np.int64)
    np.cumsum([len(r) for r in rows], out=chip_offsets[1:])
    flat = [c for r in rows for c in r]
    return rows, chip_offsets, flat


def array_join_counts(rows, x, y, res):
    """joinArrayRows literally: array_contains, array_position (first match), element_at"""
    cells = oracle.h3_point_to_index(np.asarray(x), np.asarray(y), res)
    counts = np.zeros(len(rows), np.int64)
    first = []
    for r in rows:
        d = {}
        for pos, (_, cid, _) in enumerate(r):
            d.setdefault(cid, pos)  # array_position: the first index of the value
        first.append(d)
    for i in range(len(x)):
        c = int(cells[i])
        for p, r in enumerate(rows):
            pos = first[p].get(c)
            if pos is None:
                continue
            core, _, w = r[pos]
            if core or (len(w) and oracle.wkb_contains(w, float(x[i]), float(y[i]))):
                counts[p] += 1
    return counts


def test_literal_array_join_equals_exploded_without_duplicates():
    zones = PolygonSet.load("nyc_taxi_zones").subset(list(range(0, 263, 40)))
    res = 8
    chips = tessellate("H3", zones, res)
    rng = np.random.default_rng(1)
    rows, _, _ = _arrays(chips, len(zones), rng, 0)
    x, y = quickstart_points(zones, 4000, seed=3)
    want, _ = oracle.pip_join(dict(index_id=chips["index_id"], is_core=chips["is_core"],
                                   polygon_key=chips["polygon_key"], wkb_offsets=chips["wkb"][0],
                                   wkb=chips["wkb"][1]), oracle.GRID_H3, res, x, y, len(zones))
    assert np.array_equal(array_join_counts(rows, x, y, res), want)


@pytest.mark.gpu
def test_gpu_array_join_matches_literal():
    from mosaic_amd import MosaicContext
    ctx = MosaicContext.build("H3", "JTS")
    try:
        zones = PolygonSet.load("nyc_taxi_zones").subset(list(range(0, 263, 7)))
        res = 9
        chips = tessellate("H3", zones, res, ctx=ctx)
        rng = np.random.default_rng(5)
        rows, chip_offsets, flat = _arrays(chips, len(zones), rng, 12)
        table = ctx.chip_table_arrays(chip_offsets, [c[0] for c in flat], [c[1] for c in flat],
                                      [c[2] for c in flat], res)
        x, y = quickstart_points(zones, 20000, seed=9)
        got = ctx.pip_join_count(table, x, y)
        want = array_join_counts(rows, x, y, res)
        assert np.array_equal(got, want)
        # the exploded form of the same rows counts the duplicated cells' points twice
        exploded = ctx.chip_table([c[0] for c in flat], [c[1] for c in flat], [c[2] for c in flat],
                                  np.repeat(np.arange(len(rows), dtype=np.int32), [len(r) for r in rows]), res,
                                  n_polygons=len(rows))
        assert int(ctx.pip_join_count(exploded, x, y).sum()) > int(got.sum())
        table.close()
        exploded.close()
    finally:
        ctx.close()
