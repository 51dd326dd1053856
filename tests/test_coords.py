"""grid_pointascellid over the COORDS form of points (§8(a) row a4 / §8(f) row 3): st_point's output
InternalRow(typeId, srid, [[[x, y]]], [[]]) (expressions/constructors/ST_Point.scala:27-32,
core/types/model/InternalGeometry.scala) decoded on the GPU (k_decode_coords) the way
MosaicPointJTS.fromInternal reads it (core/geometry/point/MosaicPointJTS.scala:82-89:
boundaries.head.head; InternalCoord takes 2 values or the first 3), then indexed.  The oracle is
oracle/point_decode.py coords_point (rows the reference would throw on or whose centroid it would
take go to the row path) and the H3 / BNG oracles for the cells."""
import numpy as np
import pytest

import oracle
from oracle.point_decode import coords_point

pytestmark = pytest.mark.gpu


def _rows(rng, n):
    rows = []
    for i in range(n):
        k = i % 10
        x, y = float(rng.uniform(-74.2, -73.7)), float(rng.uniform(40.5, 40.9))
        if k == 0:
            rows.append(None)
        elif k == 1:
            rows.append((1, 4326, [[[x, y, 12.5]]], [[]]))  # 3D point: z ignored
        elif k == 2:
            rows.append((5, 0, [[[x, y], [x + 0.01, y], [x, y + 0.01], [x, y]]], [[]]))  # POLYGON: centroid
        elif k == 3:
            rows.append((1, 0, [], [[]]))  # no boundary: the reference throws
        elif k == 4:
            rows.append((1, 0, [[]], [[]]))  # no coordinate
        elif k == 5:
            rows.append((1, 0, [[[x]]], [[]]))  # one value
        elif k == 6:
            rows.append((1, 0, [[[x, y, 1.0, 2.0]]], [[]]))  # four values: the first three are read
        elif k == 7:
            rows.append((2, 0, [[[x, y]], [[x + 1e-3, y]]], [[]]))  # MULTIPOINT: centroid
        else:
            rows.append((1, 0, [[[x, y]], [[x + 1.0, y + 1.0]]], [[]]))
    return rows


@pytest.mark.parametrize("grid", ["H3", "BNG"])
def test_coords_column_matches_oracle(grid):
    from mosaic_amd import MosaicContext
    from mosaic_amd.context import CoordsColumn, st_point

    ctx = MosaicContext.build(grid, "JTS")
    try:
        rng = np.random.default_rng(17)
        if grid == "H3":
            x, y = rng.uniform(-74.3, -73.6, 200_000), rng.uniform(40.4, 41.0, 200_000)
            res = 9
            want = oracle.h3_point_to_index(x, y, res)
        else:
            x, y = rng.uniform(500000, 560000, 200_000), rng.uniform(150000, 210000, 200_000)
            res = 4
            want, err = oracle.bng_point_to_index_batch(x, y, res)
        got = ctx.grid_pointascellid(st_point(x, y), res, raw=True)
        assert np.array_equal(got, want)
        rows = _rows(rng, 5000)
        if grid == "BNG":
            rows = [None if r is None else (r[0], r[1], [[[c[0] * 1e4 + 5e5, c[1] * 1e4 - 2e5] + list(c[2:])
                                                         if len(c) >= 2 else c for c in b] for b in r[2]], r[3])
                    for r in rows]
        col = CoordsColumn.from_rows(rows)
        cells, status = ctx.grid_pointascellid(col, res, raw=True, return_status=True)
        for i, r in enumerate(rows):
            exp = coords_point(r)
            if exp[0] == "null":
                assert status[i] == 0, i
            elif exp[0] == "path":
                assert status[i] == 2, (i, r)
            else:
                assert status[i] == 1, (i, r)
                if grid == "H3":
                    c = oracle.h3_point_to_index([exp[1]], [exp[2]], res)[0]
                else:
                    c = oracle.bng_point_to_index(exp[1], exp[2], res)
                assert cells[i] == c, (i, r)
        # decode alone
        from mosaic_amd import RowPathRequired

        with pytest.raises(RowPathRequired):
            ctx.grid_pointascellid(col, res)
    finally:
        ctx.close()
