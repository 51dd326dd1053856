"""Writes tests/golden/kring_k200_pentagons.json: for the 12 pentagons of tests/test_h3_kring.py at
k = 200 (past the device's k <= 128 search: mosaic_cell_kring answers those rows on host threads),
order-free digests of the oracle's sphere-search k-ring (oracle.h3_kring_set, independent of H3's
tables) and of the k-loop (ring k minus ring k - 1): count, sum, xor and sum of squares (mod 2^64).
~12 minutes of CPU; run once, the digests are the fixture."""
import json
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(_HERE, "..", ".."))

import oracle  # noqa: E402
from tests.test_h3_kring import PENTAGON_BASE_CELLS, pentagon_cell  # noqa: E402

K = 200
M = (1 << 64) - 1


def digest(cells):
    cells = [int(c) & M for c in cells]
    s = x = q = 0
    for c in cells:
        s = (s + c) & M
        x ^= c
        q = (q + c * c) & M
    return dict(n=len(cells), sum=s, xor=x, sumsq=q)


rows = []
for i, bc in enumerate(PENTAGON_BASE_CELLS):
    p = pentagon_cell(bc, 7 + i % 4)
    ring = set(int(c) for c in oracle.h3_kring_set(p, K))
    inner = set(int(c) for c in oracle.h3_kring_set(p, K - 1))
    rows.append(dict(cell=p, ring=digest(ring), loop=digest(ring - inner)))
    print(i, len(ring), len(ring - inner), flush=True)
json.dump(dict(k=K, source="oracle.h3_kring_set (sphere search), tests/golden/make_kring_k200.py", rows=rows),
          open(os.path.join(_HERE, "kring_k200_pentagons.json"), "w"), indent=1)
