"""GPU: one context shared by concurrent caller threads ("All entry points are
thread-safe.  Concurrent callers are multiplexed onto per-thread HIP streams"; INTEGRATION.md: one
context per executor, used by its task threads).  Four Python threads (ctypes releases the GIL, so
the calls overlap) join different point sets against the same chip table, counts and pairs, host
and device inputs, with different options changing underneath them; every result equals the oracle."""
import threading
import time

import numpy as np
import pytest

import oracle
from mosaic_amd.context import tessellate
from mosaic_amd.data import PolygonSet, quickstart_points

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def h3ctx():
    from mosaic_amd import MosaicContext

    ctx = MosaicContext.build("H3", "JTS")
    yield ctx
    ctx.close()


def test_concurrent_joins_on_one_context(h3ctx):
    import torch

    zones = PolygonSet.load("nyc_taxi_zones_35")
    chips = tessellate("H3", zones, 9)
    table = h3ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 9,
                             n_polygons=len(zones))
    assert table.tiles()["stream"] == 1
    offs, data = chips["wkb"]
    oc = dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
              wkb_offsets=offs, wkb=data)
    cases = []
    for t in range(4):
        x, y = quickstart_points(zones, 150_000 + 7919 * t, seed=100 + t)
        want, total = oracle.pip_join(oc, oracle.GRID_H3, 9, x, y, len(zones), threads=4)
        _, _, orow, okey = oracle.pip_join(oc, oracle.GRID_H3, 9, x, y, len(zones), pairs=True)
        cases.append((x, y, want, set(zip(orow.tolist(), okey.tolist()))))
    errors = []
    barrier = threading.Barrier(4)

    def worker(t):
        try:
            x, y, want, pairs = cases[t]
            xt = torch.from_numpy(x).cuda() if t % 2 else x
            yt = torch.from_numpy(y).cuda() if t % 2 else y
            barrier.wait()
            for it in range(6):
                got = h3ctx.pip_join_count(table, xt, yt)
                got = got.cpu().numpy() if hasattr(got, "cpu") else got
                if not np.array_equal(got, want):
                    errors.append((t, it, "counts"))
                if it % 3 == 2:
                    rows, keys = h3ctx.pip_join_pairs(table, x, y)
                    if set(zip(rows.tolist(), keys.tolist())) != pairs:
                        errors.append((t, it, "pairs"))
                # options change under the other threads; each call copies them once at entry
                h3ctx.set_option("stream_block", 512 if (t + it) % 2 else 1024)
                h3ctx.set_option("mixed_rows", (1, 2, 4)[(t + it) % 3])
        except Exception as e:  # surfaced below
            errors.append((t, "exception", repr(e)))

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=300)
    h3ctx.set_option("stream_block", 1024)
    h3ctx.set_option("mixed_rows", 2)
    table.close()
    assert not any(th.is_alive() for th in threads)
    assert not errors, errors[:5]


def test_short_lived_threads_release_their_state(h3ctx):
    """An executor's worker pool retires threads and starts new ones: every thread's state (stream,
    scratch) goes when the thread exits, a new thread never inherits a dead thread's state (even
    where the runtime reuses its pthread id), mosaic_thread_release frees the caller's state, and
    option scratch_limit frees scratch above the limit when a call returns."""
    zones = PolygonSet.load("nyc_taxi_zones_35")
    chips = tessellate("H3", zones, 9)
    table = h3ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 9,
                             n_polygons=len(zones))
    offs, data = chips["wkb"]
    oc = dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
              wkb_offsets=offs, wkb=data)
    x, y = quickstart_points(zones, 200_000, seed=7)
    want, _ = oracle.pip_join(oc, oracle.GRID_H3, 9, x, y, len(zones), threads=4)
    base, _ = h3ctx.thread_states()  # this (main) thread's state
    errors, seen = [], []

    def worker(k):
        try:
            got = h3ctx.pip_join_count(table, x, y)
            if not np.array_equal(got, want):
                errors.append((k, "counts"))
            seen.append(h3ctx.thread_states()[0])
            if k % 4 == 3:  # explicit release before exit; the next call recreates the state
                h3ctx.thread_release()
                got = h3ctx.pip_join_count(table, x, y)
                if not np.array_equal(got, want):
                    errors.append((k, "after release"))
        except Exception as e:
            errors.append((k, repr(e)))

    for wave in range(6):  # 6 rounds of 8 short-lived threads
        ths = [threading.Thread(target=worker, args=(wave * 8 + i,)) for i in range(8)]
        for th in ths:
            th.start()
        for th in ths:
            th.join(timeout=120)
        assert not any(th.is_alive() for th in ths)
        # join() returns when the Python thread is done; its OS thread runs the thread_local
        # destructors (the release) just after, so wait briefly for them
        deadline = time.time() + 10
        while h3ctx.thread_states()[0] != base and time.time() < deadline:
            time.sleep(0.01)
        assert h3ctx.thread_states()[0] == base, "exited threads left their state behind"
    assert not errors, errors[:5]
    assert max(seen) <= base + 8
    # scratch_limit: a call above the limit leaves no scratch behind; 0 keeps it
    h3ctx.set_option("scratch_limit", 1)
    got = h3ctx.pip_join_count(table, x, y)
    assert np.array_equal(got, want)
    n, held = h3ctx.thread_states()
    assert held == 0
    h3ctx.set_option("scratch_limit", 0)
    h3ctx.pip_join_count(table, x, y)
    assert h3ctx.thread_states()[1] > 0
    table.close()
