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
    h3ctx.set_option("mixed_rows", 1)
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


def test_stream_order_after_release_and_wait_event(h3ctx):
    """after set_stream + thread_release the next call runs on a fresh context stream, so
    columns torch writes on its own stream must still be ordered before the engine reads them (the
    mirror records an event on torch's stream and the engine's stream waits for it,
    mosaic_stream_wait_event).  The columns are produced by a long chain of torch kernels right
    before each call, so reading them early would see zeros."""
    import torch

    zones = PolygonSet.load("nyc_taxi_zones_35")
    chips = tessellate("H3", zones, 9)
    table = h3ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], 9,
                             n_polygons=len(zones))
    offs, data = chips["wkb"]
    oc = dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
              wkb_offsets=offs, wkb=data)
    x, y = quickstart_points(zones, 2_000_000, seed=11)
    want, _ = oracle.pip_join(oc, oracle.GRID_H3, 9, x, y, len(zones), threads=8)
    side = torch.cuda.Stream()

    def produce():
        with torch.cuda.stream(side):
            xt = torch.zeros(len(x), dtype=torch.float64, device="cuda")
            yt = torch.zeros(len(y), dtype=torch.float64, device="cuda")
            big = torch.ones(1 << 26, dtype=torch.float64, device="cuda")
            for _ in range(20):  # delay the columns' final write
                big.mul_(1.0000001)
            xt.copy_(torch.from_numpy(x).pin_memory(), non_blocking=True)
            yt.copy_(torch.from_numpy(y).pin_memory(), non_blocking=True)
        return xt, yt, big

    h3ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    h3ctx.thread_release()
    assert getattr(h3ctx._bound, "stream", "unset") is None
    with torch.cuda.stream(side):
        xt, yt, big = produce()
        got = h3ctx.pip_join_count(table, xt, yt)  # ordered after `side` by the mirror's event
        got = got.cpu().numpy() if hasattr(got, "cpu") else got
    assert np.array_equal(got, want)
    # the raw ABI: an event recorded on the producer stream, waited for by the engine's stream
    xt, yt, big = produce()
    ev = torch.cuda.Event()
    ev.record(side)
    h3ctx.wait_event(ev.cuda_event)
    h3ctx._bound.stream = "bound"  # bypass the mirror's own ordering: only the event orders the call
    try:
        got = h3ctx.pip_join_count(table, xt, yt)
    finally:
        h3ctx._bound.stream = None
    got = got.cpu().numpy() if hasattr(got, "cpu") else got
    assert np.array_equal(got, want)
    del big
    table.close()
