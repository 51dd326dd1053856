"""Benchmark: PIP-join points/sec (whole node) at H3 res 9 -- BASELINE.json metric.

Workload (BASELINE.json configs[1], the single-GPU config): 1e9 uniform synthetic points per GPU
over the NYC taxi-zone bounding box, joined to the 263 taxi zones' res-9 chips
(grid_tessellateexplode output, built once on the host), Quickstart semantics
(cell == chip.index_id && (is_core || st_contains(chip.wkb, point))), reduced to per-zone counts.
A step = one pass of the fused join kernel over the resident batch (+ the exact-H3 pass for the
rare ambiguous points); with N > 1 GPUs each rank owns its own 1e9-point shard (weak scaling) and
the step ends with one RCCL all-reduce of the int64[263] counts.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Rank 0 prints one JSON line.  `roofline` prices the fused join kernel against the HBM roofline of
its 16 B/point algorithmic input stream (kernel time from HIP events on the launch stream);
`cpu_baseline` times the CPU restatement (oracle/, "port") of the same join on a bounded sample.
"""
import argparse
import glob
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BYTES_PER_POINT = 16     # two float64 coordinates
# the fused join kernel of the default pip_mode (3): k_join_tiled when the chip table has an H3 tile
# directory (tiles.h), else k_join_raster; set in main() from the table
JOIN_KERNEL = "k_join_tiled"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--points-per-gpu", type=float, default=1e9)
    p.add_argument("--res", type=int, default=9)
    p.add_argument("--cpu-sample", type=float, default=3e8, help="points for the CPU baseline (0 = skip)")
    p.add_argument("--cpu-threads", type=int, default=16)
    p.add_argument("--pmc", type=int, default=1, help="1: measure HBM traffic with a rocprofv3 PMC child pass")
    p.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--block", type=int, default=256)
    p.add_argument("--blocks-per-cu", type=int, default=8)
    return p.parse_args()


def build_chips(res):
    from mosaic_amd.context import tessellate
    from mosaic_amd.data import PolygonSet

    zones = PolygonSet.load("nyc_taxi_zones")
    chips = tessellate("H3", zones, res)
    return zones, chips


def cpu_baseline(zones, chips, res, n, threads):
    """The oracle (C restatement of the reference's algorithm, pthreads) on a bounded sample."""
    import oracle
    from mosaic_amd.data import uniform_points

    x, y = uniform_points(zones.bbox(), int(n), config=2)
    offs, data = chips["wkb"]
    oc = dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
              wkb_offsets=offs, wkb=data)
    oracle.lib()
    t0 = time.perf_counter()
    counts, total = oracle.pip_join(oc, oracle.GRID_H3, res, x, y, len(zones), threads=threads)
    dt = time.perf_counter() - t0
    return {"value": len(x) / dt, "unit": "points/s", "cores": threads, "kind": "port",
            "sample": f"{len(x):.0f} uniform points over the NYC zone bbox, H3 res {res}, same chips "
                      f"({total} pairs), {dt:.1f} s, CPU restatement (oracle/join.c), not Spark"}


def pmc_traffic(args):
    """rocprofv3 PMC child pass (FETCH_SIZE / WRITE_SIZE only, its own run) on the same launch shape;
    returns HBM bytes per fused-kernel launch with the gfx950 FETCH_SIZE x2 correction."""
    import shutil

    exe = shutil.which("rocprofv3")
    if not exe:
        return None, "rocprofv3 not found"
    out_dir = os.path.join(ROOT, "gpurun_out", "bench_pmc")
    os.makedirs(out_dir, exist_ok=True)
    res = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(out_dir, counter)
        cmd = [exe, "--pmc", counter, "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "pmc", "--",
               sys.executable, os.path.join(ROOT, "bench.py"), "--pmc-child", "--steps", "2", "--warmup", "1",
               "--points-per-gpu", str(args.points_per_gpu), "--res", str(args.res), "--cpu-sample", "0",
               "--pmc", "0"]
        r = subprocess.run(cmd, cwd="/tmp", capture_output=True, text=True, timeout=900)
        if r.returncode != 0:
            return None, f"rocprofv3 {counter} failed: {r.stderr[-400:]}"
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            return None, f"no counter csv for {counter}"
        vals = []
        import csv

        for f in files:
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if JOIN_KERNEL in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                        vals.append(float(row["Counter_Value"]))
        if not vals:
            return None, f"no {JOIN_KERNEL} rows for {counter}"
        res[counter] = float(np.mean(vals))
    # FETCH_SIZE / WRITE_SIZE are in KiB; gfx950 FETCH_SIZE reads half of a wide streaming read
    # (MI355X_MICROARCH.md, HBM section): double it.
    traffic = (2.0 * res["FETCH_SIZE"] + res["WRITE_SIZE"]) * 1024.0
    return traffic, res


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from mosaic_amd import distributed as D

    rank, world, local = D.init("nccl")
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")

    from mosaic_amd import MosaicContext
    from mosaic_amd.data import SEED_BASE, uniform_points_device

    zones, chips = build_chips(args.res)
    ctx = MosaicContext.build("H3", "JTS", device=local)
    ctx.set_option("block", args.block)
    ctx.set_option("blocks_per_cu", args.blocks_per_cu)
    table = ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], args.res,
                           n_polygons=len(zones))
    global JOIN_KERNEL
    tiles = table.tiles()
    JOIN_KERNEL = ("k_join_stream" if tiles["raster"] else "k_join_tiled") if tiles["built"] else "k_join_raster"
    n = int(args.points_per_gpu)
    x, y = uniform_points_device(zones.bbox(), n, seed=SEED_BASE + 2 + 1000 * rank, device=dev)
    counts = torch.zeros(len(zones), dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)
    ctx.set_option("async", 1)

    def step():
        ctx.pip_join_count(table, x, y, out=counts)
        D.allreduce_counts(counts)

    for _ in range(args.warmup):
        step()
    ctx.sync()
    ctx.set_option("timing", 1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.sync()  # deferred errors (e.g. exact-path queue overflow) surface here
    kernel_ms = ctx.kernel_times()
    ctx.set_option("timing", 0)
    elapsed = D.max_over_ranks(elapsed, device=dev)

    # one synchronous step for counters (exact-path rows, contains tests)
    ctx.set_option("async", 0)
    check = ctx.pip_join_count(table, x, y)
    stats = ctx.last_stats()
    if args.pmc_child:
        return
    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    total_points = world * n * args.steps
    value = total_points / elapsed
    k_avg_ms = float(np.mean(kernel_ms)) if len(kernel_ms) else None
    achieved = (BYTES_PER_POINT * n) / (k_avg_ms * 1e-3) / 1e9 if k_avg_ms else None
    traffic, pmc_note = (None, "skipped")
    if args.pmc and world == 1:
        try:
            traffic, pmc_note = pmc_traffic(args)
        except Exception as e:  # the measurement is optional; never fail the bench on it
            traffic, pmc_note = None, f"pmc error: {e}"
    cpu = None
    if args.cpu_sample > 0 and world == 1:
        cpu = cpu_baseline(zones, chips, args.res, args.cpu_sample, args.cpu_threads)
    info = table.info()
    line = {
        "metric": "PIP-join points/sec (whole node) at H3 res 9, 1/2/4/8 MI355X vs CPU host",
        "value": value,
        "unit": "points/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (uniform points over the NYC taxi-zone bbox, torch Philox on device; "
                "263 NYC taxi zones from the reference's notebooks/data)",
        "config": {"workload": "configs[1]: 1e9 uniform points per GPU vs 263 NYC taxi zones, H3 res "
                               f"{args.res}, Quickstart chip join reduced to per-zone counts",
                   "points_per_gpu": n, "res": args.res, "chips": info["n_chips"], "border_chips": info["n_border"],
                   "chip_cells": info["n_cells"], "tile_directory": {k: tiles[k] for k in
                                                                     ("built", "nx", "ny", "records", "entries")},
                   "parallelism": f"dp{world}",
                   "collective": "RCCL all_reduce int64[263] per step" if world > 1 else "none"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": (achieved / HBM_PEAK_GBPS) if achieved else None,
                     "traffic": traffic, "kernel": JOIN_KERNEL,
                     "kernel_ms": k_avg_ms, "algorithmic_bytes_per_launch": BYTES_PER_POINT * n,
                     "pmc": pmc_note},
        "cpu_baseline": cpu,
        "stats": {"exact_path_rows_per_step": stats["exact_path_rows"],
                  "contains_tests_per_step": stats["contains_tests"],
                  "pairs_per_step": int(check.sum().item())},
    }
    print(json.dumps(line))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
