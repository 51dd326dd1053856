"""Benchmark: PIP-join points/sec (whole node) at H3 res 9 -- BASELINE.json metric.

Workload (BASELINE.json configs[1], the single-GPU config): 1e9 uniform synthetic points per GPU
over the NYC taxi-zone bounding box, joined to the 263 taxi zones' res-9 chips
(grid_tessellateexplode output), Quickstart semantics
(cell == chip.index_id && (is_core || st_contains(chip.wkb, point))), reduced to per-zone counts.
A step = one pass of the join over the resident batch (stream kernel, mixed-row kernel, exact-H3
pass for the rare ambiguous points); with N > 1 GPUs each rank owns its own 1e9-point shard (weak
scaling) and the step ends with one RCCL all-reduce of the int64[263] counts.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Without a torchrun environment, --gpus N > 1 relaunches itself under torch.distributed.run (before
touching the GPU) and exits with its status.  Rank 0 prints one JSON line.  `roofline` prices the
stream kernel against the HBM roofline of its 16 B/point algorithmic input stream (kernel time from
HIP events on the launch stream); `cpu_baseline` times the CPU restatement (oracle/, "port") on a
bounded prefix of the SAME device points, whose counts must equal the GPU's on that prefix
(`parity`; the bench fails otherwise); `config.build_s` is the build side (tessellation + chip
table with tile directory and point raster) and `end_to_end_points_per_s` one pass including it.
"""
import argparse
import glob
import json
import os
import platform
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BYTES_PER_POINT = 16     # two float64 coordinates
JOIN_KERNEL = "k_join_stream_cpt"  # set in main() from the first join


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--points-per-gpu", type=float, default=1e9)
    p.add_argument("--res", type=int, default=9)
    p.add_argument("--cpu-sample", type=float, default=2e8,
                   help="prefix of the device points joined by the CPU oracle (0 = skip)")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="threads of the CPU baseline (0 = every CPU this process may run on)")
    p.add_argument("--pmc", type=int, default=1, help="1: measure HBM traffic with a rocprofv3 PMC child pass")
    p.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    return p.parse_args()


def relaunch(args):
    """--gpus N > 1 outside torchrun: run this script under torch.distributed.run as a child."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def host_info():
    cpu = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    rocm = None
    for path in ("/opt/rocm/.info/version", "/opt/rocm/.info/version-dev"):
        try:
            with open(path) as f:
                rocm = f.read().strip()
                break
        except OSError:
            pass
    return {"cpu_model": cpu, "nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "cgroup_cpus": cgroup_cpus(), "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "usable_cpus": usable_cpus(), "rocm": rocm}


def cgroup_cpus():
    """The CPU quota of this process's cgroup (cpu.max quota / period), or None when unlimited."""
    try:
        with open("/proc/self/cgroup") as f:
            rel = [l.strip().split(":", 2)[2] for l in f if l.startswith("0::")][0]
        with open(os.path.join("/sys/fs/cgroup", rel.lstrip("/"), "cpu.max")) as f:
            quota, period = f.read().split()
        return None if quota == "max" else float(quota) / float(period)
    except (OSError, IndexError, ValueError):
        return None


def usable_cpus():
    """CPUs this process may use: its affinity mask, capped by its cgroup's CPU quota and by the
    lease's declared share (OMP_NUM_THREADS, which the GPU box sets to its CPU share)."""
    n = len(os.sched_getaffinity(0))
    q = cgroup_cpus()
    if q:
        n = min(n, int(q))
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return max(1, n)


def build_chips(ctx, res, rank, world):
    """Rank 0 tessellates (grid_tessellateexplode, cell classification on its GPU); the chip columns go
    to the other ranks as raw buffers over the process group (broadcast_chip_set: one build per node
    instead of one per rank, no pickling)."""
    from mosaic_amd.data import PolygonSet

    zones = PolygonSet.load("nyc_taxi_zones")
    t0 = time.perf_counter()
    chips = None
    if rank == 0:
        chips = ctx.grid_tessellateexplode(zones, res)
    if world > 1:
        import torch
        import torch.distributed as dist

        from mosaic_amd.distributed import broadcast_chip_set

        dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else None
        chips = broadcast_chip_set(chips, src=0, device=dev)
    return zones, chips, time.perf_counter() - t0


def cpu_baseline(chips, res, n_zones, x, y, threads):
    """The oracle (C restatement of the reference's algorithm, pthreads) on the given host points."""
    import oracle

    offs, data = chips["wkb"]
    oc = dict(index_id=chips["index_id"], is_core=chips["is_core"], polygon_key=chips["polygon_key"],
              wkb_offsets=offs, wkb=data)
    oracle.lib()
    t0 = time.perf_counter()
    counts, total = oracle.pip_join(oc, oracle.GRID_H3, res, x, y, n_zones, threads=threads)
    dt = time.perf_counter() - t0
    return counts, total, dt


def pmc_traffic(args):
    """rocprofv3 PMC child pass (FETCH_SIZE / WRITE_SIZE only, each its own run) on the same launch
    shape; returns HBM bytes per stream-kernel launch with the gfx950 FETCH_SIZE x2 correction."""
    import csv
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
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch(args))
    import torch
    import torch.distributed as dist

    from mosaic_amd import distributed as D

    rank, world, local = D.init("nccl")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
        sys.exit(2)
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")

    from mosaic_amd import MosaicContext
    from mosaic_amd.data import SEED_BASE, uniform_points_device

    ctx = MosaicContext.build("H3", "JTS", device=local)
    # HIP runtime start-up (code object load, first launch) is paid once per process, before any
    # build: timed apart from the build side
    t0 = time.perf_counter()
    ctx.grid_longlatascellid(np.zeros(1), np.zeros(1), args.res, raw=True)
    gpu_init_s = time.perf_counter() - t0
    zones, chips, tess_s = build_chips(ctx, args.res, rank, world)
    t0 = time.perf_counter()
    table = ctx.chip_table(chips["is_core"], chips["index_id"], chips["wkb"], chips["polygon_key"], args.res,
                           n_polygons=len(zones))
    table_s = time.perf_counter() - t0
    global JOIN_KERNEL
    tiles = table.tiles()
    # the point-raster join on 16-byte aligned device columns runs the software-pipelined stream kernel
    JOIN_KERNEL = "k_join_stream_cpt"  # until the first pass reports the kernel that ran
    n = int(args.points_per_gpu)
    x, y = uniform_points_device(zones.bbox(), n, seed=SEED_BASE + 2 + 1000 * rank, device=dev)
    counts = torch.zeros(len(zones), dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)
    ctx.set_option("async", 1)

    def step():
        ctx.pip_join_count(table, x, y, out=counts)
        D.allreduce_counts(counts)

    # one untimed first pass: the end-to-end (build + one join) figure
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    step()
    torch.cuda.synchronize(dev)
    first_pass_s = time.perf_counter() - t0
    JOIN_KERNEL = ctx.last_kernel()  # the stream kernel the join ran (roofline label, PMC filter)
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
    # parity on the full-size workload: the CPU oracle on a prefix of the same device points
    parity = None
    cpu = None
    if args.cpu_sample > 0 and rank == 0:
        m = int(min(args.cpu_sample, n))
        gpu_prefix = ctx.pip_join_count(table, x[:m], y[:m]).cpu().numpy()
        hx, hy = x[:m].cpu().numpy(), y[:m].cpu().numpy()
        threads = args.cpu_threads or usable_cpus()
        want, total, dt = cpu_baseline(chips, args.res, len(zones), hx, hy, threads)
        match = bool(np.array_equal(gpu_prefix, want))
        parity = {"points": m, "pairs": int(total), "match": match,
                  "against": "oracle/join.c (CPU restatement of the reference's join) on the first "
                             f"{m} of this rank's device points"}
        cpu = {"value": m / dt, "unit": "points/s", "cores": threads, "kind": "port",
               "sample": f"the first {m:.0f} of the benchmarked device points (uniform over the NYC zone bbox), "
                         f"H3 res {args.res}, same chips ({total} pairs), {dt:.1f} s, CPU restatement "
                         "(oracle/join.c), not Spark"}
        del hx, hy
    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    if parity is not None and not parity["match"]:
        print(json.dumps({"error": "GPU counts differ from the oracle on the parity prefix", "parity": parity}))
        sys.exit(3)

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
    info = table.info()
    binfo = table.build_info()
    build_s = tess_s + table_s
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
                   "chip_cells": info["n_cells"],
                   "tile_directory": {k: tiles[k] for k in ("built", "nx", "ny", "records", "entries")},
                   "point_raster": {k: tiles[k] for k in ("raster", "raster_sub", "raster_cell", "quad_entries",
                                                          "raster_bytes", "stream")},
                   "parallelism": f"dp{world}",
                   "collective": "RCCL all_reduce int64[263] per step" if world > 1 else "none",
                   "build_s": round(build_s, 4), "tessellate_s": round(tess_s, 4), "chip_table_s": round(table_s, 4),
                   "chip_table_ms": {k: round(binfo[k], 2) for k in ("core_ms", "directory_ms", "raster_classify_ms",
                                                                     "raster_assemble_ms")},
                   "gpu_init_s": round(gpu_init_s, 3),
                   "first_pass_s": round(first_pass_s, 4),
                   "end_to_end_points_per_s": world * n / (build_s + elapsed / args.steps)},
        "host": host_info(),
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": (achieved / HBM_PEAK_GBPS) if achieved else None,
                     "traffic": traffic, "kernel": JOIN_KERNEL,
                     "kernel_ms": k_avg_ms, "algorithmic_bytes_per_launch": BYTES_PER_POINT * n,
                     "pmc": pmc_note},
        "cpu_baseline": cpu,
        "parity": parity,
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
