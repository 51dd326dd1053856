#!/bin/bash
# GPU steps of this session (round 2, fourth part): named step groups, each GPU step under its own time limit; the first
# failing step ends the script.  usage: bash tools/gpu_r02d.sh STEP
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP=${1:-quick}
run() {  # run NAME SECONDS CMD...: output to gpurun_out/NAME.log
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STEP $name FAILED rc=$rc"; exit $rc; fi
}
PYT="python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread"
case $STEP in
  bng)
    run t_bng 600 $PYT "tests/test_gpu_parity.py::test_join_bng_dense_table" "tests/test_gpu_parity.py::test_join_bng" -s
    run kb_c5_16 300 python -u tools/kbench_bng.py --cells 16
    run kb_c5_32 300 python -u tools/kbench_bng.py --cells 32
    run kb_c5_16r4 300 python -u tools/kbench_bng.py --cells 16 --build-opts mixed_rows=4
    run kb_c5_16r1 300 python -u tools/kbench_bng.py --cells 16 --build-opts mixed_rows=1
    ;;
  abnt)
    for v in base leafnt allnt; do
      if [ $v = base ]; then L=$PWD/mosaic_amd/libmosaic_hip.so; else L=$PWD/abbuild/lib_$v.so; fi
      MOSAIC_HIP_LIB=$L run kb_ab_$v 300 python -u tools/kbench.py --n 1e9 --reps 8
      MOSAIC_HIP_LIB=$L run kb_ab_bng_$v 300 python -u tools/kbench_bng.py --cells 32
    done
    ;;
  ab)  # A/B of abbuild/lib_$V.so variants against the in-tree library: VARIANTS="a b" bash tools/gpu_r02d.sh ab
    for v in base $VARIANTS; do
      if [ $v = base ]; then L=$PWD/mosaic_amd/libmosaic_hip.so; else L=$PWD/abbuild/lib_$v.so; fi
      MOSAIC_HIP_LIB=$L run kb_ab_$v 300 python -u tools/kbench.py --n 1e9 --reps 8
    done
    ;;
  qc)
    run t_qc 900 $PYT tests/test_raster_build.py "tests/test_gpu_parity.py::test_join_tiled_nyc_zones_match_oracle" \
        "tests/test_gpu_parity.py::test_join_point_raster_sizes" "tests/test_gpu_parity.py::test_join_counts_match_oracle" \
        "tests/test_gpu_parity.py::test_join_bng_dense_table" -s
    run kb_qc_c2 300 python -u tools/kbench.py --n 1e9 --reps 8
    run kb_qc_c3 300 python -u tools/kbench.py --n 1e9 --res 10 --clustered --reps 8
    run kb_qc_c5 300 python -u tools/kbench_bng.py --cells 32
    ;;
  tess)
    run t_tess 900 $PYT tests/test_tessellate_gpu.py -s
    ;;
  kring)
    run t_kring 600 $PYT tests/test_h3_kring.py tests/test_kring.py -s
    ;;
  geom)
    run t_geom 600 $PYT tests/test_h3_geom.py tests/test_h3_kring.py tests/test_bng_boundary.py -s
    ;;
  tests)
    run gpu_tests 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
    ;;
  bench)
    run bench 900 python -u bench.py
    ;;
  t)  # TESTS="tests/a.py tests/b.py" bash tools/gpu_r02d.sh t
    run t_sel 900 $PYT $TESTS -s
    ;;
  perf)  # stream-kernel change: parity subset, C2 / C3 kernel bench, SQ instruction counters
    run t_perf 900 $PYT "tests/test_gpu_parity.py::test_join_counts_match_oracle" "tests/test_gpu_parity.py::test_join_tiled_nyc_zones_match_oracle" "tests/test_gpu_parity.py::test_join_point_raster_sizes" -s
    run kb_c2 300 python -u tools/kbench.py --n 1e9 --reps 8
    run kb_c3 300 python -u tools/kbench.py --n 1e9 --res 10 --clustered --reps 8
    bash tools/pmc_sq.sh
    ;;
  full)  # whole GPU suite, smoke, bench line, kernel stats of the bench
    run gpu_tests 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
    run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
    run bench 600 python -u bench.py
    run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 -u bench.py --steps 10 --warmup 2 --cpu-sample 0 --pmc 0
    find gpurun_out/prof -name '*kernel_stats.csv' | head -3
    ;;
  *) echo "unknown step $STEP"; exit 2;;
esac
