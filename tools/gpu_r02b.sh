#!/bin/bash
# GPU steps of this session: named step groups, each GPU step under its own time limit; the first
# failing step ends the script.  usage: bash tools/gpu_r02b.sh STEP
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
  qrec)
    run t_qrec 600 $PYT tests/test_raster_build.py "tests/test_gpu_parity.py::test_join_tiled_nyc_zones_match_oracle" \
        "tests/test_gpu_parity.py::test_join_point_raster_sizes" "tests/test_gpu_parity.py::test_join_counts_match_oracle" -s
    run kb_qrec_c2 300 python -u tools/kbench.py --n 1e9 --build-opts raster_quad_records=0 raster_quad_records=1
    run kb_qrec_c3 300 python -u tools/kbench.py --n 1e9 --res 10 --clustered --build-opts raster_quad_records=0 raster_quad_records=1
    ;;
  probe)
    run stream_probe 120 ./tools/probes/stream_probe 1e9
    ;;
  sweep1)
    run kb_sweep1 400 python -u tools/kbench.py --n 1e9 --reps 6 --stream-blocks 1024 512 --sweep stream_pipe=0 stream_pipe=1 \
        stream_pipe=1,mixed_rows=1 stream_pipe=1,mixed_rows=2 stream_pipe=1,mixed_blocks_per_cu=16
    ;;
  rbw)
    run t_rbw 600 $PYT tests/test_raster_build.py -s
    run build_prof 300 python -u tools/build_prof.py
    ;;
  clip)
    run t_clip 900 $PYT tests/test_tessellate_gpu.py tests/test_raster_build.py -s
    run build_prof 300 python -u tools/build_prof.py
    run kb_tess 300 python -u tools/kbench_tess.py
    ;;
  cfg)
    run t_cfg 900 $PYT tests/test_gpu_configs.py tests/test_tessellate_gpu.py -s
    ;;
  bprof0)
    run build_prof 300 python -u tools/build_prof.py
    cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/bprof -o bp -- \
        python3 $GRAFT_REPO_ROOT/tools/build_prof.py > $GRAFT_REPO_ROOT/gpurun_out/bprof.log 2>&1 \
        || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/bprof.log; exit 1; }
    cd $GRAFT_REPO_ROOT && find gpurun_out/bprof -name "*kernel_stats.csv" -exec head -20 {} \;
    ;;
  bprof)
    run t_bprof 600 $PYT tests/test_raster_build.py "tests/test_gpu_parity.py::test_join_counts_match_oracle" \
        "tests/test_gpu_parity.py::test_join_c4_buildings" -s
    run build_prof 300 python -u tools/build_prof.py
    cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/bprof -o bp -- \
        python3 $GRAFT_REPO_ROOT/tools/build_prof.py > $GRAFT_REPO_ROOT/gpurun_out/bprof.log 2>&1 \
        || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/bprof.log; exit 1; }
    cd $GRAFT_REPO_ROOT && find gpurun_out/bprof -name "*kernel_stats.csv" -exec head -20 {} \;
    ;;
  tests)
    run gpu_tests 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
    ;;
  bench)
    run bench 900 python -u bench.py
    ;;
  *) echo "unknown step $STEP"; exit 2;;
esac
