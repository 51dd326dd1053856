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
  tests)
    run gpu_tests 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
    ;;
  bench)
    run bench 900 python -u bench.py
    ;;
  *) echo "unknown step $STEP"; exit 2;;
esac
