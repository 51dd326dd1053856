#!/bin/bash
# Round-2 GPU session: GPU test suite, kernel bench, bench line, rocprofv3 kernel stats.
# Every GPU step has its own time limit; the first failing step ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP=${1:-all}
if [[ $STEP == all || $STEP == tests ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
      > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -3 gpurun_out/gpu_tests.log
fi
if [[ $STEP == all || $STEP == kbench ]]; then
  timeout -k 10 300 python -u tools/kbench.py --n 1e9 --stream-blocks 1024 512 256 > gpurun_out/kbench.log 2>&1 \
      || { echo "kbench failed"; tail -20 gpurun_out/kbench.log; exit 1; }
  cat gpurun_out/kbench.log
fi
if [[ $STEP == configs ]]; then
  timeout -k 10 300 python -u tools/kbench.py --n 1e9 --res 10 --clustered > gpurun_out/kbench_c3.log 2>&1 \
      || { echo "kbench c3 failed"; tail -20 gpurun_out/kbench_c3.log; exit 1; }
  cat gpurun_out/kbench_c3.log
  timeout -k 10 300 python -u tools/kbench_bng.py --n 1e9 --res 4 > gpurun_out/kbench_c5.log 2>&1 \
      || { echo "kbench c5 failed"; tail -20 gpurun_out/kbench_c5.log; exit 1; }
  cat gpurun_out/kbench_c5.log
fi
if [[ $STEP == pipe ]]; then
  timeout -k 10 600 python -u -m pytest "tests/test_gpu_parity.py::test_join_tiled_nyc_zones_match_oracle" \
      "tests/test_gpu_parity.py::test_join_tessellated_chips_every_strategy" "tests/test_gpu_parity.py::test_join_point_raster_sizes" \
      "tests/test_gpu_parity.py::test_join_counts_match_oracle" tests/test_gpu_threads.py -m gpu -v \
      --timeout 300 --timeout-method thread > gpurun_out/gpu_pipetests.log 2>&1 \
      || { echo "pipe gpu tests failed"; tail -40 gpurun_out/gpu_pipetests.log; exit 1; }
  tail -3 gpurun_out/gpu_pipetests.log
  timeout -k 10 300 python -u tools/kbench.py --n 1e9 --sweep stream_pipe=0 stream_pipe=1 > gpurun_out/kbench_pipe.log 2>&1 \
      || { echo "kbench failed"; tail -20 gpurun_out/kbench_pipe.log; exit 1; }
  cat gpurun_out/kbench_pipe.log
  timeout -k 10 300 python -u tools/kbench.py --n 1e9 --res 10 --clustered --sweep stream_pipe=0 stream_pipe=1 > gpurun_out/kbench_pipe_c3.log 2>&1 \
      || { echo "kbench c3 failed"; tail -20 gpurun_out/kbench_pipe_c3.log; exit 1; }
  cat gpurun_out/kbench_pipe_c3.log
  timeout -k 10 300 python -u tools/kbench_bng.py --n 1e9 --res 4 > gpurun_out/kbench_c5.log 2>&1 \
      || { echo "kbench c5 failed"; tail -20 gpurun_out/kbench_c5.log; exit 1; }
  cat gpurun_out/kbench_c5.log
  timeout -k 10 600 python -u -m pytest "tests/test_gpu_parity.py::test_join_bng_dense_table" "tests/test_gpu_parity.py::test_join_bng" \
      tests/test_bng_parse.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_bngtests.log 2>&1 \
      || { echo "bng gpu tests failed"; tail -40 gpurun_out/gpu_bngtests.log; exit 1; }
  tail -3 gpurun_out/gpu_bngtests.log
fi
if [[ $STEP == newtests ]]; then
  timeout -k 10 600 python -u -m pytest tests/test_coords.py tests/test_bng_parse.py tests/test_tessellate_gpu.py \
      "tests/test_gpu_parity.py::test_join_bng_dense_table" "tests/test_gpu_parity.py::test_join_bng" -m gpu -v \
      --timeout 300 --timeout-method thread > gpurun_out/gpu_newtests.log 2>&1 \
      || { echo "new gpu tests failed"; tail -40 gpurun_out/gpu_newtests.log; exit 1; }
  tail -3 gpurun_out/gpu_newtests.log
fi
if [[ $STEP == all || $STEP == bench ]]; then
  timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err \
      || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
if [[ $STEP == all || $STEP == prof ]]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o bench \
      -- python3 "$GRAFT_REPO_ROOT/bench.py" --pmc 0 --cpu-sample 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 \
      || { echo "rocprof failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
  cd "$GRAFT_REPO_ROOT"
  find gpurun_out/prof -name "*kernel_stats.csv" | head -3
  for f in $(find gpurun_out/prof -name "*kernel_stats.csv"); do head -8 "$f"; done
fi
