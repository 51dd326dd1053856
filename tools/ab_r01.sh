# A/B on the GPU box: kbench of the in-tree library and of each alternative build in abbuild/
# (same 1e9 uniform NYC res-9 workload); optional GPU parity tests first (AB_TESTS=1).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${AB_TESTS:-0}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo tests_exit=$?; tail -20 gpurun_out/ab_tests.log; exit 1; }
  tail -2 gpurun_out/ab_tests.log
fi
KB="tools/kbench.py --n 1e9 --rasters 16 --lane-edges 0 --modes 1:1 --point-raster 64x16 --reps 7 ${AB_ARGS:-}"
timeout -k 10 300 python $KB > gpurun_out/ab_new.log 2>&1 || { echo kb_new_exit=$?; tail -5 gpurun_out/ab_new.log; exit 1; }
for lib in abbuild/*.so; do
  MOSAIC_HIP_LIB=$PWD/$lib timeout -k 10 300 python $KB ${AB_ARGS_ALT:-} > gpurun_out/ab_$(basename $lib .so).log 2>&1 || { echo kb_exit=$?; tail -5 gpurun_out/ab_$(basename $lib .so).log; exit 1; }
done
for f in gpurun_out/ab_*.log; do echo "== $f"; grep -h join_ $f; done
