# GPU box: kring probe, the round's GPU checks, C2 / C3 / C4 kernel timing (each step under its own
# limit, stop at the first failure; the kring test runs last)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04d
mkdir -p $O
cd $R
timeout -k 10 60 ./tools/probes/kring_probe > $O/kring_probe.txt 2>&1 || exit 1
bash tools/gpu_round.sh r04d "tests|tests/test_binned.py tests/test_polyfill.py tests/test_h3_geom.py tests/test_raster_build.py tests/test_gpu_parity.py tests/test_gpu_h3_exact.py tests/test_notebook_vectors.py" \
  "run|tools/kbench.py --n 1e9 --reps 10" "run|tools/kbench.py --n 1e9 --res 10 --clustered --reps 10" \
  "run|tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 3" "prof|tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 3" \
  "tests|tests/test_h3_kring.py"
