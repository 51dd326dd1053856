# GPU box: kring step trace; C4 with the branch-light ring walk (tests, timing, kernel stats, 5e6
# buildings with and without small-ring rasters); C2 bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04f
mkdir -p $O
cd $R
timeout -k 10 60 ./tools/probes/kring_trace tools/probes/kring_cells.txt > $O/kring_trace.txt 2>&1 || exit 1
bash tools/gpu_round.sh r04f "tests|tests/test_binned.py tests/test_gpu_configs.py -k c4_million" \
  "run|tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 3" "prof|tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 3" \
  "run|tools/kbench_c4.py --buildings 5e6 --n 2.5e8 --reps 3 --variants raster_min_segments=16" \
  "run|bench.py --steps 20 --warmup 5" || exit 1
