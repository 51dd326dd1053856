# GPU box: C4 with envelope-raster candidate lists in the tile images (tests, 1e6 / 5e6 timing,
# kernel stats, counters)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04i
mkdir -p $O
cd $R
bash tools/gpu_round.sh r04i "tests|tests/test_binned.py tests/test_gpu_configs.py::test_c4_million_buildings_vs_oracle" \
  "run|tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 3" \
  "prof|tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 3" \
  "pmc|SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES@tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 2" \
  "run|tools/kbench_c4.py --buildings 5e6 --n 2.5e8 --reps 3" || exit 1
