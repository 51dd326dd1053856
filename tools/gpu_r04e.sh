# GPU box: kring probes (h3_neighbors.h alone vs the library), C4 join with compacted ring walks
# (tests, timing, kernel stats, two counter passes), C4 build side at scale with phase traces
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04e
mkdir -p $O
cd $R
timeout -k 10 60 ./tools/probes/kring_probe tools/probes/kring_cells.txt 1 > $O/kring_probe_k1.txt 2>&1 || exit 1
timeout -k 10 120 python3 -u tools/probes/kring_so_probe.py tools/probes/kring_cells.txt 1 > $O/kring_so_k1.txt 2>&1 || exit 1
bash tools/gpu_round.sh r04e "tests|tests/test_binned.py tests/test_gpu_configs.py -k c4_million" \
  "run|tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 3" "prof|tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 3" \
  "pmc|SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES@tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 2" \
  "pmc|SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT@tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 2" \
  "pmc|FETCH_SIZE@tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 2" || exit 1
MOSAIC_BUILD_TRACE=1 timeout -k 10 400 python3 -u tools/c4_build_probe.py --sizes 1e6 5e6 > $O/build_probe.txt 2> $O/build_probe.err
