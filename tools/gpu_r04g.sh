# GPU box: kring stop reasons; C4 pair path for image-less runs and the parallel table build (tests,
# 1e6 and 5e6 timing, 1e6 counters); the chip-table error paths
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04g
mkdir -p $O
cd $R
timeout -k 10 60 ./tools/probes/kring_reason tools/probes/kring_cells.txt > $O/kring_reason.txt 2>&1 || exit 1
bash tools/gpu_round.sh r04g "tests|tests/test_binned.py tests/test_abi.py tests/test_gpu_parity.py -k not_full" \
  "run|tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 3" \
  "pmc|SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES@tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 2" \
  "pmc|SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT@tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 2" \
  "run|tools/kbench_c4.py --buildings 5e6 --n 2.5e8 --reps 3" || exit 1
