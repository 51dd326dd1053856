#!/bin/bash
# GPU box: C4 (border-chip-heavy, H3 res 11) join -- parity tests of the binned join, timing at 1e6
# buildings (binned and unbinned) and 5e6 buildings, rocprofv3 kernel stats of the 1e6 run, then
# PMC passes (one counter group per run).  Every GPU step under its own time limit; stops at the
# first failure.
#   usage: bash tools/gpu_c4_measure.sh OUTNAME [pmc]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-c4}
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_binned.py tests/test_gpu_threads.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --variants bin_points=1 bin_points=0 > $O/c4_1e6.txt 2>&1 || exit 1
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u $R/tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 3 > $O/c4_prof.log 2>&1 || exit 1
if [ "$2" == "pmc" ]; then
i=0
for grp in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 -s KILL 200 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/p$i -o run -- \
      python3 -u $R/tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 2 > $O/p$i.log 2>&1
  rc=$?
  echo "group $i ($grp) exit=$rc"
  if [ $rc -ne 0 ]; then tail -3 $O/p$i.log; exit 1; fi
done
fi
cd $R
timeout -k 10 400 python3 -u tools/kbench_c4.py --buildings 5e6 --n 2.5e8 --reps 3 > $O/c4_5e6.txt 2>&1
