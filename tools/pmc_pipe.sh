#!/bin/bash
# PMC passes for the dominant stream kernel on tools/kbench.py (k_join_stream_pipe, 1e9 device points;
# KB=tools/kbench_bng.py for k_join_stream_bng), one counter group per rocprofv3 run, kernel trace
# only (never combined with other trace domains), each pass under its own time limit; stops at the
# first failure.
#   usage: [KB=tools/kbench_bng.py] bash tools/pmc_pipe.sh OUTDIR [bench args...]
# Groups stay within one pass's limits (<= 8 SQ, <= 4 TCC: FETCH_SIZE uses 3, WRITE_SIZE 2).
set -o pipefail
out=${1:-gpurun_out/pmc_pipe}
shift
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/$out
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL"; do
  i=$((i+1))
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/$out/p$i -o run -- \
      python3 -u $R/${KB:-tools/kbench.py} --reps 2 "$@" > $R/$out/p$i.log 2>&1
  rc=$?
  echo "group $i ($grp) exit=$rc"
  if [ $rc -ne 0 ]; then tail -3 $R/$out/p$i.log; break; fi
done
python3 $R/tools/pmc_summary.py $R/$out > $R/$out/summary.json && cat $R/$out/summary.json
