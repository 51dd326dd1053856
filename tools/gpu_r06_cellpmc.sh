#!/bin/bash
# GPU box (round 6): counters of kernel (a) k_cell_h3 on 1e9 resident points (tools/cellrun.py, three
# launches; the join kernels of the same run are filtered out by tools/pmc_summary.py).  One rocprofv3
# --pmc pass per group (<= 8 SQ, <= 4 TCC counters), each under its own time limit.
#   usage: bash tools/gpu_r06_cellpmc.sh OUTNAME
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
pass() {  # pass NAME COUNTERS...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d /tmp/cpmc_$name -o run -- \
      python3 -u $R/tools/cellrun.py 1e9 > $O/$name.log 2>&1
  local rc=$?
  tail -2 $O/$name.log
  if [ $rc -ne 0 ]; then echo "PASS $name FAILED rc=$rc"; exit $rc; fi
  find /tmp/cpmc_$name -name "*counter_collection.csv" -exec cp {} $O/$name.csv \;
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass inst SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES
pass act SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT
pass f64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM
echo pmc done
