# PMC passes over tools/cellrun.py (GPU box).  One counter group per rocprofv3 run, kernel trace
# only (no sys/runtime traces with --pmc).
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 120 rocprofv3 --list-avail > $R/gpurun_out/pmc/avail.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU" "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" \
           "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/gpurun_out/pmc/p$i -o run -- python3 $R/tools/cellrun.py > $R/gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "group $i ($grp) exit=$rc"
  if [ $rc -ne 0 ]; then tail -5 $R/gpurun_out/pmc/p$i.log; fi
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then break; fi
done
