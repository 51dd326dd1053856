# PMC passes over tools/joinrun.py (GPU box), one counter group per rocprofv3 run, kernel trace only.
# usage: bash tools/pmc_stream.sh SUBxCELL OUTDIR
set -o pipefail
cfg=${1:-16x8}
out=${2:-gpurun_out/pmc_stream}
R=$GRAFT_REPO_ROOT
mkdir -p $R/$out
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_LDS" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/$out/p$i -o run -- python3 $R/tools/joinrun.py $cfg 1e8 > $R/$out/p$i.log 2>&1
  rc=$?
  echo "group $i ($grp) exit=$rc"
  if [ $rc -ne 0 ]; then tail -3 $R/$out/p$i.log; fi
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then break; fi
done
