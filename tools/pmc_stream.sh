# PMC passes over tools/joinrun.py (GPU box), one counter group per rocprofv3 run, kernel trace only
# (never combined with other trace domains).  usage: bash tools/pmc_stream.sh SUBxCELL NPOINTS OUTDIR
set -o pipefail
cfg=${1:-64x16}
npts=${2:-1e9}
out=${3:-gpurun_out/pmc_stream}
R=$GRAFT_REPO_ROOT
mkdir -p $R/$out
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/$out/p$i -o run -- python3 $R/tools/joinrun.py $cfg $npts > $R/$out/p$i.log 2>&1
  rc=$?
  echo "group $i ($grp) exit=$rc"
  if [ $rc -ne 0 ]; then tail -3 $R/$out/p$i.log; fi
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then break; fi
done
python3 $R/tools/pmc_summary.py $R/$out > $R/$out/summary.json && cat $R/$out/summary.json
