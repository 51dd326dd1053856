# GPU box: C4 -- head kernel stats and kbench (1e6), keygen / tile-join variants (abbuild, stats
# only), PMC passes of the head (k_join_tiles, k_bin_cover), and the 5e6-building join
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04q
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in head nolb ppt4 ppt16 norare calls; do
  lib=""
  [ "$v" != head ] && lib="$R/abbuild/lib_$v.so"
  MOSAIC_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$v -o c4 -- python3 -u $R/tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 5 > $O/c4_$v.txt 2>&1 || exit 1
  find /tmp/prof_$v -name "*kernel_stats.csv" -exec cp {} $O/stats_$v.csv \;
  echo "$v done"
done
cd $R
KB=tools/kbench_c4.py timeout -k 10 600 bash tools/pmc_pipe.sh gpurun_out/r04q/pmc --buildings 1e6 --n 2.5e8 > $O/pmc.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/r04q/pmc k_bin_cover > $O/pmc/summary_bin_cover.json || exit 1
rm -rf $O/pmc/p*/
echo pmc done
timeout -k 10 600 python3 -u tools/kbench_c4.py --buildings 5e6 --n 2.5e8 --reps 3 > $O/c4_5e6.txt 2>&1 || exit 1
echo 5e6 done
