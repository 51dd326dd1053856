# GPU box: k_join_tiles occupancy variants (abbuild lib_wpe3 / lib_wpe5 vs head at 4) on C4 1e6 and
# 5e6, kernel stats only; WRITE_SIZE of the wpe3 tile join
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04t
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in head wpe3 wpe5; do
  lib=""
  [ "$v" != head ] && lib="$R/abbuild/lib_$v.so"
  for nb in 1e6 5e6; do
    MOSAIC_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_${v}_$nb -o c4 -- python3 -u $R/tools/kbench_c4.py --buildings $nb --n 2.5e8 --reps 3 > $O/c4_${v}_$nb.txt 2>&1 || exit 1
    find /tmp/prof_${v}_$nb -name "*kernel_stats.csv" -exec cp {} $O/stats_${v}_$nb.csv \;
    echo "$v $nb done"
  done
done
MOSAIC_HIP_LIB=$R/abbuild/lib_wpe3.so timeout -k 10 -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d /tmp/pmc_w3 -o run -- python3 -u $R/tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 2 > $O/pmc_w3.log 2>&1 || exit 1
find /tmp/pmc_w3 -name "*counter_collection.csv" -exec cp {} $O/pmc_w3_counters.csv \;
echo pmc done
