# GPU box: tile-join segment size (kSegPoints 1024 / 4096 / 8192 builds in abbuild vs 2048 head)
# on C4 1e6 and 5e6, kernel stats only
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04y
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in head seg1024 seg4096 seg8192; do
  lib=""
  [ "$v" != head ] && lib="$R/abbuild/lib_$v.so"
  for nb in 1e6 5e6; do
    MOSAIC_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_${v}_$nb -o c4 -- python3 -u $R/tools/kbench_c4.py --buildings $nb --n 2.5e8 --reps 3 > $O/c4_${v}_$nb.txt 2>&1 || exit 1
    find /tmp/prof_${v}_$nb -name "*kernel_stats.csv" -exec cp {} $O/stats_${v}_$nb.csv \;
    echo "$v $nb done"
  done
done
