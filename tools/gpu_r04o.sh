# GPU box: k_bin_cover variants (nolb: in-place keys, no look-back; ppt4 / ppt16: points per
# thread; norare: tile join without its rare paths, wrong answers) under a kernel trace each
# (kernel stats only are kept)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04o
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in nolb ppt4 ppt16 norare; do
  MOSAIC_HIP_LIB=$R/abbuild/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$v -o c4 -- python3 -u $R/tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 3 > $O/c4_$v.txt 2>&1 || exit 1
  find /tmp/prof_$v -name "*kernel_stats.csv" -exec cp {} $O/stats_$v.csv \;
  echo "$v done"
done
