# GPU box: the two-pass wide-radix sort (17-22 bit image keys) -- binned tests, the 5e6-building
# full-size test, C4 1e6 and 5e6 kbench with kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04v
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_binned.py "tests/test_gpu_configs.py::test_c4_million_buildings_vs_oracle" "tests/test_gpu_configs.py::test_c4_full_size_five_million_buildings" > $O/tests.log 2>&1 || exit 1
echo tests done
cd /tmp && export TMPDIR=/tmp
for nb in 1e6 5e6; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$nb -o c4 -- python3 -u $R/tools/kbench_c4.py --buildings $nb --n 2.5e8 --reps 5 > $O/c4_$nb.txt 2>&1 || exit 1
  find /tmp/prof_$nb -name "*kernel_stats.csv" -exec cp {} $O/stats_$nb.csv \;
  echo "$nb done"
done
