# GPU box: padded chip records (9-word stride) -- binned tests, C4 1e6 kernel stats of head and the
# k_bin_cover occupancy builds (abbuild kw6 / kw8)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04w
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_binned.py "tests/test_gpu_configs.py::test_c4_million_buildings_vs_oracle" > $O/tests.log 2>&1 || exit 1
echo tests done
cd /tmp && export TMPDIR=/tmp
for v in head kw6 kw8; do
  lib=""
  [ "$v" != head ] && lib="$R/abbuild/lib_$v.so"
  MOSAIC_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$v -o c4 -- python3 -u $R/tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 5 > $O/c4_$v.txt 2>&1 || exit 1
  find /tmp/prof_$v -name "*kernel_stats.csv" -exec cp {} $O/stats_$v.csv \;
  echo "$v done"
done
timeout -k 10 -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES --kernel-trace --output-format csv -d /tmp/pmc_lds -o run -- python3 -u $R/tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 2 > $O/pmc_lds.log 2>&1 || exit 1
find /tmp/pmc_lds -name "*counter_collection.csv" -exec cp {} $O/pmc_lds_counters.csv \;
echo pmc done
