# GPU box: tests of the overlapped stream join and the binned join, C2 kbench over mixed_overlap,
# the bench, then the k_bin_cover variants (abbuild) under kernel traces (stats only kept)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04p
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_binned.py tests/test_gpu_parity.py \
  "tests/test_gpu_configs.py::test_c2_full_size_raster_vs_generic_vs_oracle" "tests/test_gpu_configs.py::test_c4_million_buildings_vs_oracle" > $O/tests.log 2>&1 || exit 1
echo tests done
timeout -k 10 300 python3 -u tools/kbench.py --reps 10 --sweep mixed_overlap=1 mixed_overlap=2 mixed_overlap=3 mixed_overlap=4 > $O/kbench_c2.txt 2>&1 || exit 1
echo kbench done
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench.txt 2>&1 || exit 1
echo bench done
cd /tmp && export TMPDIR=/tmp
for v in nolb ppt4 ppt16 norare; do
  MOSAIC_HIP_LIB=$R/abbuild/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$v -o c4 -- python3 -u $R/tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 3 > $O/c4_$v.txt 2>&1 || exit 1
  find /tmp/prof_$v -name "*kernel_stats.csv" -exec cp {} $O/stats_$v.csv \;
  echo "$v done"
done
