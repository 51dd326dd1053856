# GPU box: binned-join tests, then C4 1e6 kbench (+ optional kernel trace) of the in-tree library.
# usage: [AB="v1 v2"] bash tools/gpu_c4.sh TAG [prof]   (AB: abbuild/lib_v1.so ... benched too)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_binned.py tests/test_gpu_configs.py::test_c4_million_buildings_vs_oracle > $O/tests.log 2>&1 || exit 1
echo tests done
timeout -k 10 300 python3 -u tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 5 > $O/c4.txt 2>&1 || exit 1
echo bench done
for v in $AB; do
  MOSAIC_HIP_LIB=$R/abbuild/lib_$v.so timeout -k 10 300 python3 -u tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 5 > $O/c4_$v.txt 2>&1 || exit 1
  echo "$v done"
done
if [ "$2" = prof ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_c4 -o c4 -- python3 -u $R/tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 5 > $O/prof.txt 2>&1 || exit 1
  find /tmp/prof_c4 -name "*kernel_stats.csv" -exec cp {} $O/stats.csv \;
  echo prof done
fi
