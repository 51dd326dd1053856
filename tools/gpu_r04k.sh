# GPU box: C4 1e6 k_join_tiles probes (head: rare paths inlined; p1: no ring walk; p2: no pairs;
# w0 / w5: occupancy targets; head: + compacting cover keygen) and a kernel trace of head
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04k
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_binned.py tests/test_gpu_configs.py::test_c4_million_buildings_vs_oracle > $O/tests.log 2>&1 || exit 1
echo tests done
for v in head base p1 p2 w0 w5; do
  lib=""
  [ "$v" != head ] && lib="$R/abbuild/lib_$v.so"
  MOSAIC_HIP_LIB=$lib timeout -k 10 300 python3 -u tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 5 > $O/$v.txt 2>&1 || exit 1
  echo "$v done"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o c4 -- python3 -u $R/tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 5 > $O/prof.txt 2>&1 || exit 1
echo prof done
