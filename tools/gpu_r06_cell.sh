#!/bin/bash
# GPU box (round 6): kernel (a) alone -- rocprofv3 kernel stats of tools/cellrun.py (k_cell_h3 on 1e9
# resident points, 3 launches) -- after the GPU test suite (TESTS=..., skipped with NOTESTS=1).
#   usage: [AB="v1 v2"] bash tools/gpu_r06_cell.sh OUTNAME   (AB: abbuild/lib_v1.so ... profiled too)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
if [ -z "$NOTESTS" ]; then
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
echo tests done
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_cell -o cell -- python3 -u $R/tools/cellrun.py 1e9 > $O/cell_prof.txt 2>&1 || exit 1
find /tmp/prof_cell -name "*kernel_stats.csv" -exec cp {} $O/cell_kernel_stats.csv \;
for v in $AB; do
  MOSAIC_HIP_LIB=$R/abbuild/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_cell_$v -o cell -- python3 -u $R/tools/cellrun.py 1e9 > $O/cell_prof_$v.txt 2>&1 || exit 1
  find /tmp/prof_cell_$v -name "*kernel_stats.csv" -exec cp {} $O/cell_kernel_stats_$v.csv \;
done
echo cell done
