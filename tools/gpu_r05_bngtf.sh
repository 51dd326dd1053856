#!/bin/bash
# GPU box (round 5): cell-frame BNG line records -- BNG / config tests, then C5 against the previous
# library (abbuild/lib_head.so).
#   usage: bash tools/gpu_r05_bngtf.sh OUTNAME
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_bng_boundary.py > $O/tests.txt 2>&1 || exit 1
echo tests done
for k in ${REPS:-1 2}; do
  timeout -k 10 200 python3 -u tools/kbench_bng.py --reps 5 --sweep bng_group_lines=1 > $O/c5_new$k.txt 2>&1 || exit 1
  timeout -k 10 200 python3 -u tools/kbench_bng.py --reps 5 --build-opts ${OLD_OPTS:-bng_wedges=0} > $O/c5_old$k.txt 2>&1 || exit 1
done
echo kbench done
