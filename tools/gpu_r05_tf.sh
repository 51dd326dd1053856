#!/bin/bash
# GPU box (round 5): tile-frame line records -- the GPU suite, then C2 / C3 against the previous
# library (abbuild/lib_head.so).
#   usage: bash tools/gpu_r05_tf.sh OUTNAME
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.txt 2>&1 || exit 1
echo tests done
for k in 1 2; do
  timeout -k 10 200 python3 -u tools/kbench.py --reps 10 > $O/c2_new$k.txt 2>&1 || exit 1
  MOSAIC_HIP_LIB=$R/abbuild/lib_head.so timeout -k 10 200 python3 -u tools/kbench.py --reps 10 > $O/c2_old$k.txt 2>&1 || exit 1
done
timeout -k 10 200 python3 -u tools/kbench.py --reps 10 --res 10 --clustered > $O/c3_new.txt 2>&1 || exit 1
MOSAIC_HIP_LIB=$R/abbuild/lib_head.so timeout -k 10 200 python3 -u tools/kbench.py --reps 10 --res 10 --clustered > $O/c3_old.txt 2>&1 || exit 1
echo kbench done
