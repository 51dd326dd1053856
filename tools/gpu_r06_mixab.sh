#!/bin/bash
# GPU box (round 6): the headline join (kbench, 1e9 uniform points, res 9) for the product library and
# abbuild/lib_s0.so (an earlier tree), each on its own chips and on the other's (chips saved by
# kbench --save-chips): separates the planar border clip's chips from code changes.
#   usage: bash tools/gpu_r06_mixab.sh OUTNAME
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u tools/kbench.py --reps 10 --save-chips /tmp/chips_new.npz > $O/new_new.txt 2>&1 || exit 1
MOSAIC_HIP_LIB=$R/abbuild/lib_s0.so timeout -k 10 300 python3 -u tools/kbench.py --reps 10 --save-chips /tmp/chips_old.npz > $O/old_old.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/kbench.py --reps 10 --chips /tmp/chips_old.npz > $O/new_oldchips.txt 2>&1 || exit 1
MOSAIC_HIP_LIB=$R/abbuild/lib_s0.so timeout -k 10 300 python3 -u tools/kbench.py --reps 10 --chips /tmp/chips_new.npz > $O/old_newchips.txt 2>&1 || exit 1
echo mixab done
