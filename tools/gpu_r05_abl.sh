#!/bin/bash
# GPU box (round 5): upper bound of the stream kernel's gather misses -- C2 with the in-tree library
# against measurement builds whose line (1), leaf (2) and sub-block (4) gathers stay within 4 KB
# (abbuild/lib_ablN.so, -DMOSAIC_ABL_GATHER_HIT=N; every such row answers key 0; 8: that answer with
# the gathers at their real addresses -- the control; timing only).
#   usage: bash tools/gpu_r05_abl.sh OUTNAME
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 200 python3 -u tools/kbench.py --reps 10 > $O/head.txt 2>&1 || exit 1
for v in ${ABL_VARIANTS:-8 1 2 3}; do
  MOSAIC_HIP_LIB=$R/abbuild/lib_abl$v.so timeout -k 10 200 python3 -u tools/kbench.py --reps 10 > $O/abl$v.txt 2>&1 || exit 1
done
timeout -k 10 200 python3 -u tools/kbench.py --reps 10 > $O/head2.txt 2>&1 || exit 1
echo done
