#!/bin/bash
# GPU box (round 6): tessellation timing with the planar border clip (tools/kbench_tess.py), C4 kernel
# stats at 5e6 buildings, then the k_cell_h3 counter passes (tools/gpu_r06_cellpmc.sh).
#   usage: bash tools/gpu_r06_meas.sh OUTNAME
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 500 python3 -u tools/kbench_tess.py --buildings 2e5 > $O/tess.txt 2>&1 || exit 1
echo tess done
(cd /tmp && TMPDIR=/tmp timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4prof5e6 -o run -- \
    python3 -u $R/tools/kbench_c4.py --buildings 5e6 --n 2.5e8 --reps 3 > $O/c4prof5e6.log 2>&1) || exit 1
echo c4 done
bash tools/gpu_r06_cellpmc.sh $1/cellpmc || exit 1
