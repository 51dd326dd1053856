#!/bin/bash
# GPU box (round 6): k_cell_h3 time against its grid (tools/cell_sweep.py), for the product library and
# the A/B builds named in AB (abbuild/lib_<name>.so).   usage: [AB="v1 v2"] bash tools/gpu_r06_cellsweep.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u tools/cell_sweep.py 1e9 ${BPC:-0,64,128,256,1024} > $O/sweep.txt 2>&1 || exit 1
for v in $AB; do
  MOSAIC_HIP_LIB=$R/abbuild/lib_$v.so timeout -k 10 300 python3 -u tools/cell_sweep.py 1e9 ${BPC:-0,64,128,256,1024} > $O/sweep_$v.txt 2>&1 || exit 1
done
echo sweep done
