#!/bin/bash
# GPU box (round 5): C5 FETCH_SIZE / WRITE_SIZE per launch of k_join_stream_bng_cpt with the round-5
# BNG tables, and with the cell-frame / group-line / wedge options off (build options) for contrast.
#   usage: bash tools/gpu_r05_pmc_c5.sh OUTNAME
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE; do
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_new_$c -o run -- \
      python3 -u $R/tools/kbench_bng.py --reps 2 --n 5e8 > $O/pmc_new_$c.log 2>&1 || exit 1
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_off_$c -o run -- \
      python3 -u $R/tools/kbench_bng.py --reps 2 --n 5e8 --build-opts bng_group_lines=0,bng_wedges=0 > $O/pmc_off_$c.log 2>&1 || exit 1
  echo "$c done"
done
