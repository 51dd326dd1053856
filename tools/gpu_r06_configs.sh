#!/bin/bash
# GPU box (round 6): the other configs on the round's final code -- C3 (clustered, res 10) and C2
# (kbench), C5 (kbench_bng), C4 at 1e6 and 5e6 buildings (kbench_c4), kernel (a) alone (cell_sweep);
# each under its own time limit.    usage: bash tools/gpu_r06_configs.sh OUTNAME
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 240 python3 -u tools/kbench.py --reps 10 > $O/c2.txt 2>&1 || exit 1
timeout -k 10 240 python3 -u tools/kbench.py --reps 10 --clustered --res 10 > $O/c3.txt 2>&1 || exit 1
timeout -k 10 240 python3 -u tools/kbench_bng.py --reps 5 > $O/c5.txt 2>&1 || exit 1
echo c2 c3 c5 done
timeout -k 10 300 python3 -u tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 5 > $O/c4_1e6.txt 2>&1 || exit 1
timeout -k 10 400 python3 -u tools/kbench_c4.py --buildings 5e6 --n 2.5e8 --reps 3 > $O/c4_5e6.txt 2>&1 || exit 1
echo c4 done
timeout -k 10 200 python3 -u tools/cell_sweep.py 1e9 256 > $O/cell.txt 2>&1 || exit 1
echo configs done
