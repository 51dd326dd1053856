#!/bin/bash
# GPU box: C4 A/B of the in-tree library against abbuild/lib_old.so -- 5e6 buildings x 2.5e8 points
# timing, then one WRITE_SIZE and one FETCH_SIZE rocprofv3 pass per library at 1e6 buildings.
#   usage: bash tools/gpu_c4_ab.sh OUTNAME
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u tools/kbench_c4.py --buildings 5e6 --n 2.5e8 --reps 3 > $O/c4_5e6_new.txt 2>&1 || exit 1
MOSAIC_HIP_LIB=$R/abbuild/lib_old.so timeout -k 10 400 python3 -u tools/kbench_c4.py --buildings 5e6 --n 2.5e8 --reps 3 > $O/c4_5e6_old.txt 2>&1 || exit 1
export TMPDIR=/tmp; cd /tmp
for v in new old; do
  for c in WRITE_SIZE FETCH_SIZE; do
    if [ $v = old ]; then export MOSAIC_HIP_LIB=$R/abbuild/lib_old.so; else unset MOSAIC_HIP_LIB; fi
    timeout -k 10 -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_${v}_$c -o run -- \
        python3 -u $R/tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 2 > $O/pmc_${v}_$c.log 2>&1 || exit 1
    echo "$v $c done"
  done
done
cd $R
for k in 1 2; do
  timeout -k 10 120 python3 -u tools/build_var.py > $O/build_var_p$k.txt 2>&1 || exit 1
done
timeout -k 10 120 python3 -u tools/build_var.py --sleep 0.5 > $O/build_var_sleep.txt 2>&1 || exit 1
echo build_var done
