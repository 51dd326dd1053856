#!/bin/bash
# GPU box (round 6): C4 A/B -- tests/test_binned.py on the GPU, kbench_c4 at 1e6 and 5e6 buildings and a
# WRITE_SIZE pass at 1e6 for the product library and each AB build (abbuild/lib_<name>.so).
#   usage: [AB="v1 v2"] bash tools/gpu_r06_c4ab.sh OUTNAME
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_binned.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo tests done
run() {  # run TAG [lib]
  local tag=$1 lib=$2
  MOSAIC_HIP_LIB=$lib timeout -k 10 300 python3 -u tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 5 > $O/c4_1e6_$tag.txt 2>&1 || exit 1
  MOSAIC_HIP_LIB=$lib timeout -k 10 400 python3 -u tools/kbench_c4.py --buildings 5e6 --n 2.5e8 --reps 3 > $O/c4_5e6_$tag.txt 2>&1 || exit 1
  (cd /tmp && MOSAIC_HIP_LIB=$lib TMPDIR=/tmp timeout -k 10 -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pw_$tag -o run -- \
      python3 -u $R/tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 2 > $O/pw_$tag.log 2>&1) || exit 1
  echo "$tag done"
}
run product ""
for v in $AB; do run $v $R/abbuild/lib_$v.so; done
echo all done
