#!/bin/bash
# GPU box (round 6): the GPU test suite (optionally a subset: TESTS=...), then a default bench run.
#   usage: bash tools/gpu_r06_suite.sh OUTNAME
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
echo tests done
if [ -z "$NOBENCH" ]; then
timeout -k 10 400 python3 -u bench.py > $O/bench.txt 2>&1 || exit 1
echo bench done
fi
