#!/bin/bash
# GPU box (round 6): the full GPU test suite, smoke, the bench line, and the bench under a rocprofv3
# kernel trace (stats) whose summary goes to profiles/.
#   usage: bash tools/gpu_r05_final.sh OUTNAME
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
echo tests done
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
echo smoke done
timeout -k 10 400 python3 -u bench.py > $O/bench.txt 2>&1 || exit 1
echo bench done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 -u $R/bench.py --pmc 0 > $O/bench_prof.txt 2>&1 || exit 1
echo prof done
