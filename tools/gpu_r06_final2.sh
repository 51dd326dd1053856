#!/bin/bash
# GPU box (round 6, last run): the full GPU test suite, smoke, the bench line, the bench under a
# rocprofv3 kernel trace (stats), then C3 (clustered, res 10) on the same code.
#   usage: bash tools/gpu_r06_final2.sh OUTNAME
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
echo tests done
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
echo smoke done
timeout -k 10 300 python3 -u bench.py > $O/bench.txt 2>&1 || exit 1
echo bench done
(cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 -u $R/bench.py --pmc 0 > $O/bench_prof.txt 2>&1) || exit 1
echo prof done
timeout -k 10 200 python3 -u tools/kbench.py --reps 10 --clustered --res 10 > $O/c3.txt 2>&1 || exit 1
echo c3 done
timeout -k 10 200 python3 -u tools/kbench_bng.py --reps 5 > $O/c5.txt 2>&1 || exit 1
echo c5 done
timeout -k 10 300 python3 -u tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 5 > $O/c4_1e6.txt 2>&1 || exit 1
timeout -k 10 400 python3 -u tools/kbench_c4.py --buildings 5e6 --n 2.5e8 --reps 3 > $O/c4_5e6.txt 2>&1 || exit 1
echo c4 done
