# GPU box: the bench as the box's first GPU command (context-entry warm-up: build_s on a fresh box),
# a second bench, then ABI / binned tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04z
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u bench.py > $O/bench1.txt 2>&1 || exit 1
echo bench1 done
timeout -k 10 400 python3 -u bench.py --pmc 0 > $O/bench2.txt 2>&1 || exit 1
echo bench2 done
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_abi.py tests/test_binned.py tests/test_gpu_threads.py > $O/tests.log 2>&1 || exit 1
echo tests done
