# GPU box: GPU tests (minus the full-size configs), smoke, bench, rocprof kernel stats of the bench,
# then the full-size config tests; every GPU step under its own time limit, stop at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-verify}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "not full_size" > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || exit 1
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --pmc 0 --cpu-sample 0 > $O/bench_prof.log 2>&1 || exit 1
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -v -s --timeout 500 --timeout-method thread -k "full_size" > $O/full_size.log 2>&1
