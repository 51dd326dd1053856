set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2> gpurun_out/bench_full.err
echo bench_exit=$?
tail -1 gpurun_out/bench_full.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r01 -o bench -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --cpu-sample 0 --pmc 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_r01.log 2>&1
echo prof_exit=$?
