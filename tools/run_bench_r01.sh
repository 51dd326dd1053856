# Round-1 bench + profile on the GPU box: full bench line (PMC traffic pass + CPU baseline), then a
# rocprofv3 kernel-trace --stats run of the same bench for the per-kernel summary in profiles/.
# Each GPU step has its own time limit; a failing step ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2> gpurun_out/bench_full.err || { echo bench_exit=$?; exit 1; }
tail -1 gpurun_out/bench_full.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r01 -o bench -- python $R/bench.py --steps 5 --warmup 2 --cpu-sample 0 --pmc 0 > $R/gpurun_out/prof_r01.log 2>&1 || { echo prof_exit=$?; exit 1; }
echo prof_ok
