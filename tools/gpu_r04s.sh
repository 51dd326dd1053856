# GPU box: round-4 profile set -- the bench (line + kernel stats), C4 1e6 PMC (k_join_tiles,
# k_bin_cover), C4 5e6 kbench + kernel stats, C3 kbench + PMC (k_join_stream_cpt)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04s
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $O/bench.txt 2>&1 || exit 1
echo bench done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bench -o bench -- python3 -u $R/bench.py --steps 20 --warmup 5 --pmc 0 --cpu-sample 0 > $O/bench_prof.txt 2>&1 || exit 1
find /tmp/prof_bench -name "*kernel_stats.csv" -exec cp {} $O/bench_kernel_stats.csv \;
echo bench prof done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_c4b -o c4 -- python3 -u $R/tools/kbench_c4.py --buildings 5e6 --n 2.5e8 --reps 3 > $O/c4_5e6.txt 2>&1 || exit 1
find /tmp/prof_c4b -name "*kernel_stats.csv" -exec cp {} $O/stats_c4_5e6.csv \;
echo c4 5e6 done
cd $R
KB=tools/kbench_c4.py timeout -k 10 600 bash tools/pmc_pipe.sh gpurun_out/r04s/pmc_c4 --buildings 1e6 --n 2.5e8 > $O/pmc_c4.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/r04s/pmc_c4 k_bin_cover > $O/pmc_c4/summary_bin_cover.json || exit 1
rm -rf $O/pmc_c4/p*/
echo c4 pmc done
timeout -k 10 300 python3 -u tools/kbench.py --res 10 --clustered --reps 10 > $O/kbench_c3.txt 2>&1 || exit 1
timeout -k 10 600 bash tools/pmc_pipe.sh gpurun_out/r04s/pmc_c3 --res 10 --clustered > $O/pmc_c3.log 2>&1 || exit 1
rm -rf $O/pmc_c3/p*/
echo c3 done
