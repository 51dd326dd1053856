# GPU box: the compacted stream kernel on C3 (24 coordinate bits per pending row): C2 / C3 tests,
# C3 and C2 kbench with stream_pipe 1 vs 2
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04u
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread "tests/test_gpu_configs.py::test_c3_all_zones_res10_vs_oracle" "tests/test_gpu_configs.py::test_c3_full_size_clustered_res10" "tests/test_gpu_configs.py::test_c2_full_size_raster_vs_generic_vs_oracle" > $O/tests.log 2>&1 || exit 1
echo tests done
timeout -k 10 300 python3 -u tools/kbench.py --res 10 --clustered --reps 10 --sweep stream_pipe=1 stream_pipe=2 > $O/kbench_c3.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/kbench.py --reps 10 --sweep stream_pipe=1 stream_pipe=2 > $O/kbench_c2.txt 2>&1 || exit 1
echo kbench done
