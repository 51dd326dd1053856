# GPU box: the full GPU test suite, smoke, the bench, and kernel (a) (k_cell_h3, grid_longlatascellid)
# in isolation: kernel stats and PMC passes on 1e9 resident points (tools/cellrun.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-round_end}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
echo tests done
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
echo smoke done
timeout -k 10 400 python3 -u bench.py > $O/bench.txt 2>&1 || exit 1
echo bench done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_cell -o cell -- python3 -u $R/tools/cellrun.py 1e9 > $O/cell_prof.txt 2>&1 || exit 1
find /tmp/prof_cell -name "*kernel_stats.csv" -exec cp {} $O/cell_kernel_stats.csv \;
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d /tmp/pmc_cell_$i -o run -- python3 -u $R/tools/cellrun.py 1e9 > $O/cell_pmc_$i.log 2>&1 || exit 1
  find /tmp/pmc_cell_$i -name "*counter_collection.csv" -exec cp {} $O/cell_pmc_$i.csv \;
done
echo cell done
