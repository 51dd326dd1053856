#!/bin/bash
# SQ instruction / cycle counters of the stream kernel (kbench, 1e9 uniform points, res 9): one
# rocprofv3 --pmc pass per counter group (<= 8 SQ counters each), each under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc_sq
export TMPDIR=/tmp
pass() {  # pass NAME COUNTERS...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_sq/$name -o run -- \
      python3 -u tools/kbench.py --n 1e9 --reps 2 > gpurun_out/pmc_sq/$name.log 2>&1
  local rc=$?
  tail -3 gpurun_out/pmc_sq/$name.log
  if [ $rc -ne 0 ]; then echo "PASS $name FAILED rc=$rc"; exit $rc; fi
}
pass inst SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES
pass act SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT
