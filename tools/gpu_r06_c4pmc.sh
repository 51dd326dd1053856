#!/bin/bash
# GPU box (round 6): C4 on HEAD -- kbench_c4 at 1e6 and 5e6 buildings (tessellation, table build and
# join times), rocprofv3 kernel stats at 1e6, then one PMC pass per counter group at 1e6 and the
# WRITE_SIZE pass at 5e6 (k_join_tiles' spill stores).  Every GPU step under its own time limit.
#   usage: [AB="v1 v2"] bash tools/gpu_r06_c4pmc.sh OUTNAME   (AB: abbuild/lib_v1.so ... timed and WRITE_SIZE too)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 5 > $O/c4_1e6.txt 2>&1 || exit 1
timeout -k 10 400 python3 -u tools/kbench_c4.py --buildings 5e6 --n 2.5e8 --reps 3 > $O/c4_5e6.txt 2>&1 || exit 1
for v in $AB; do
  MOSAIC_HIP_LIB=$R/abbuild/lib_$v.so timeout -k 10 300 python3 -u tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 5 > $O/c4_1e6_$v.txt 2>&1 || exit 1
  MOSAIC_HIP_LIB=$R/abbuild/lib_$v.so timeout -k 10 400 python3 -u tools/kbench_c4.py --buildings 5e6 --n 2.5e8 --reps 3 > $O/c4_5e6_$v.txt 2>&1 || exit 1
done
echo kbench done
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u $R/tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 3 > $O/c4_prof.log 2>&1 || exit 1
i=0
for grp in "WRITE_SIZE" "FETCH_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 200 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/p$i -o run -- \
      python3 -u $R/tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 2 > $O/p$i.log 2>&1
  rc=$?
  echo "group $i ($grp) exit=$rc"
  if [ $rc -ne 0 ]; then tail -3 $O/p$i.log; exit 1; fi
done
timeout -k 10 -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/p5e6 -o run -- \
    python3 -u $R/tools/kbench_c4.py --buildings 5e6 --n 2.5e8 --reps 2 > $O/p5e6.log 2>&1 || exit 1
for v in $AB; do
  MOSAIC_HIP_LIB=$R/abbuild/lib_$v.so timeout -k 10 -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pw_$v -o run -- \
      python3 -u $R/tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 2 > $O/pw_$v.log 2>&1 || exit 1
done
echo pmc done
