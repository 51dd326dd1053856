#!/bin/bash
# GPU box: a round's check-and-measure call.  Steps (each one quoted word "kind|args", each under its
# own time limit; the call stops at the first failure):
#   tests|<pytest args>   run|<python script + args>   prof|<script + args> (rocprofv3 kernel stats)
#   pmc|<counters>@<script + args> (one rocprofv3 counter pass)
# usage: bash tools/gpu_round.sh OUTNAME STEP...
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
shift
mkdir -p $O
cd $R
export TMPDIR=/tmp
i=0
for st in "$@"; do
  i=$((i+1))
  kind=${st%%|*}
  args=${st#*|}
  case $kind in
    tests) timeout -k 10 900 python3 -u -m pytest $args -m gpu -x -v --timeout 300 --timeout-method thread > $O/s$i.tests.log 2>&1 ;;
    run) timeout -k 10 600 python3 -u $args > $O/s$i.run.txt 2>&1 ;;
    prof) (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s$i.prof -o run -- python3 -u $R/$args > $O/s$i.prof.log 2>&1) ;;
    pmc) grp=${args%%@*}; cmd=${args#*@}
         (cd /tmp && timeout -k 10 -s KILL 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/s$i.pmc -o run -- python3 -u $R/$cmd > $O/s$i.pmc.log 2>&1) ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
  rc=$?
  echo "step $i ($kind) exit=$rc"
  if [ $rc -ne 0 ]; then tail -5 $O/s$i.* 2>/dev/null; exit 1; fi
done
