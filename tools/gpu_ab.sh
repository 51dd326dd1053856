# GPU box: A/B of stream-kernel builds with tools/kbench.py (C2 uniform and C3 clustered, 1e9 points).
#   usage: bash tools/gpu_ab.sh OUTDIR VARIANT...   (VARIANT: "head" = the in-tree library, else abbuild/lib_VARIANT.so)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
shift
mkdir -p $O
cd $R
i=0
for v in "$@"; do
  i=$((i+1))
  lib=""
  [ "$v" != head ] && lib=$R/abbuild/lib_$v.so
  MOSAIC_HIP_LIB=$lib timeout -k 10 240 python -u tools/kbench.py --reps 10 > $O/ab_c2_${v}_$i.txt 2>&1 || exit 1
  [ -n "$AB_C2_ONLY" ] && continue
  MOSAIC_HIP_LIB=$lib timeout -k 10 240 python -u tools/kbench.py --reps 10 --clustered --res 10 > $O/ab_c3_${v}_$i.txt 2>&1 || exit 1
done
for f in $O/ab_*.txt; do echo "## $f"; grep stream_ms $f; done
