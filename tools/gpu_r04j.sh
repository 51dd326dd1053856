# GPU box: A/B of k_join_tiles variants on C4 1e6 (head: envelope raster, occupancy 4, rare paths as
# calls; v2: hexagon chip ranges; v4: ranges, paths inlined; v5: raster, paths inlined)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04j
mkdir -p $O
cd $R
for v in head v2 v4 v5; do
  lib=""
  [ "$v" != head ] && lib="$R/abbuild/lib_$v.so"
  MOSAIC_HIP_LIB=$lib timeout -k 10 300 python3 -u tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 5 > $O/$v.txt 2>&1 || exit 1
  echo "$v done"
done
