# GPU box: C4 1e6 tile-join counting probes (s1 survivors, s2 f64 fallbacks, s3 no f64 fallback
# (timing), s4 survivors on global-geometry chips) and PMC passes of the head library
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04m
mkdir -p $O
cd $R
for v in s1 s2 s3 s4; do
  MOSAIC_HIP_LIB=$R/abbuild/lib_$v.so timeout -k 10 300 python3 -u tools/kbench_c4.py --buildings 1e6 --n 2.5e8 --reps 3 > $O/c4_$v.txt 2>&1 || exit 1
  echo "$v done"
done
KB=tools/kbench_c4.py bash tools/pmc_pipe.sh gpurun_out/r04m/pmc --buildings 1e6 --n 2.5e8 > $O/pmc.log 2>&1 || exit 1
echo pmc done
