#!/bin/bash
# CPU probe (not a test), VERDICT r4 "close f2": the kepler.ipynb cell-27 rings against the oracle's
# h3ToGeoBoundary with sin / cos / asin / atan / atan2 taken from the glibc restatement compiled
# with FMA contraction everywhere (an aarch64-style libm), alone (H3 in x87 / double steps) and
# combined with the H3-side contraction variants of run.sh (modes 5 / 6).  Also the same restatement
# without extra contraction (must reproduce the oracle: 23).  usage: bash tools/probes/kepler_ulp/run_fma.sh
set -e
here=$(cd "$(dirname "$0")" && pwd)
root=$(cd "$here/../../.." && pwd)
w=$(mktemp -d)
cp "$root/oracle/h3.c" "$root/oracle/oracle.h" "$w/"
(cd "$w" && patch -s -p1 < "$here/h3_variants.patch")
# g_cr bit 32: every libm call from the restatement object linked in
sed -i -e 's/static double Q_atan(double x) { return/static double Q_atan(double x) { if (g_cr \& 32) return lf_atan(x); return/' \
       -e 's/static double Q_atan2(double y, double x) { return/static double Q_atan2(double y, double x) { if (g_cr \& 32) return lf_atan2(y, x); return/' \
       -e 's/static double Q_sin(double x) { return/static double Q_sin(double x) { if (g_cr \& 32) return lf_sin(x); return/' \
       -e 's/static double Q_cos(double x) { return/static double Q_cos(double x) { if (g_cr \& 32) return lf_cos(x); return/' \
       -e 's/static double Q_asin(double x) { return/static double Q_asin(double x) { if (g_cr \& 32) return lf_asin(x); return/' \
       -e 's/^int g_cr = 0/double lf_sin(double), lf_cos(double), lf_asin(double), lf_atan(double), lf_atan2(double, double);\nint g_cr = 0/' "$w/h3.c"
grep -q "lf_atan2(y, x)" "$w/h3.c"
for v in contract nocontract; do
  flags="-O2 -mfma -ffp-contract=fast"; [ $v = nocontract ] && flags="-O2 -ffp-contract=off"
  g++ $flags -std=c++17 -c -o "$w/libm_$v.o" "$here/libm_fma.cpp"
  gcc -O2 -ffp-contract=off -I "$root/oracle" -o "$w/drv_$v" "$here/drv.c" "$w/h3.c" "$w/libm_$v.o" -lquadmath -lm -lstdc++
done
python3 "$here/sweep_fma.py" "$w" "$root/tests/golden/notebook_vectors.json"
rm -rf "$w"
