#!/bin/bash
# CPU probe (not a test): the kepler.ipynb cell-27 boundary rings (tests/golden/notebook_vectors.json)
# against variants of the oracle's h3ToGeoBoundary -- x87 excess precision through the r chain,
# double-only constants, binary128 long double with and without FMA contraction (aarch64 builds),
# correctly rounded atan / atan2 / sin / cos / asin in every combination (libquadmath), +-1 ulp
# on r, atan(r) and the azimuth, and the JDK degree conversions.  Prints exact-ring counts per
# variant (the oracle's own arithmetic: 23 of 47).  usage: bash tools/probes/kepler_ulp/run.sh
set -e
here=$(cd "$(dirname "$0")" && pwd)
root=$(cd "$here/../../.." && pwd)
w=$(mktemp -d)
cp "$root/oracle/h3.c" "$root/oracle/oracle.h" "$w/"
(cd "$w" && patch -s -p1 < "$here/h3_variants.patch")
gcc -O2 -ffp-contract=off -I "$root/oracle" -o "$w/drv" "$here/drv.c" "$w/h3.c" -lquadmath -lm
python3 "$here/sweep.py" "$w/drv" "$root/tests/golden/notebook_vectors.json"
rm -rf "$w"
