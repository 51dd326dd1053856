#!/bin/bash
# A/B measurement builds (not the product): libmosaic_hip.so variants with one translation unit
# compiled with extra -D flags, in abbuild/, selected at run time with MOSAIC_HIP_LIB.
# usage: tools/ab_build.sh NAME SOURCE.hip "-DFOO=1 -DBAR=2"   (SOURCE: join_stream.hip, join_binned.hip)
# The variant must be the in-tree source (its headers are then the same files every other object was
# built from): a source from another checkout with its own headers links objects with different struct
# layouts -- round 5's illegal-address fault (gpurun_out/r05h); mosaic_init also refuses such a library
# (mosaic_layout_* fingerprints, join_binned.h).
set -e
cd "$(dirname "$0")/../mosaic_amd/csrc"
case "$2" in */*) echo "ab_build.sh: SOURCE must be a file of mosaic_amd/csrc, not $2" >&2; exit 2;; esac
[ -f "$2" ] || { echo "ab_build.sh: no $2 in mosaic_amd/csrc" >&2; exit 2; }
make -s ../libmosaic_hip.so >/dev/null
mkdir -p ../../abbuild
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-function \
    -Wno-unused-variable -munsafe-fp-atomics $3 -c -o ../../abbuild/$1.o $2
objs=""
for o in $(sed -n 's/^OBJS = //p' Makefile); do
  [ "$o" = "${2%.hip}.o" ] && objs="$objs ../../abbuild/$1.o" || objs="$objs $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../abbuild/lib_$1.so $objs
rm -f ../../abbuild/$1.o
