#!/bin/bash
# A/B measurement builds (not the product): libmosaic_hip.so variants with one translation unit
# compiled with extra -D flags, in abbuild/, selected at run time with MOSAIC_HIP_LIB.
# usage: tools/ab_build.sh NAME SOURCE.hip "-DFOO=1 -DBAR=2"   (SOURCE: join_stream.hip, join_binned.hip)
set -e
cd "$(dirname "$0")/../mosaic_amd/csrc"
make -s ../libmosaic_hip.so >/dev/null
mkdir -p ../../abbuild
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-function \
    -Wno-unused-variable -munsafe-fp-atomics $3 -c -o ../../abbuild/$1.o $2
objs=""
for o in mosaic_hip.o join_stream.o join_binned.o polyfill.o tessellate.o tiles_build.o chip_arrays.o; do
  [ "$o" = "${2%.hip}.o" ] && objs="$objs ../../abbuild/$1.o" || objs="$objs $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../abbuild/lib_$1.so $objs
rm -f ../../abbuild/$1.o
