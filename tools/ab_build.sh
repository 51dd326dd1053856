#!/bin/bash
# A/B measurement builds of the stream kernels (not the product): libmosaic_hip.so variants whose
# join_stream.hip is compiled with extra -D flags, in abbuild/, selected at run time with
# MOSAIC_HIP_LIB.  usage: tools/ab_build.sh NAME "-DFOO=1 -DBAR=2"
set -e
cd "$(dirname "$0")/../mosaic_amd/csrc"
make -s ../libmosaic_hip.so >/dev/null
mkdir -p ../../abbuild
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-function \
    -Wno-unused-variable -munsafe-fp-atomics $2 -c -o ../../abbuild/$1.o join_stream.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../abbuild/lib_$1.so mosaic_hip.o ../../abbuild/$1.o \
    polyfill.o tessellate.o tiles_build.o chip_arrays.o
rm -f ../../abbuild/$1.o
