#!/bin/bash
# Build an experimental variant of the engine library with extra compile flags:
#   scripts/build_variant.sh NAME "-DRBG_EXP_X=1"  ->  roaringbitmap_amd/lib/variants/NAME.so
# (load it with RBG_LIB=... ; the default library is untouched)
set -e
NAME=$1; FLAGS="$2 -DRBG_PROFILING_BUILD=1"
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/roaringbitmap_amd/csrc
OUT=$ROOT/roaringbitmap_amd/lib/variants/$NAME
mkdir -p $OUT
for s in $(cd $C && ls *.hip); do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $FLAGS -x hip -c $C/$s -o $OUT/$s.o &
done
for s in engine.cpp format.cpp; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $FLAGS -c $C/$s -o $OUT/$s.o &
done
for j in $(jobs -p); do wait $j || { echo "compile failed"; exit 1; }; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $OUT.so $OUT/*.o -lpthread
rm -rf $OUT
echo $OUT.so
