#!/bin/bash
# The working tree's engine with a patch applied (an experiment), built into roaringbitmap_amd/lib/exp/NAME.so
# for alternating runs against the default library (RBG_LIB=...); the working tree is untouched.
#   scripts/r6/build_patched.sh NAME PATCH
set -e
NAME=$1; PATCH=$(cd "$(dirname "$2")" && pwd)/$(basename "$2")
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
T=$(mktemp -d)
mkdir -p $T/roaringbitmap_amd $T/include
cp -r $ROOT/roaringbitmap_amd/csrc $T/roaringbitmap_amd/ && cp $ROOT/include/*.h $T/include/
(cd $T && patch -p1 -s < $PATCH)
C=$T/roaringbitmap_amd/csrc
OUT=$ROOT/roaringbitmap_amd/lib/exp/$NAME
mkdir -p $OUT
for s in $(cd $C && ls *.hip); do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -x hip -c $C/$s -o $OUT/$s.o &
done
for s in engine.cpp format.cpp; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -c $C/$s -o $OUT/$s.o &
done
for j in $(jobs -p); do wait $j || { echo "compile failed"; exit 1; }; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $OUT.so $OUT/*.o -lpthread
rm -rf $OUT $T
echo $OUT.so
