#!/bin/bash
# Build the engine library of a git revision (default HEAD) into roaringbitmap_amd/lib/exp/NAME.so, for
# alternating-run comparisons on one box (load with RBG_LIB=...); the working tree's library is untouched.
set -e
NAME=${1:-head}; REV=${2:-HEAD}
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
T=$(mktemp -d)
git -C $ROOT archive $REV roaringbitmap_amd/csrc include | tar -x -C $T
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
