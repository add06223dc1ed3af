#!/bin/bash
# kind_matrix under each experimental library variant (VARIANTS="a b ...")
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in base $VARIANTS; do
  if [ $v = base ]; then unset RBG_LIB; else export RBG_LIB=$PWD/roaringbitmap_amd/lib/variants/$v.so; fi
  timeout -k 10 200 python scripts/kind_matrix.py > gpurun_out/km_$v.txt 2>&1 || { echo "$v failed"; tail gpurun_out/km_$v.txt; exit 1; }
  echo "== $v"; grep -v in_MB gpurun_out/km_$v.txt | grep -v amdgpu.ids | tr '\n' ' ' ; echo
done
