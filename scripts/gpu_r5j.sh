#!/bin/bash
# round 5 (j): order of the cost bands in the balanced pairwise walk (RBG_BAL_WALK 0 / 1 / 2), alternating on one box
set -e
mkdir -p gpurun_out
V=roaringbitmap_amd/lib/variants
for r in 1 2 3; do
  for lib in $V/walk0.so $V/walk1.so $V/walk2.so; do
    RBG_LIB=$lib timeout -k 10 120 python -u scripts/c2_kern.py >> gpurun_out/r5j_walk.txt 2>&1
  done
done
