#!/bin/bash
# round 5 (v): k_bsi_reg unit-pool group size (4 / 8 / 16 workgroups) and the static striding, C5 step
# (bench.py --only c5), alternating
set -e
mkdir -p gpurun_out
V=roaringbitmap_amd/lib/variants
for r in 1 2 3; do
  for lib in bsistatic bsig4 bsig8 bsig16; do
    RBG_LIB=$V/$lib.so timeout -k 10 150 python -u bench.py --only c5 --steps 60 --warmup 5 2>/dev/null | sed "s/^/$lib /" | cut -c1-220 >> gpurun_out/r5v_c5.txt
  done
done
