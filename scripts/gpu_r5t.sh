#!/bin/bash
# round 5 (t): k_bsi_reg issue priority by dispatch tier (RBG_BSI_TIER 0 / 1 / 2), probe builds, alternating
set -e
mkdir -p gpurun_out
V=roaringbitmap_amd/lib/variants
for r in 1 2; do
  for lib in probe probe_t1 probe_t2; do
    RBG_LIB=$V/$lib.so timeout -k 10 150 python -u scripts/bsi_probe.py 2>&1 | grep -v amdgpu.ids | head -3 >> gpurun_out/r5t_bsi.txt
  done
done
