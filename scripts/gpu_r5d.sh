#!/bin/bash
# round 5 (d): issue-priority variants of the pairwise kernel (RBG_PRIO_TIER), alternating on one box, and the
# per-wave probe under variant 1
set -e
mkdir -p gpurun_out
V=roaringbitmap_amd/lib/variants
for r in 1 2; do
  for lib in "" $V/prio1.so $V/prio2.so $V/prio3.so; do
    RBG_LIB=$lib timeout -k 10 120 python -u scripts/c2_kern.py >> gpurun_out/r5d_prio.txt 2>&1
  done
done
RBG_LIB=$V/probe1.so timeout -k 10 100 python -u scripts/xcd_probe.py > gpurun_out/r5d_xcd.txt 2>&1
