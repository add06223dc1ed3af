#!/bin/bash
# round 5 (m): claim order inside k_pair_cu (RBG_CU_ORDER 0 vs 2) and the per-wave walk, alternating on one box
set -e
mkdir -p gpurun_out
V=roaringbitmap_amd/lib/variants
for r in 1 2 3; do
  RBG_PW_CU=0 RBG_LIB=$V/cuorder0.so timeout -k 10 120 python -u scripts/c2_kern.py | sed 's/^/cu=0 /' >> gpurun_out/r5m_cu.txt 2>&1
  RBG_PW_CU=1 RBG_LIB=$V/cuorder0.so timeout -k 10 120 python -u scripts/c2_kern.py | sed 's/^/cu=1 /' >> gpurun_out/r5m_cu.txt 2>&1
  RBG_PW_CU=1 RBG_LIB=$V/cuorder2.so timeout -k 10 120 python -u scripts/c2_kern.py | sed 's/^/cu=1 /' >> gpurun_out/r5m_cu.txt 2>&1
done
