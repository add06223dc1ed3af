#!/bin/bash
# round 5 (y): k_pair_cu with per-wave chunk claims from per-XCD pools (RBG_CU_GLOBAL chunk 1 / 2 / 4) vs the
# per-CU LDS pool: parity of the variants, then alternating timings
set -e
mkdir -p gpurun_out
V=roaringbitmap_amd/lib/variants
for c in 1 4; do
  RBG_LIB=$V/cug$c.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_pairwise.py tests/test_gpu_fullsize.py -k "task_orders or c2_full" > gpurun_out/r5y_tests_$c.log 2>&1
done
for r in 1 2 3; do
  for c in 0 1 2 4; do
    RBG_LIB=$V/cug$c.so timeout -k 10 120 python -u scripts/c2_kern.py | grep balance=1 | sed "s/^/chunk=$c /" >> gpurun_out/r5y_cug.txt 2>&1
  done
done
