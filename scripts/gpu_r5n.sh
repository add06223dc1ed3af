#!/bin/bash
# round 5 (n): k_pair_cu with the last RBG_CU_TAIL bands in shared per-XCD pools: parity of the variants,
# then alternating timings (tail 0 / 1 / 2 / 4)
set -e
mkdir -p gpurun_out
V=roaringbitmap_amd/lib/variants
for t in 1 4; do
  RBG_LIB=$V/cutail$t.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_pairwise.py tests/test_gpu_fullsize.py -k "task_orders or c2_full" > gpurun_out/r5n_tests_$t.log 2>&1
done
for r in 1 2 3; do
  for t in 0 1 2 4; do
    RBG_PW_CU=1 RBG_LIB=$V/cutail$t.so timeout -k 10 120 python -u scripts/c2_kern.py | grep balance=1 | sed "s/^/tail=$t /" >> gpurun_out/r5n_tail.txt 2>&1
  done
done
