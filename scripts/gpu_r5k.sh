#!/bin/bash
# round 5 (k): the CU-pooled pairwise kernel (k_pair_cu, RBG_PW_CU=1): parity, then alternating timings
set -e
mkdir -p gpurun_out
RBG_PW_CU=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_pairwise.py tests/test_gpu_fullsize.py -k "pairwise or c2 or dense or random or mode" > gpurun_out/r5k_tests.log 2>&1
V=roaringbitmap_amd/lib/variants
for r in 1 2 3; do
  RBG_PW_CU=0 RBG_LIB=$V/cuorder0.so timeout -k 10 120 python -u scripts/c2_kern.py | sed 's/^/cu=0 /' >> gpurun_out/r5k_cu.txt 2>&1
  RBG_PW_CU=1 RBG_LIB=$V/cuorder0.so timeout -k 10 120 python -u scripts/c2_kern.py | sed 's/^/cu=1 /' >> gpurun_out/r5k_cu.txt 2>&1
  RBG_PW_CU=1 RBG_LIB=$V/cuorder1.so timeout -k 10 120 python -u scripts/c2_kern.py | sed 's/^/cu=1 /' >> gpurun_out/r5k_cu.txt 2>&1
done
