#!/bin/bash
# round 5 (r): pooled serializer (k_serialize_pool, RBG_SER_POOL=1): parity on the serializing suites, then
# alternating C2 timings
set -e
mkdir -p gpurun_out
RBG_SER_POOL=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_pairwise.py tests/test_gpu_fullsize.py tests/test_gpu_wide.py tests/test_gpu_inplace.py > gpurun_out/r5r_tests.log 2>&1
for r in 1 2 3; do
  for p in 0 1; do
    RBG_SER_POOL=$p timeout -k 10 120 python -u scripts/c2_kern.py | grep balance=1 | sed "s/^/pool=$p /" >> gpurun_out/r5r_ser.txt 2>&1
  done
done
