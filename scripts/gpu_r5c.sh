#!/bin/bash
# round 5 (c): the balanced task order of the pairwise kernels -- parity (pairwise, full size, shards,
# in-place), the key-order / balanced timing on one box, the per-wave probe of both forms
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_pairwise.py \
  tests/test_gpu_fullsize.py tests/test_gpu_shard.py tests/test_gpu_inplace.py > gpurun_out/r5c_t.log 2>&1
timeout -k 10 300 python -u scripts/c2_balance.py > gpurun_out/r5c_bal.txt 2>&1
RBG_LIB=roaringbitmap_amd/lib/variants/probe.so RBG_PW_BALANCE=1 timeout -k 10 100 python -u scripts/xcd_probe.py \
  > gpurun_out/r5c_xcd.txt 2>&1
