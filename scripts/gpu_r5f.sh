#!/bin/bash
# round 5 (f): buffer pairwise ops on the GPU, the paths they touch, and a runOptimize kernel trace
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_buffer_pairwise.py tests/test_gpu_pairwise.py tests/test_gpu_bsi_buffer.py tests/test_gpu_inplace.py \
  > gpurun_out/r5f_tests.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5f_ro -o ro -- python3 bench.py --only runopt --steps 10 --warmup 3 > gpurun_out/r5f_ro.txt 2>&1
