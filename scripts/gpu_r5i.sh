#!/bin/bash
# round 5 (i): runOptimize as one kernel (input layout kept, lazy statistics); suites that use the scan or runOptimize
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_runopt.py \
  tests/test_gpu_decode.py tests/test_gpu_bsi.py tests/test_gpu_range.py tests/test_gpu_aggregations.py > gpurun_out/r5i_tests.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5i_ro -o ro -- python3 bench.py --only runopt --steps 10 --warmup 3 > gpurun_out/r5i_ro.txt 2>&1
