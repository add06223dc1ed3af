#!/bin/bash
# round 5 (g): runOptimize with the run flags off the totals' cache line: tests + kernel trace
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_runopt.py \
  > gpurun_out/r5g_tests.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5g_ro -o ro -- python3 bench.py --only runopt --steps 10 --warmup 3 > gpurun_out/r5g_ro.txt 2>&1
