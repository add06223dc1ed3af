#!/bin/bash
# round 6: the fused-serialization tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_gpu_pairwise.py -m gpu -x -v --timeout 200 --timeout-method thread -k "fused or tile_sums or many_tiles" > gpurun_out/r6/t16_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r6/t16_tests.log; exit 1; }
tail -5 gpurun_out/r6/t16_tests.log
