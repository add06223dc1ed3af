#!/bin/bash
# BSI parity (heap, buffer, full size), then every compare op timed at 10^9 rows
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bsi.py tests/test_gpu_bsi_buffer.py tests/test_gpu_inplace.py tests/test_gpu_fullsize.py -k "bsi or c5 or BSI or merge" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/bsi_tests.log 2>&1
rc=$?; tail -2 gpurun_out/bsi_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bsi_time.py 1000000000 3 > gpurun_out/bsi_time.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/bsi_time.log
