#!/bin/bash
# aggregation parity, then scripts/agg_time.py on clustered (raw and runOptimize'd) and uniform batches
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_aggregations.py tests/test_gpu_wide.py tests/test_gpu_bsi_buffer.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/agg_tests.log 2>&1
rc=$?; tail -2 gpurun_out/agg_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/agg_time.py 2 1000 3 > gpurun_out/agg_c.log 2>&1 || exit 1
timeout -k 10 200 python scripts/agg_time.py 2 1000 2 "" ro > gpurun_out/agg_c_ro.log 2>&1 || exit 1
timeout -k 10 250 python scripts/agg_time.py 1 200 3 > gpurun_out/agg_u.log 2>&1 || exit 1
grep -h -v amdgpu gpurun_out/agg_c.log gpurun_out/agg_c_ro.log gpurun_out/agg_u.log
