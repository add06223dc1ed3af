#!/bin/bash
# priorityqueue parity, then kernel traces of scripts/pq_time.py on uniform and clustered batches
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_aggregations.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/agg_tests.log 2>&1
rc=$?; tail -2 gpurun_out/agg_tests.log; [ $rc -eq 0 ] || exit $rc
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/pqprof_u -o pq -- python $R/scripts/pq_time.py 1 200 1 > $R/gpurun_out/pqprof_u.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/pqprof_c -o pq -- python $R/scripts/pq_time.py 2 1000 1 > $R/gpurun_out/pqprof_c.log 2>&1 || exit 1
