#!/bin/bash
# GPU parity tests (pairwise only unless ALL=1) + per-family timing + bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TESTS:-tests/test_gpu_pairwise.py}
timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q_tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -15 gpurun_out/q_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/kind_matrix.py > gpurun_out/kind_matrix.txt 2>&1
rc=$?; cat gpurun_out/kind_matrix.txt | grep -v in_MB; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err
rc=$?; cat gpurun_out/q_bench.json; tail -3 gpurun_out/q_bench.err; exit $rc
