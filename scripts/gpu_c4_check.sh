#!/bin/bash
# batched andCardinality parity (incl. full-size C4), then the bench under base / variants
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_fullsize.py -k "batch or c4 or pair" \
  -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c4_tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -5 gpurun_out/c4_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash scripts/gpu_bench_variants.sh || exit 1
