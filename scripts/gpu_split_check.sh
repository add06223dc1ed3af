#!/bin/bash
# pairwise parity (incl. the two-window R AND R path) + full-size C2, then base vs variants
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pairwise.py tests/test_gpu_fullsize.py -k "not c3 and not c4 and not c5" \
  -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/split_tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -15 gpurun_out/split_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash scripts/gpu_bench_variants.sh || exit 1
timeout -k 10 900 bash scripts/variant_kinds.sh || exit 1
