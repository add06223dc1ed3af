#!/bin/bash
# BSI parity (incl. the full-size C5 check), then the bench under base / variants
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bsi.py tests/test_gpu_fullsize.py -k "bsi or c5 or BSI" \
  -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/bsi_tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -5 gpurun_out/bsi_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash scripts/gpu_bench_variants.sh || exit 1
