#!/bin/bash
# GPU parity tests (pairwise, wide, batch), then the per-family timing matrix.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/kind_matrix.py > gpurun_out/km_cur.txt 2>&1 || { echo "km failed"; tail gpurun_out/km_cur.txt; exit 1; }
grep -v in_MB gpurun_out/km_cur.txt | grep -v amdgpu.ids | tr '\n' ' '; echo
