#!/bin/bash
# One gpurun call: parity of the 512-record placement tiles (RBG_KTILE512), the C2 step under it,
# then the XCD-weighted static shares against the planned form.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
RBG_LIB=$PWD/roaringbitmap_amd/lib/variants/kt512.so timeout -k 10 400 python -u -m pytest tests/test_gpu_pairwise.py \
  tests/test_gpu_wide.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/kt512_tests.log 2>&1
rc=$?; tail -2 gpurun_out/kt512_tests.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="kt512" bash scripts/c2_variants.sh || exit 1
bash scripts/gpu_xw_check.sh || exit 1
