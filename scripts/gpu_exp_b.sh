#!/bin/bash
# One gpurun call: the BSI parity tests under the packed-count-row build (its results must be
# the default build's), then C5 and the C2 step under the experiment builds, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
RBG_LIB=$PWD/roaringbitmap_amd/lib/variants/bsipack.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bsi.py \
  -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/bsipack_tests.log 2>&1
rc=$?; tail -3 gpurun_out/bsipack_tests.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="bsipack" bash scripts/c5_variants.sh || exit 1
VARIANTS="ser2" bash scripts/c2_variants.sh || exit 1
