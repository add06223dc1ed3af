#!/bin/bash
# BSI parity under the variant library $VARIANT, then C5 alternating base / variant
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
RBG_LIB=$PWD/roaringbitmap_amd/lib/variants/$VARIANT.so timeout -k 10 400 python -u -m pytest tests/test_gpu_bsi.py \
  -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/bsi_variant_tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -3 gpurun_out/bsi_variant_tests.log
[ $rc -eq 0 ] || exit $rc
VARIANTS=$VARIANT timeout -k 10 600 bash scripts/c5_variants.sh
