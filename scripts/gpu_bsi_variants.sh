#!/bin/bash
# One gpurun call: BSI / C5 parity (default library), then C5 under the default library and each
# variant in $VARIANTS, twice, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bsi.py tests/test_gpu_fullsize.py tests/test_gpu_shard.py \
  -k "bsi or c5 or same_device" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/bsi_tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -3 gpurun_out/bsi_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/c5_variants.sh && bash scripts/c5_variants.sh
