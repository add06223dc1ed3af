#!/bin/bash
# One gpurun call: the full GPU suite, then C5 under $C5_VARIANTS and C2 under $C2_VARIANTS
# (each alternating with the default library, twice).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$C5_VARIANTS" ]; then VARIANTS="$C5_VARIANTS" bash scripts/c5_variants.sh && VARIANTS="$C5_VARIANTS" bash scripts/c5_variants.sh || exit 1; fi
if [ -n "$C2_VARIANTS" ]; then VARIANTS="$C2_VARIANTS" bash scripts/c2_variants.sh || exit 1; fi
