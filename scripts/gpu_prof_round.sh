#!/bin/bash
# One gpurun call: BSI + full-size parity, then the rocprofv3 passes of scripts/profile.sh (tag $1).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bsi.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/prof_tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -3 gpurun_out/prof_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/profile.sh ${1:-r03} "${2:-kt ktw pmc sq}"
