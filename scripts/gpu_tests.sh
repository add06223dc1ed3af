#!/bin/bash
# One GPU call: the given pytest selection (default: every gpu test), one process, each test
# bounded by pytest-timeout, the whole run by timeout(1).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
SEL=${1:-tests}
timeout -k 10 ${2:-900} python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests exit=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -40
exit $rc
