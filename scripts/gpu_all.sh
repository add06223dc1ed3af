#!/bin/bash
# Full GPU suite + smoke (what the driver runs at round end).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/all_tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -5 gpurun_out/all_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke exit=$rc"; tail -3 gpurun_out/smoke.log; exit $rc
