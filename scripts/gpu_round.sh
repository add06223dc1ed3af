#!/bin/bash
# One GPU call: gpu parity tests (optionally a selection), then a bench line (each step with its own time limit).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
SEL=${1:-tests}
timeout -k 10 800 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench exit=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
exit $rc
