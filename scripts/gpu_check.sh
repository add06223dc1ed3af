#!/bin/bash
# One gpurun call for a kernel change: a pytest selection (arg 1, default the pairwise
# parity + full-size C2), then the bench restricted to the headline (C2) and its
# cardinality leg; each step under its own time limit, stopping at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
SEL=${1:-"tests/test_gpu_pairwise.py tests/test_gpu_fullsize.py"}
KSEL=${2:-"not c3 and not c4 and not c5"}
timeout -k 10 500 python -u -m pytest $SEL -k "$KSEL" -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/check_tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -15 gpurun_out/check_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --c3-n 0 --c4-pairs 0 --c5-rows 0 \
  > gpurun_out/check_bench.json 2> gpurun_out/check_bench.err
rc=$?; echo "bench exit=$rc"; cat gpurun_out/check_bench.json; tail -5 gpurun_out/check_bench.err
exit $rc
