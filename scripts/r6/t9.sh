#!/bin/bash
# round 6: array AND / ANDNOT run variants -- pairwise parity first, then per-family and C2-mix compute time against the previous library (lib/exp/head.so)
# pairwise parity first, then per-family and C2-mix compute time against the previous library (lib/exp/head.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest tests/test_gpu_pairwise.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6/t9_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r6/t9_tests.log; exit 1; }
tail -2 gpurun_out/r6/t9_tests.log
for i in 1 2 3; do
  RBG_LIB=$PWD/roaringbitmap_amd/lib/exp/head.so timeout -k 10 120 python scripts/r6/fam.py mix,AA,AB,AR >> gpurun_out/r6/t9_fam.txt || exit 1
  timeout -k 10 120 python scripts/r6/fam.py mix,AA,AB,AR >> gpurun_out/r6/t9_fam.txt || exit 1
done
cat gpurun_out/r6/t9_fam.txt
for i in 1 2; do
  RBG_LIB=$PWD/roaringbitmap_amd/lib/exp/head.so timeout -k 10 120 python scripts/r6/step.py >> gpurun_out/r6/t9_steps.txt || exit 1
  timeout -k 10 120 python scripts/r6/step.py >> gpurun_out/r6/t9_steps.txt || exit 1
done
cat gpurun_out/r6/t9_steps.txt
