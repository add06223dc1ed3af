#!/bin/bash
# round 6 experiment: nontemporal stores of k_pair_cu's bitmap results (scripts/r6/nt_bstore.patch) against the
# in-tree library, alternating on one box: the C2 step, its compute and serialization, and parity of the variant
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6
for i in 1 2 3; do
  timeout -k 10 120 python scripts/r6/step.py >> gpurun_out/r6/t6_steps.txt || exit 1
  RBG_LIB=$PWD/roaringbitmap_amd/lib/exp/ntb.so timeout -k 10 120 python scripts/r6/step.py >> gpurun_out/r6/t6_steps.txt || exit 1
done
cat gpurun_out/r6/t6_steps.txt
for i in 1 2 3; do
  RBG_LIB=$PWD/roaringbitmap_amd/lib/exp/cu8.so timeout -k 10 120 python scripts/r6/step.py >> gpurun_out/r6/t6_steps.txt || exit 1
  timeout -k 10 120 python scripts/r6/step.py >> gpurun_out/r6/t6_steps.txt || exit 1
done
tail -6 gpurun_out/r6/t6_steps.txt
RBG_LIB=$PWD/roaringbitmap_amd/lib/exp/cu8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q -k "c2_full_pair or key_ranges" --timeout 200 --timeout-method thread > gpurun_out/r6/t6_cu8_tests.log 2>&1; tail -2 gpurun_out/r6/t6_cu8_tests.log
