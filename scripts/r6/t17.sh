#!/bin/bash
# round 6: k_serialize_agg with its residency cut to 2 / 3 workgroups per CU (dynamic LDS), so the resident workgroups
# cover a sliding window of the result and finished ones are replaced (lib/exp/occ2.so, occ3.so), alternating with the
# in-tree library
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6
for i in 1 2; do
  timeout -k 10 120 python scripts/r6/step.py >> gpurun_out/r6/t17_steps.txt || exit 1
  RBG_LIB=$PWD/roaringbitmap_amd/lib/exp/occ2.so timeout -k 10 120 python scripts/r6/step.py >> gpurun_out/r6/t17_steps.txt || exit 1
  RBG_LIB=$PWD/roaringbitmap_amd/lib/exp/occ3.so timeout -k 10 120 python scripts/r6/step.py >> gpurun_out/r6/t17_steps.txt || exit 1
done
cat gpurun_out/r6/t17_steps.txt
