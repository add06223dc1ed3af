#!/bin/bash
# round 6: the serializer's output stores plain instead of nontemporal (scripts/r6/ser_plain_store.patch ->
# lib/exp/serplain.so; scripts/r6/copy_ceiling.hip: plain stores copy at 6.65 TB/s, nontemporal at 6.1) against the
# in-tree library, alternating on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6
for i in 1 2 3; do
  timeout -k 10 120 python scripts/r6/step.py >> gpurun_out/r6/t10_steps.txt || exit 1
  RBG_LIB=$PWD/roaringbitmap_amd/lib/exp/serplain.so timeout -k 10 120 python scripts/r6/step.py >> gpurun_out/r6/t10_steps.txt || exit 1
done
cat gpurun_out/r6/t10_steps.txt
