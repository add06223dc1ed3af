#!/bin/bash
# round 6 timing probe: the filter path without its LDS compaction (lib/exp/nocompact.so, wrong results -- timing only)
# against the in-tree library, per array family and on the C2 mix
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6
for i in 1 2; do
  timeout -k 10 150 python scripts/r6/fam.py mix,AA,AB,AR >> gpurun_out/r6/t15_fam.txt || exit 1
  RBG_LIB=$PWD/roaringbitmap_amd/lib/exp/nocompact.so timeout -k 10 150 python scripts/r6/fam.py mix,AA,AB,AR >> gpurun_out/r6/t15_fam.txt || exit 1
done
cat gpurun_out/r6/t15_fam.txt
