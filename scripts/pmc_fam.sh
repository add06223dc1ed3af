#!/bin/bash
# One SQ counter pass per family pair of the pairwise AND (current build).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmc_fam
mkdir -p $OUT
for case in ${CASES:-"A A" "A B" "A R" "B B" "B R" "R R" "M M"}; do
  set -- $case
  tag=$1$2
  timeout -k 10 -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "k_pair_wave" --output-format csv -d $OUT/$tag -o run -- python3 scripts/kind_one.py $1 $2 and 3 > /dev/null 2> $OUT/$tag.err || { echo "$tag failed"; tail -5 $OUT/$tag.err; exit 1; }
  echo "$tag ok"
done
