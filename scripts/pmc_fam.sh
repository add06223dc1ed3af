#!/bin/bash
# One SQ counter pass per "KA KB OP" case of the pairwise kernel (current build).
# Usage: scripts/pmc_fam.sh "A A and" "R R card" ...   (default: the AND family matrix)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmc_fam
mkdir -p $OUT
[ $# -eq 0 ] && set -- "A A and" "A B and" "A R and" "B B and" "B R and" "R R and" "M M and"
for c in "$@"; do
  read -r KA KB OPN <<< "$c"
  tag=$KA$KB$OPN
  timeout -k 10 -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "k_pair_wave" --output-format csv -d $OUT/$tag -o run -- python3 scripts/kind_one.py $KA $KB $OPN 3 > /dev/null 2> $OUT/$tag.err || { echo "$tag failed"; tail -5 $OUT/$tag.err; exit 1; }
  echo "$tag ok"
done
