#!/bin/bash
# Instruction-cache counters of the pairwise kernel, per "KA KB OP" case (one pass each).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmc_icache
mkdir -p $OUT
[ $# -eq 0 ] && set -- "M M and" "M M card" "M M or" "R R and" "B B and"
for c in "$@"; do
  read -r KA KB OPN <<< "$c"
  tag=$KA$KB$OPN
  timeout -k 10 -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_INSTS_VALU --kernel-include-regex "k_pair_wave" --output-format csv -d $OUT/$tag -o run -- python3 scripts/kind_one.py $KA $KB $OPN 3 > /dev/null 2> $OUT/$tag.err || { echo "$tag failed"; tail -5 $OUT/$tag.err; exit 1; }
  echo "$tag ok"
done
