#!/bin/bash
# LDS bank-conflict / occupancy / VALU counters of the hot kernels as they run now (round 6):
# k_pair_cu per container-family case "KA KB OP" (scripts/kind_one.py, 65,536-key operands of one family
# each; M = the C2 mix) and k_wide<OR> on C3 uniform (bench.py --only c3u).  One rocprofv3 pass each,
# the program directly after "--".  Summarised by scripts/pmc_lds_summary.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/r6/pmc_lds}
mkdir -p $OUT
CTRS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"
[ $# -eq 0 ] && set -- "A A and" "A B and" "A R and" "B B and" "B R and" "R R and" "M M and" "M M card"
for c in "$@"; do
  read -r KA KB OPN <<< "$c"
  tag=$KA$KB$OPN
  timeout -k 10 -s KILL 90 rocprofv3 --pmc $CTRS --kernel-trace --kernel-include-regex "k_pair_cu" --output-format csv -d $OUT/$tag -o run -- python3 scripts/kind_one.py $KA $KB $OPN 3 > /dev/null 2> $OUT/$tag.err || { echo "$tag failed"; tail -5 $OUT/$tag.err; exit 1; }
  echo "$tag ok"
done
timeout -k 10 -s KILL 150 rocprofv3 --pmc $CTRS --kernel-trace --kernel-include-regex "k_wide" --output-format csv -d $OUT/C3Uor -o run -- python3 bench.py --only c3u --steps 3 --warmup 1 > /dev/null 2> $OUT/C3Uor.err || { echo "c3u failed"; tail -5 $OUT/C3Uor.err; exit 1; }
echo "C3Uor ok"
