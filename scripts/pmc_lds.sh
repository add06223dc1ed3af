#!/bin/bash
# LDS bank-conflict / occupancy / VALU counters of the pairwise kernel per
# container-family case "KA KB OP" (one rocprofv3 pass each).  Summarised by
# scripts/pmc_lds_summary.py into profiles/<round>/pmc_families.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc_lds}
mkdir -p $OUT
[ $# -eq 0 ] && set -- "A A and" "A B and" "A R and" "B B and" "B R and" "R R and" "M M and" "M M card" "A A or" "A R or" "M M or" "M M xor" "M M andnot"
for c in "$@"; do
  read -r KA KB OPN <<< "$c"
  tag=$KA$KB$OPN
  timeout -k 10 -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --kernel-include-regex "k_pair_wave" --output-format csv -d $OUT/$tag -o run -- python3 scripts/kind_one.py $KA $KB $OPN 3 > /dev/null 2> $OUT/$tag.err || { echo "$tag failed"; tail -5 $OUT/$tag.err; exit 1; }
  echo "$tag ok"
done
