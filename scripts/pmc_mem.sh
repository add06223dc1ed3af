#!/bin/bash
# Memory-path counters of the pairwise kernel (TLB, TA/TCP stalls, L2 hit/miss,
# DRAM credit stalls) per "KA KB OP" case, one rocprofv3 pass per counter group.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmc_mem
mkdir -p $OUT
[ $# -eq 0 ] && set -- "M M and" "M M card" "B B and"
G1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_PENDING_STALL_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES"
G2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum"
G3="TCC_EA0_WRREQ_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
for c in "$@"; do
  read -r KA KB OPN <<< "$c"
  tag=$KA$KB$OPN
  g=0
  for G in "$G1" "$G2" "$G3"; do
    g=$((g+1))
    timeout -k 10 -s KILL 90 rocprofv3 --pmc $G --kernel-include-regex "k_pair_wave" --output-format csv -d $OUT/${tag}_g$g -o run -- python3 scripts/kind_one.py $KA $KB $OPN 3 > /dev/null 2> $OUT/${tag}_g$g.err || { echo "$tag g$g failed"; tail -5 $OUT/${tag}_g$g.err; exit 1; }
  done
  echo "$tag ok"
done
