#!/bin/bash
# SQ counter passes over per-family pairwise runs (one rocprofv3 process per pass).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmc_kinds
mkdir -p $OUT
for case in "A B and" "A B card" "R R and" "R R card" "B B and" "B B card" "M M and"; do
  set -- $case
  tag=$1$2_$3
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "k_pair" --output-format csv -d $OUT/$tag -o run -- python3 scripts/kind_one.py $1 $2 $3 3 > /dev/null 2> $OUT/$tag.err || { echo "$tag failed"; tail -5 $OUT/$tag.err; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --kernel-include-regex "k_pair" --output-format csv -d $OUT/${tag}_b -o run -- python3 scripts/kind_one.py $1 $2 $3 3 > /dev/null 2> $OUT/${tag}_b.err || { echo "$tag b failed"; tail -5 $OUT/${tag}_b.err; exit 1; }
  echo "$tag ok"
done
