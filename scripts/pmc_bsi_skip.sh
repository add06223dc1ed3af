#!/bin/bash
# FETCH_SIZE of k_bsi_reg: compare(LE) without sum (low slices read only where EQ survives) vs with sum
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for mode in 0 1; do
  timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_bsi_reg" --output-format csv -d $R/gpurun_out/pmc_bsi_sum$mode -o run -- python3 $R/scripts/bsi_one.py 1000000000 LE $mode 3 > /dev/null 2> $R/gpurun_out/pmc_bsi_sum$mode.err || { echo "pass $mode failed"; tail -3 $R/gpurun_out/pmc_bsi_sum$mode.err; exit 1; }
done
find $R/gpurun_out/pmc_bsi_sum0 $R/gpurun_out/pmc_bsi_sum1 -name "*counter_collection.csv"
