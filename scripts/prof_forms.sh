#!/bin/bash
# kernel traces (rocprofv3 --kernel-trace --stats) of the BSI compare forms and the wide aggregation forms
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bsi -o run -- python3 $R/scripts/bsi_time.py 1000000000 3 > $R/gpurun_out/prof_bsi.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_agg -o run -- python3 $R/scripts/agg_time.py 1 200 3 > $R/gpurun_out/prof_agg.log 2>&1 || exit 1
find $R/gpurun_out/prof_bsi $R/gpurun_out/prof_agg -name "*kernel_stats.csv"
