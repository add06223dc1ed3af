#!/bin/bash
# orNot kernel timings per workload (scripts/ornot_perf.py) under rocprofv3 --kernel-trace --stats
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/ornot_modes
mkdir -p $OUT
for M in mixed empty bitmaps; do
  N=8192
  [ "$M" = empty ] && N=65536
  [ -n "$ORN_N" ] && [ "$M" != empty ] && N=$ORN_N
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$M -o run -- python3 scripts/ornot_perf.py $N 20 $M > $OUT/$M.txt 2>&1 || { echo "$M failed"; tail $OUT/$M.txt; exit 1; }
  grep "mode=" $OUT/$M.txt
  python3 - "$OUT/$M/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "ornot" in r["Name"] or "serialize" in r["Name"] or "k_place" in r["Name"]:
        print("  ", r["Name"][:40], r["Calls"], r["AverageNs"])
PY
done
