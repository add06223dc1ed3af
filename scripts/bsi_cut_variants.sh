#!/bin/bash
# BSI compare (no sum) timings under the default library and the cut variants, alternating twice
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
for v in base $VARIANTS; do
  if [ $v = base ]; then unset RBG_LIB; else export RBG_LIB=$PWD/roaringbitmap_amd/lib/variants/$v.so; fi
  timeout -k 10 200 python scripts/bsi_time.py 1000000000 3 > gpurun_out/bsi_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/bsi_$v.log; exit 1; }
  echo "$v $(grep -h '"op"' gpurun_out/bsi_$v.log | python3 -c 'import sys,json; print([ (d["op"], d["heap_ms"]) for d in map(json.loads, sys.stdin)])')"
done
done
