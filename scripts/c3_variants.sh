#!/bin/bash
# C3 wide-OR lines of bench.py under each library variant (VARIANTS="a b ..."), the sequence twice
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
for v in base $VARIANTS; do
  if [ $v = base ]; then unset RBG_LIB; else export RBG_LIB=$PWD/roaringbitmap_amd/lib/variants/$v.so; fi
  timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --c5-rows 0 --c4-pairs 0 > gpurun_out/c3v_$v.json 2> gpurun_out/c3v_$v.err || { echo "$v failed"; tail -3 gpurun_out/c3v_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/c3v_$v.json').read().strip().splitlines()[-1]); e=d['extra']
print('$v', d['value'], [(k, e[k]['input_GBps'], e[k]['roofline_rank0']['frac']) for k in ('c3_uniform_or','c3_clustered_or')])"
done
done
