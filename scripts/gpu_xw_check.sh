#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
XW=$PWD/roaringbitmap_amd/lib/variants/xw.so
export RBG_PAIRWISE_PLAN=1
for rep in 1 2; do
  for v in plan xw; do
    unset RBG_LIB
    [ $v = xw ] && export RBG_LIB=$XW
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --c3-n 0 --c4-pairs 0 --c5-rows 0 \
      > gpurun_out/xw_$v.json 2> gpurun_out/xw_$v.err || { echo "$v failed"; tail -5 gpurun_out/xw_$v.err; exit 1; }
    python3 - "$v" gpurun_out/xw_$v.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); e = d["extra"]
print(sys.argv[1], "step", d["ms_per_step"], "phases", e["phase_ms"], "card", e["c2_and_cardinality"]["roofline"]["kernel_ms"],
      "sha", e["result"].get("sha16"), flush=True)
PY
  done
done
