#!/bin/bash
# C2 AND / andCardinality under the default library and each variant in $VARIANTS
# (bench.py with only the headline workload), alternating on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
for v in base $VARIANTS; do
  if [ $v = base ]; then unset RBG_LIB; else export RBG_LIB=$PWD/roaringbitmap_amd/lib/variants/$v.so; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --c3-n 0 --c4-pairs 0 --c5-rows 0 \
    > gpurun_out/c2_$v.json 2> gpurun_out/c2_$v.err || { echo "$v failed"; tail -5 gpurun_out/c2_$v.err; exit 1; }
  python3 - "$v" gpurun_out/c2_$v.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); e = d["extra"]
print(sys.argv[1], "step", d["ms_per_step"], "phases", e["phase_ms"], "card", e["c2_and_cardinality"]["roofline"]["kernel_ms"], flush=True)
PY
done
done
