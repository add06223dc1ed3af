#!/bin/bash
# C2 AND / andCardinality under the default library and each variant in $VARIANTS
# (bench.py with only the headline workload), alternating on one box.  A variant is a library
# (roaringbitmap_amd/lib/variants/NAME.so) or NAME:VAR=VALUE (the default library, env setting).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
for v in base $VARIANTS; do
  # a variant is a library (lib/variants/NAME.so) or NAME:VAR=VALUE (the default library under an env setting)
  unset RBG_LIB; ENVV=""
  if [[ $v == *:* ]]; then ENVV=${v#*:}; v=${v%%:*}; elif [ $v != base ]; then export RBG_LIB=$PWD/roaringbitmap_amd/lib/variants/$v.so; fi
  env $ENVV timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --c3-n 0 --c4-pairs 0 --c5-rows 0 \
    > gpurun_out/c2_$v.json 2> gpurun_out/c2_$v.err || { echo "$v failed"; tail -5 gpurun_out/c2_$v.err; exit 1; }
  python3 - "$v" gpurun_out/c2_$v.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); e = d["extra"]
print(sys.argv[1], "step", d["ms_per_step"], "phases", e["phase_ms"], "card", e["c2_and_cardinality"]["roofline"]["kernel_ms"],
      "card_step", e["c2_and_cardinality"]["ms_per_step"], "sha", e["result"].get("sha16"), flush=True)
PY
done
done
