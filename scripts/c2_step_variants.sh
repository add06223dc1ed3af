#!/bin/bash
# The C2 headline step alone (no C3-C5 extras, no CPU baseline) under the default library and
# each variant in $VARIANTS, the whole sequence twice (alternating runs on one box).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for v in base $VARIANTS; do
    if [ $v = base ]; then unset RBG_LIB; else export RBG_LIB=$PWD/roaringbitmap_amd/lib/variants/$v.so; fi
    timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --c3-n 0 --c4-pairs 0 --c5-rows 0 \
      > gpurun_out/c2step_${v}_$rep.json 2> gpurun_out/c2step_${v}_$rep.err || { echo "$v failed"; tail -5 gpurun_out/c2step_${v}_$rep.err; exit 1; }
    python3 - "$v" gpurun_out/c2step_${v}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); e = d["extra"]
print(f"{sys.argv[1]:10s} step {d['ms_per_step']:.4f} ev {e['gpu_event_ms_per_step']:.4f} phases {e['phase_ms']} "
      f"card {e['c2_and_cardinality']['roofline']['kernel_ms']} 2str {e.get('c2_and_two_streams', {}).get('ms_per_op')}")
PY
  done
done
