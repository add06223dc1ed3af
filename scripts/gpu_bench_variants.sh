#!/bin/bash
# bench.py (no CPU baseline) under the default library and each variant in $VARIANTS
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in base $VARIANTS; do
  if [ $v = base ]; then unset RBG_LIB; else export RBG_LIB=$PWD/roaringbitmap_amd/lib/variants/$v.so; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err || { echo "$v failed"; tail -5 gpurun_out/bench_$v.err; exit 1; }
  python3 - "$v" gpurun_out/bench_$v.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); e = d["extra"]
print(sys.argv[1], "AND ms", e["phase_ms"]["compute"], "card", e["c2_and_cardinality"]["roofline"]["kernel_ms"],
      "C3u", e["c3_uniform_or"]["roofline_rank0"]["kernel_ms"], "C3c", e["c3_clustered_or"]["roofline_rank0"]["kernel_ms"],
      "C3uand", e["c3_uniform_and"]["ms_per_step"], "C4", e["c4_batch_and_card"]["ms_per_step"], "C5", e["c5_bsi_range_sum"]["ms_per_step"],
      "ro", e["run_optimize_c2"]["ms_per_call"])
PY
done
