#!/bin/bash
# Per-XCD dynamic claiming (RBG_DYN build) against the default build, both in the planned form
# (RBG_PAIRWISE_PLAN=1; the claim counters are zeroed by the plan kernel), and the default direct
# form: C2 parity of the dyn build first, then the C2 step / family times, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
DYN=$PWD/roaringbitmap_amd/lib/variants/dyn.so
RBG_PAIRWISE_PLAN=1 RBG_LIB=$DYN timeout -k 10 400 python -u -m pytest tests/test_gpu_pairwise.py tests/test_gpu_fullsize.py \
  -k "pairwise or c2 or mode or random or dense" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/dyn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/dyn_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in direct plan dyn; do
    unset RBG_LIB RBG_PAIRWISE_PLAN
    [ $v != direct ] && export RBG_PAIRWISE_PLAN=1
    [ $v = dyn ] && export RBG_LIB=$DYN
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --c3-n 0 --c4-pairs 0 --c5-rows 0 \
      > gpurun_out/dyn_$v.json 2> gpurun_out/dyn_$v.err || { echo "$v failed"; tail -5 gpurun_out/dyn_$v.err; exit 1; }
    python3 - "$v" gpurun_out/dyn_$v.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); e = d["extra"]
print(sys.argv[1], "step", d["ms_per_step"], "phases", e["phase_ms"], "card", e["c2_and_cardinality"]["roofline"]["kernel_ms"],
      "sha", e["result"].get("sha16"), flush=True)
PY
  done
done
for v in plan dyn; do
  unset RBG_LIB; export RBG_PAIRWISE_PLAN=1
  [ $v = dyn ] && export RBG_LIB=$DYN
  timeout -k 10 200 python scripts/kind_matrix.py > gpurun_out/km_dyn_$v.txt 2>&1 || { echo "km $v failed"; exit 1; }
  echo "== $v"; grep -v in_MB gpurun_out/km_dyn_$v.txt | grep -v amdgpu.ids | tr '\n' ' '; echo
done
