#!/bin/bash
# C4 alone under the default library and each variant in $VARIANTS (the sequence twice)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
for v in base $VARIANTS; do
  if [ $v = base ]; then unset RBG_LIB; else export RBG_LIB=$PWD/roaringbitmap_amd/lib/variants/$v.so; fi
  timeout -k 10 200 python bench.py --only c4 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/c4_$v.json 2> gpurun_out/c4_$v.err || { echo "$v failed"; tail -5 gpurun_out/c4_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['pairs_per_s'])" gpurun_out/c4_$v.json $v
done
done
