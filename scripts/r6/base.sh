#!/bin/bash
# round-6 baseline: default bench line + kernel trace of the C2 step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r6/bench_base.json 2> gpurun_out/r6/bench_base.err || { echo "bench failed"; tail gpurun_out/r6/bench_base.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6/bench_base.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], json.dumps(d['extra'].get('phase_ms')))"
