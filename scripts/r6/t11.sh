#!/bin/bash
# round 6: the driver's bench command (--steps 20 --warmup 5) beside the default (200 / 10) on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6/t11_driver.json 2> gpurun_out/r6/t11_driver.err || { echo "bench failed"; tail gpurun_out/r6/t11_driver.err; exit 1; }
timeout -k 10 500 python bench.py > gpurun_out/r6/t11_default.json 2> gpurun_out/r6/t11_default.err || { echo "bench failed"; tail gpurun_out/r6/t11_default.err; exit 1; }
for f in driver default; do python3 -c "import json; d=json.load(open('gpurun_out/r6/t11_$f.json')); e=d['extra']; print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], json.dumps(e.get('phase_ms')), e['c5_bsi_range_sum']['ms_per_step'], e['c3_uniform_or']['ms_per_step'])"; done
