#!/bin/bash
# round 6: the driver's bench command (--steps 20 --warmup 5) with and without the device settle before the warmups
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6
for s in 0 0.25 0 0.25; do
  RBG_BENCH_SETTLE_S=$s timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --c3-n 0 --c4-pairs 0 --c5-rows 0 --no-cpu-baseline > gpurun_out/r6/t12_$s.json 2> gpurun_out/r6/t12_$s.err || { echo "bench failed"; tail gpurun_out/r6/t12_$s.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r6/t12_$s.json')); e=d['extra']; print('settle $s', d['value'], d['ms_per_step'], d['roofline']['frac'], e['timed_phase_ms'], json.dumps(e.get('phase_ms')))" | tee -a gpurun_out/r6/t12.txt
done
