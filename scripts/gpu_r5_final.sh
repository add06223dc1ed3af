#!/bin/bash
# round-5 validation: the whole GPU suite, smoke(), then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_full.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests_full.log; exit 1; }
tail -3 gpurun_out/gpu_tests_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench_latest.json 2> gpurun_out/bench_latest.err || { echo "bench failed"; tail gpurun_out/bench_latest.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_latest.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['extra'].get('ornot_c2'))"
