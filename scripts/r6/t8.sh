#!/bin/bash
# round 6 validation after the last kernel change: the whole GPU suite, smoke(), one default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r6/t8_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r6/t8_tests.log; exit 1; }
tail -2 gpurun_out/r6/t8_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/t8_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r6/t8_smoke.log; exit 1; }
tail -1 gpurun_out/r6/t8_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r6/t8_bench.json 2> gpurun_out/r6/t8_bench.err || { echo "bench failed"; tail gpurun_out/r6/t8_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6/t8_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], json.dumps(d['extra'].get('phase_ms')))"
