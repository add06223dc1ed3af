#!/bin/bash
# round 6 validation of the final tree: the whole GPU suite, smoke(), the default bench line and the driver's command
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r6/t13_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r6/t13_tests.log; exit 1; }
tail -1 gpurun_out/r6/t13_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/t13_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r6/t13_smoke.log; exit 1; }
tail -1 gpurun_out/r6/t13_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r6/t13_bench.json 2> gpurun_out/r6/t13_bench.err || { echo "bench failed"; tail gpurun_out/r6/t13_bench.err; exit 1; }
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6/t13_driver.json 2> gpurun_out/r6/t13_driver.err || { echo "bench failed"; tail gpurun_out/r6/t13_driver.err; exit 1; }
for f in bench driver; do python3 -c "import json; d=json.load(open('gpurun_out/r6/t13_$f.json')); e=d['extra']; print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], json.dumps(e.get('phase_ms')), e['c5_bsi_range_sum']['ms_per_step'], e['c3_uniform_or']['ms_per_step'])"; done
