#!/bin/bash
# round 6: new-path parity (packed decode, workAndMemoryShyAnd, BSI target, pairwise cleanup), the full
# default bench line, then the LDS / occupancy counter passes of the current hot kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_wide.py tests/test_gpu_bsi.py tests/test_gpu_pairwise.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6/t3_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r6/t3_tests.log; exit 1; }
tail -3 gpurun_out/r6/t3_tests.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r6/t3_bench.json 2> gpurun_out/r6/t3_bench.err || { echo "bench failed"; tail gpurun_out/r6/t3_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6/t3_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], json.dumps(d['extra'].get('phase_ms'))); print(json.dumps(d['extra'].get('c3_uniform_or_decoded'))); print(json.dumps(d['extra'].get('rank_slice_ms'))[:1500])"
bash scripts/r6/pmc_lds_cu.sh && python3 scripts/pmc_lds_summary.py gpurun_out/r6/pmc_lds gpurun_out/r6/pmc_lds.json
