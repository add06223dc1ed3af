#!/bin/bash
# round 6, R AND R windows: parity tests of the new path, then per-family times against HEAD's library (alternating)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_gpu_pairwise.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6/t1_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r6/t1_tests.log; exit 1; }
tail -3 gpurun_out/r6/t1_tests.log
for i in 1 2; do
  RBG_LIB=$PWD/roaringbitmap_amd/lib/exp/head.so timeout -k 10 120 python scripts/r6/fam.py >> gpurun_out/r6/t1_fam.txt || exit 1
  timeout -k 10 120 python scripts/r6/fam.py >> gpurun_out/r6/t1_fam.txt || exit 1
done
cat gpurun_out/r6/t1_fam.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r6/t1_bench.json 2> gpurun_out/r6/t1_bench.err || { echo "bench failed"; tail gpurun_out/r6/t1_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6/t1_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], json.dumps(d['extra'].get('phase_ms')), d['extra']['result']['sha16'])"
