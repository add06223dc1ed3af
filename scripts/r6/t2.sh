#!/bin/bash
# round 6: k_pair_cu shared tail pools -- parity (pairwise + fullsize), then the C2 kernel against round 5's library
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest tests/test_gpu_pairwise.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6/t2_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r6/t2_tests.log; exit 1; }
tail -3 gpurun_out/r6/t2_tests.log
for i in 1 2 3; do
  RBG_LIB=$PWD/roaringbitmap_amd/lib/exp/head.so timeout -k 10 120 python scripts/r6/fam.py mix,RR,BB >> gpurun_out/r6/t2_fam.txt || exit 1
  timeout -k 10 120 python scripts/r6/fam.py mix,RR,BB >> gpurun_out/r6/t2_fam.txt || exit 1
done
cat gpurun_out/r6/t2_fam.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --c3-n 0 --c4-pairs 0 --c5-rows 0 > gpurun_out/r6/t2_bench.json 2> gpurun_out/r6/t2_bench.err || { echo "bench failed"; tail gpurun_out/r6/t2_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6/t2_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], json.dumps(d['extra'].get('phase_ms')), d['extra']['result']['sha16'])"
