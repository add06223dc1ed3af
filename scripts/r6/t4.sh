#!/bin/bash
# round 6: the whole GPU suite, smoke(), then the N = 2 headline rehearsed on one GPU (two ranks, gloo:
# the strong step with its gather to rank 0)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6/t4_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r6/t4_tests.log; exit 1; }
tail -3 gpurun_out/r6/t4_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6/t4_smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/r6/t4_smoke.log; exit 1; }
tail -1 gpurun_out/r6/t4_smoke.log
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --backend gloo --c3-n 400 --c4-pairs 100000 --c5-rows 100000000 > gpurun_out/r6/t4_mp2.json 2> gpurun_out/r6/t4_mp2.err || { echo "mp bench failed"; tail -20 gpurun_out/r6/t4_mp2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6/t4_mp2.json')); print(d['value'], d['ms_per_step'], d['n_gpus'], json.dumps(d['extra'].get('c2_strong')))"
timeout -k 10 120 ./scripts/r6/bb_ceiling > gpurun_out/r6/bb_ceiling.txt 2>&1 || { echo "bb_ceiling failed"; cat gpurun_out/r6/bb_ceiling.txt; exit 1; }
cat gpurun_out/r6/bb_ceiling.txt
