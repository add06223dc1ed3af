#!/bin/bash
# round 6: the N = 2 headline rehearsed on one GPU after the device settle was added (two ranks, gloo)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --backend gloo --c3-n 400 --c4-pairs 100000 --c5-rows 100000000 > gpurun_out/r6/t14_mp2.out 2> gpurun_out/r6/t14_mp2.err || { echo "mp bench failed"; tail -20 gpurun_out/r6/t14_mp2.err; exit 1; }
grep '^{"metric' gpurun_out/r6/t14_mp2.out > gpurun_out/r6/t14_mp2.json
python3 -c "import json; d=json.load(open('gpurun_out/r6/t14_mp2.json')); e=d['extra']; print(d['n_gpus'], d['value'], d['ms_per_step'], d['scaling'], json.dumps(e['c2_strong'])[:400])"
