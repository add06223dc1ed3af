#!/bin/bash
# N=1 bench line, then a 2-rank rehearsal on the one GPU over gloo.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err
rc=$?; echo "bench N=1 exit=$rc"; cat gpurun_out/bench1.json; tail -3 gpurun_out/bench1.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --no-cpu-baseline > gpurun_out/bench2.json 2> gpurun_out/bench2.err
rc=$?; echo "bench N=2 (gloo rehearsal) exit=$rc"; cat gpurun_out/bench2.json; tail -3 gpurun_out/bench2.err; exit $rc
