set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard_mp.py -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/mp.log 2>&1
rc=$?; tail -2 gpurun_out/mp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; tail -c 300 gpurun_out/bench.json; exit $rc
