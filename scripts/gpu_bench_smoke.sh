set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 5 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
echo "bench exit=$?"
cat gpurun_out/bench1.json
tail -5 gpurun_out/bench1.err
