#!/bin/bash
# round 5 (aa): whole GPU suite + smoke on the current tree, C5 kernel trace, then the default bench line
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r5aa_tests.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5aa_smoke.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5aa_c5 -o c5 -- python3 bench.py --only c5 --steps 20 --warmup 3 > gpurun_out/r5aa_c5.txt 2>&1
timeout -k 10 900 python -u bench.py > gpurun_out/r5aa_bench.json 2> gpurun_out/r5aa_bench.err
