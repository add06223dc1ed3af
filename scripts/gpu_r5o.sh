#!/bin/bash
# round 5 (o): whole GPU suite + smoke on the current tree, then the default bench line and its kernel trace
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r5o_tests.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5o_smoke.log 2>&1
timeout -k 10 600 python -u bench.py > gpurun_out/r5o_bench.json 2> gpurun_out/r5o_bench.err
