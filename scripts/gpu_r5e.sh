#!/bin/bash
# round 5 (e): the whole GPU suite and smoke() on the current tree
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r5e_tests.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5e_smoke.log 2>&1
