#!/bin/bash
# round 5: parity of the changed paths, then the pipelined C2 step, workShyAnd, C5, runOptimize timings and
# the production-speed XCD probe (each step under its own time limit; the first failure ends the call)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fullsize.py \
  tests/test_gpu_wide.py tests/test_gpu_bsi.py tests/test_gpu_runopt.py tests/test_gpu_range.py > gpurun_out/r5_t2.log 2>&1
timeout -k 10 300 python -u scripts/c2_pipe.py > gpurun_out/r5_pipe.txt 2>&1
timeout -k 10 120 python -u bench.py --only c3u_and --steps 20 --warmup 3 > gpurun_out/r5_shy.txt 2>&1
timeout -k 10 200 python -u bench.py --only c5 --steps 20 --warmup 3 > gpurun_out/r5_c5.txt 2>&1
timeout -k 10 200 python -u bench.py --only runopt --steps 20 --warmup 3 > gpurun_out/r5_ro.txt 2>&1
timeout -k 10 100 python -u scripts/xcd_probe.py > gpurun_out/r5_xcd.txt 2>&1
RBG_LIB=roaringbitmap_amd/lib/variants/probe.so timeout -k 10 100 python -u scripts/xcd_probe.py >> gpurun_out/r5_xcd.txt 2>&1
