#!/bin/bash
# round 5 (b): runOptimize with the CSR copies folded into its write kernel (tests + timing), the XCD probe,
# a kernel trace of the pipelined C2 step at K = 2 (why it is slower), then the full bench line
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_runopt.py \
  tests/test_gpu_bsi.py > gpurun_out/r5b_t.log 2>&1
timeout -k 10 200 python -u bench.py --only runopt --steps 20 --warmup 3 > gpurun_out/r5b_ro.txt 2>&1
timeout -k 10 100 python -u scripts/xcd_probe.py > gpurun_out/r5b_xcd.txt 2>&1
RBG_LIB=roaringbitmap_amd/lib/variants/probe.so timeout -k 10 100 python -u scripts/xcd_probe.py >> gpurun_out/r5b_xcd.txt 2>&1
N=10 CONFIGS=base,2:0:1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5b_pipe_kt \
  -o pipe -- python3 scripts/c2_pipe.py > gpurun_out/r5b_pipe_kt.txt 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/r5b_bench.txt 2>&1
