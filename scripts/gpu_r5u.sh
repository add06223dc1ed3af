#!/bin/bash
# round 5 (u): k_bsi_reg with units claimed per group of four workgroups: parity, then probe timings vs the
# static striding, alternating
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_bsi.py tests/test_gpu_bsi_buffer.py tests/test_gpu_fullsize.py -k "bsi or c5" > gpurun_out/r5u_tests.log 2>&1
V=roaringbitmap_amd/lib/variants
for r in 1 2; do
  for lib in probe_static probe; do
    RBG_LIB=$V/$lib.so timeout -k 10 150 python -u scripts/bsi_probe.py 2>&1 | grep -v amdgpu.ids | head -3 >> gpurun_out/r5u_bsi.txt
  done
done
