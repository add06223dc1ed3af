#!/bin/bash
# round 5 (z): k_wide with keys claimed from per-XCD pools (default) vs the static stride: parity on the wide
# suites, then C3 uniform / clustered OR alternating
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_wide.py tests/test_gpu_aggregations.py tests/test_gpu_range.py tests/test_gpu_fullsize.py -k "not c2 and not c5" > gpurun_out/r5z_tests.log 2>&1
V=roaringbitmap_amd/lib/variants
for r in 1 2 3; do
  for lib in widestatic widepool; do
    for w in c3u c3c; do
      RBG_LIB=$V/$lib.so timeout -k 10 200 python -u bench.py --only $w --steps 20 --warmup 3 2>/dev/null | sed "s/^/$lib /" | cut -c1-300 >> gpurun_out/r5z_wide.txt
    done
  done
done
