#!/bin/bash
# round 5 (l): whole GPU suite on the CU-pooled default; per-wave probe of both walks; C2 kernel trace
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r5l_tests.log 2>&1
V=roaringbitmap_amd/lib/variants
RBG_PW_CU=0 RBG_LIB=$V/probe.so timeout -k 10 100 python -u scripts/xcd_probe.py > gpurun_out/r5l_probe_walk.txt 2>&1
RBG_PW_CU=1 RBG_LIB=$V/probe.so timeout -k 10 100 python -u scripts/xcd_probe.py > gpurun_out/r5l_probe_cu.txt 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5l_c2 -o c2 -- python3 bench.py --only c2 --steps 20 --warmup 5 > gpurun_out/r5l_c2.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5l_c2card -o c2card -- python3 bench.py --only c2card --steps 20 --warmup 5 > gpurun_out/r5l_c2card.txt 2>&1
