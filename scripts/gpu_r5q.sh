#!/bin/bash
# round 5 (q): the default bench line (no flags) on the current tree
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/r5q_bench.json 2> gpurun_out/r5q_bench.err
