#!/bin/bash
# round 5 (s): per-workgroup end times of C5's k_bsi_reg (probe build)
set -e
mkdir -p gpurun_out
V=roaringbitmap_amd/lib/variants
timeout -k 10 150 python -u scripts/bsi_probe.py > gpurun_out/r5s_bsi.txt 2>&1
RBG_LIB=$V/probe.so timeout -k 10 150 python -u scripts/bsi_probe.py >> gpurun_out/r5s_bsi.txt 2>&1
