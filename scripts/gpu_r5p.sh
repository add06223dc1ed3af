#!/bin/bash
# round 5 (p): cost of the phase events in the timed C2 loop
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/c2_events.py > gpurun_out/r5p_events.txt 2>&1
