#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python scripts/c3_probe.py 2 10000 > gpurun_out/c3c.json 2> gpurun_out/c3c.err || { tail gpurun_out/c3c.err; exit 1; }
cat gpurun_out/c3c.json
timeout -k 10 300 python scripts/c3_probe.py 1 1000 > gpurun_out/c3u1k.json 2> gpurun_out/c3u1k.err || { tail gpurun_out/c3u1k.err; exit 1; }
cat gpurun_out/c3u1k.json
timeout -k 10 400 python scripts/c3_probe.py 1 10000 > gpurun_out/c3u.json 2> gpurun_out/c3u.err || { tail gpurun_out/c3u.err; exit 1; }
cat gpurun_out/c3u.json
