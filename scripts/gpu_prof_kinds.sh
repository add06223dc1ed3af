#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/profile.sh ${1:-r01} && timeout -k 10 200 python scripts/kind_matrix.py > gpurun_out/kind_matrix.txt 2>&1
rc=$?; cat gpurun_out/kind_matrix.txt; exit $rc
