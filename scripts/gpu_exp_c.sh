#!/bin/bash
# One gpurun call: family timings under the LDS-probe / scatter builds, then the BSI parity tests
# and C5 under the packed-count-row build, then the C2 step under the two-record serializer.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
VARIANTS="probe64 scat64 both64" bash scripts/variant_kinds.sh || exit 1
bash scripts/gpu_exp_b.sh || exit 1
