#!/bin/bash
# One gpurun call: the full GPU suite and a bench line on the default build, then the round-4
# experiment builds (scripts/gpu_exp_e.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_round.sh tests || exit $?
bash scripts/gpu_exp_e.sh || exit $?
