#!/bin/bash
# One gpurun call: per-family LDS / occupancy counters under the default library and the two
# attribution builds, then the kernel trace of the bench and of each
# workload alone (profiles/r04).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
VARIANTS="base probelin scatlin" bash scripts/pmc_attrib.sh "A A and" "A B and" "A R and" "B B and" "B R and" \
  "R R and" "M M and" "M M card" || exit 1
python3 scripts/pmc_families_json.py gpurun_out gpurun_out/pmc_families.json || exit 1
bash scripts/profile.sh r04 "kt ktw" || exit 1
