#!/bin/bash
# LDS counters of k_pair_wave per family case under each library variant ($VARIANTS,
# built by scripts/build_variant.sh; "base" = the default library).  Attribution builds
# (RBG_EXP_PROBE_LIN / RBG_EXP_SCAT_LIN: one access made lane-linear, wrong results) show
# how much of the conflict count a named access causes.
#   VARIANTS="base probelin scatlin" bash scripts/pmc_attrib.sh "A A and" "M M and" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for v in ${VARIANTS:-base}; do
  if [ $v = base ]; then unset RBG_LIB; else export RBG_LIB=$PWD/roaringbitmap_amd/lib/variants/$v.so; fi
  PMC_OUT=gpurun_out/pmc_lds_$v bash scripts/pmc_lds.sh "$@" || exit 1
  python3 scripts/pmc_lds_summary.py gpurun_out/pmc_lds_$v gpurun_out/pmc_lds_$v.json > gpurun_out/pmc_lds_$v.txt || exit 1
  echo "== $v"; cat gpurun_out/pmc_lds_$v.txt
done
