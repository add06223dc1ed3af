#!/bin/bash
# rocprofv3 passes for the bench kernels (run on the GPU box via gpurun):
#   1) kernel trace + stats of the whole bench, then of each workload alone (bench.py --only W)
#   2) per workload, run ALONE (bench.py --only W): a FETCH_SIZE pass and a WRITE_SIZE pass,
#      so each dominant kernel's HBM traffic is its own (TCC slots: FETCH_SIZE 3, WRITE_SIZE 2)
#   3) SQ occupancy / LDS bank-conflict counters for C2 AND and C3 uniform OR
# Counter passes never combine with runtime/system tracing.
set -o pipefail
TAG=${1:-r02}
PASSES=${2:-"kt ktw pmc sq"}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
RX='k_pair|k_emit|k_plan|k_place|k_serialize|k_wide|k_batch|k_bsi|k_dec|k_runopt|k_scan|k_shard|k_header'
if [[ " $PASSES " == *" kt "* ]]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > $OUT/bench_kt.json 2> $OUT/kt.err || { echo "kt failed"; tail $OUT/kt.err; exit 1; }
  echo "kernel trace done"
fi
if [[ " $PASSES " == *" ktw "* ]]; then
  # each workload alone under the kernel trace: per-workload kernel_stats (bench.py --only W)
  for W in c2 c2card c3u c3c c4 c5; do
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktw_$W -o run -- python3 bench.py --only $W --steps 10 --warmup 2 > $OUT/only_kt_$W.json 2> $OUT/ktw_$W.err || { echo "ktw $W failed"; tail $OUT/ktw_$W.err; exit 1; }
    echo "ktw $W done"
  done
fi
if [[ " $PASSES " == *" pmc "* ]]; then
  for W in c2 c2card c3u c3c c5; do
    for C in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 240 rocprofv3 --pmc $C --kernel-include-regex "$RX" --output-format csv -d $OUT/pmc_${W}_$C -o run -- python3 bench.py --only $W --steps 5 --warmup 1 > $OUT/only_${W}_$C.json 2> $OUT/pmc_${W}_$C.err || { echo "pmc $W $C failed"; tail $OUT/pmc_${W}_$C.err; exit 1; }
      echo "pmc $W $C done"
    done
  done
fi
if [[ " $PASSES " == *" sq "* ]]; then
  for W in c2 c3u c5; do
    timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex "$RX" --output-format csv -d $OUT/sq_$W -o run -- python3 bench.py --only $W --steps 5 --warmup 1 > /dev/null 2> $OUT/sq_$W.err || { echo "sq $W failed"; tail $OUT/sq_$W.err; exit 1; }
    echo "sq $W done"
  done
fi
find $OUT -name "*.csv" | head -60
