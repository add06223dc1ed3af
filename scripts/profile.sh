#!/bin/bash
# rocprofv3 passes for the bench kernels (run on the GPU box via gpurun):
#   1) kernel trace + stats   2) FETCH_SIZE   3) WRITE_SIZE   4) SQ occupancy/LDS counters
# Kernel names are kept whole (no -T), so each template instance (k_pair_wave<OP, MODE>)
# gets its own line: MODE 0 materialises results, MODE 1 is andCardinality.
# Counter passes are separate (TCC slots: FETCH_SIZE 3, WRITE_SIZE 2) and never combined
# with runtime/system tracing.
set -o pipefail
TAG=${1:-r01}
ARGS=${2:-"--steps 20 --warmup 3 --no-cpu-baseline"}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
RX='k_pair|k_emit|k_compact|k_plan|k_place|k_wide|k_batch|k_bsi|k_dec|k_runopt|k_scan'
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py $ARGS > $OUT/bench_kt.json 2> $OUT/kt.err || { echo "kt failed"; tail $OUT/kt.err; exit 1; }
echo "kernel trace done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --c3-n 2000 --c4-pairs 200000 --c5-rows 100000000 > /dev/null 2> $OUT/pmc_fetch.err || { echo "fetch failed"; tail $OUT/pmc_fetch.err; exit 1; }
echo "fetch done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --c3-n 2000 --c4-pairs 200000 --c5-rows 100000000 > /dev/null 2> $OUT/pmc_write.err || { echo "write failed"; tail $OUT/pmc_write.err; exit 1; }
echo "write done"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex "$RX" --output-format csv -d $OUT/pmc_sq -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --c3-n 2000 --c4-pairs 200000 --c5-rows 100000000 > /dev/null 2> $OUT/pmc_sq.err || { echo "sq failed"; tail $OUT/pmc_sq.err; exit 1; }
echo "sq done"
find $OUT -name "*.csv" | head -50
