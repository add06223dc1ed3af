#!/bin/bash
# round 6 profiles: kernel traces of the whole bench and of each workload alone, per-workload FETCH / WRITE
# passes, SQ occupancy passes (c2, c3u, c5), the LDS / VALU pass of k_bsi_reg, then two driver-style bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
bash scripts/profile.sh r06 "kt ktw pmc sq" > gpurun_out/r6/t5_profile.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/r6/t5_profile.log; exit 1; }
tail -3 gpurun_out/r6/t5_profile.log
timeout -k 10 -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --kernel-include-regex "k_bsi_reg" --output-format csv -d gpurun_out/r6/pmc_c5/C5bsi -o run -- python3 bench.py --only c5 --steps 3 --warmup 1 > /dev/null 2> gpurun_out/r6/pmc_c5.err || { echo "c5 pmc failed"; tail -5 gpurun_out/r6/pmc_c5.err; exit 1; }
python3 scripts/pmc_lds_summary.py gpurun_out/r6/pmc_c5 gpurun_out/r6/pmc_c5.json
for i in 1 2; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r6/t5_bench_$i.json 2> gpurun_out/r6/t5_bench_$i.err || { echo "bench failed"; tail gpurun_out/r6/t5_bench_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r6/t5_bench_$i.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], json.dumps(d['extra'].get('phase_ms')), d['extra']['c5_bsi_range_sum']['ms_per_step'])"
done
