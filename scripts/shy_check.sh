#!/bin/bash
# wide parity, then C3 FastAggregation.and (workShyAnd) under the default library and $VARIANTS, alternating
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_aggregations.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/wide_tests.log 2>&1
rc=$?; tail -2 gpurun_out/wide_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in base $VARIANTS; do
  if [ $v = base ]; then unset RBG_LIB; else export RBG_LIB=$PWD/roaringbitmap_amd/lib/variants/$v.so; fi
  for w in c3u_and c3c_and; do
    timeout -k 10 200 python bench.py --only $w --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/shy_${v}_$w.json 2> gpurun_out/shy_${v}_$w.err || { echo "$v $w failed"; tail -3 gpurun_out/shy_${v}_$w.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline_rank0']; print(sys.argv[2], sys.argv[3], d['ms_per_step'], r['kernel_ms'], r['bytes_read_per_launch'])" gpurun_out/shy_${v}_$w.json $v $w
  done
done
done
