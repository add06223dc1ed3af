#!/bin/bash
# GPU tests given in $TESTS, then (only when pytest ended normally: all passed or
# assertion failures, no crash / time limit) the kind matrix under each library
# variant in $VARIANTS.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 ${TEST_LIMIT:-700} python -u -m pytest $TESTS -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/tests.log | tail -150
tail -5 gpurun_out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
[ -z "$VARIANTS" ] && exit $rc
VARIANTS="$VARIANTS" bash scripts/variant_kinds.sh || exit 1
exit $rc
