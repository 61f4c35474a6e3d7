#!/bin/bash
# One GPU session: parity tests, smoke, a short bench.  Stops at the first crash / timeout (exit >= 2 from
# pytest other than test failures, or any signal exit) so a faulting kernel never gets a second launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
rocm-smi --showproductname > $OUT/rocm_smi.txt 2>&1 || true
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" | tee -a $OUT/gpu_tests.log
tail -5 $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"; tail -3 $OUT/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "$BENCH_ARGS" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py $BENCH_ARGS > $OUT/bench.log 2>&1
  rc=$?
  echo "bench rc=$rc"; tail -3 $OUT/bench.log
  exit $rc
fi
