#!/bin/bash
# Round-3 GPU session: the new concurrency tests first, then the whole GPU suite, then the 1-vs-4-thread QPS line
# and a short C3 bench with host trace.  Every GPU step has its own time limit; the first crash / timeout stops.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -4 $OUT/$name.log
  return $rc
}
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step conc 300 $PT tests/test_concurrency_gpu.py -m gpu || exit $?
[ -n "$SKIP_SUITE" ] || step suite 900 $PT tests -m gpu || exit $?
step qps 300 python -u tools/qps.py --workload c1 --segments 1 --threads 1 4 --seconds 3 || exit $?
[ -n "$BENCH_ARGS" ] && { step bench 600 python -u bench.py $BENCH_ARGS || exit $?; }
exit 0
