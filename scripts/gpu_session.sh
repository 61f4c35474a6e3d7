#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel-trace summary.  Every GPU step has its own time
# limit and the script stops at the first failure (no GPU step runs after a crash / timeout).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
set -o pipefail
step() { local name=$1; shift; echo "== $name"; "$@"; local rc=$?; echo "== $name rc=$rc"; return $rc; }
if [ -z "$SKIP_TESTS" ]; then
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
fi
step bench timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
if [ -n "$PROF" ]; then
step rocprof timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u bench.py ${PROF_ARGS:---steps 10 --warmup 2 --no-cpu-baseline} > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
tail -1 $OUT/prof.log
find $OUT/prof -name '*stats*' | head -5
fi
