#!/bin/bash
# GPU suite, then one C3 bench with the host trace and a kernel / copy timeline (rocprofv3, no counters).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out/tl
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -le 1 ] || exit $rc
fi
PGPU_TRACE=1 timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pmc --host-profile ${BENCH_ARGS} > gpurun_out/tl/trace.log 2>&1 || exit 1
tail -1 gpurun_out/tl/trace.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/tl/prof -o run -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pmc --no-bytes ${BENCH_ARGS} > gpurun_out/tl/prof.log 2>&1
echo prof rc=$?
