#!/bin/bash
# r04 session b: the whole -m gpu suite, the transient diagnosis of the driver's bench command, an A/B of the SADDR
# gathers (PGPU_SADDR=0 library) on C2 / C3 / C1, the multi-rank rehearsal over the C ABI combine.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04b_suite.log 2>&1
rc=$?
tail -5 gpurun_out/r04b_suite.log
[ $rc -eq 0 ] || exit $rc
fi
bash scripts/gpu_transient.sh || exit 1
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab0.so" BENCH_ARGS="--workload c2" bash scripts/ab_lib.sh || exit 1
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab0.so" BENCH_ARGS="--workload adanalytics --no-bytes" bash scripts/ab_lib.sh || exit 1
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab0.so" BENCH_ARGS="--workload c1" bash scripts/ab_lib.sh || exit 1
bash scripts/gpu_mr_bench.sh
