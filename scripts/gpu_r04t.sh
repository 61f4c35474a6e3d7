#!/bin/bash
# r04 session t: the pure-AND sparse instance (FAST) -- parity, then C3 against PGPU_NO_FAST_INSTANCE=1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out/t
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_workloads_gpu.py tests/test_timeout_gpu.py \
  tests/test_concurrency_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t/suite.log 2>&1
rc=$?
tail -3 gpurun_out/t/suite.log
[ $rc -eq 0 ] || exit $rc
VARIANTS="PGPU_X=0 PGPU_NO_FAST_INSTANCE=1" BENCH_ARGS="--workload adanalytics" bash scripts/ab_env.sh || exit 1
