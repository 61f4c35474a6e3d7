#!/bin/bash
# r04 session m: the dense "simple" instance (no LUT / dictionary gathers, 4 waves per SIMD with spills) -- parity,
# then C4's scan path and C1 against the full dense instance (PGPU_NO_SIMPLE) and a 3-wave simple build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out/m
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_workloads_gpu.py tests/test_concurrency_gpu.py \
  tests/test_startree_gpu.py tests/test_orderby_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/m/suite.log 2>&1
rc=$?
tail -3 gpurun_out/m/suite.log
[ $rc -eq 0 ] || exit $rc
VARIANTS="PGPU_X=0 PGPU_NO_SIMPLE=1" BENCH_ARGS="--workload c4 --no-star-tree --no-bytes" bash scripts/ab_env.sh || exit 1
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab3.so" BENCH_ARGS="--workload c4 --no-star-tree --no-bytes" bash scripts/ab_lib.sh || exit 1
STEPS=200 VARIANTS="PGPU_X=0 PGPU_NO_SIMPLE=1" BENCH_ARGS="--workload c1 --no-bytes" bash scripts/ab_env.sh || exit 1
