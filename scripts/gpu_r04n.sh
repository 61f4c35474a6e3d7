#!/bin/bash
# r04 session n: the index leaf + scan leaf pair evaluated together (bitdir_range) -- parity of indexed leaves, then
# the indexed C3 line against PGPU_NO_PAIR_LEAVES=1, and C3 (no index) unchanged.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out/n
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_workloads_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/n/suite.log 2>&1
rc=$?
tail -3 gpurun_out/n/suite.log
[ $rc -eq 0 ] || exit $rc
VARIANTS="PGPU_X=0 PGPU_NO_PAIR_LEAVES=1" BENCH_ARGS="--workload adanalytics_inv" bash scripts/ab_env.sh || exit 1
STEPS=20 VARIANTS="PGPU_X=0" BENCH_ARGS="--workload adanalytics --no-bytes" bash scripts/ab_env.sh || exit 1
