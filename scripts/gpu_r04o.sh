#!/bin/bash
# r04 session o: the pair path with the directory entry loaded a tile ahead -- parity, then the indexed C3 line
# (prefetch / no prefetch / leaf by leaf) and C3 beside it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out/o
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_workloads_gpu.py tests/test_hash_partition_gpu.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/o/suite.log 2>&1
rc=$?
tail -3 gpurun_out/o/suite.log
[ $rc -eq 0 ] || exit $rc
VARIANTS="PGPU_X=0 PGPU_PAIR_PREFETCH=0 PGPU_NO_PAIR_LEAVES=1" BENCH_ARGS="--workload adanalytics_inv" bash scripts/ab_env.sh || exit 1
VARIANTS="PGPU_X=0" BENCH_ARGS="--workload adanalytics" bash scripts/ab_env.sh || exit 1
