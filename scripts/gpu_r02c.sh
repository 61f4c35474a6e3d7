#!/bin/bash
# GPU parity suite, then A/B of the consecutive-dictionary lookups on C2, C1 and C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -4 gpurun_out/gpu_tests.log
[ $rc -le 1 ] || exit $rc
export VARIANTS="PGPU_DICT_GATHERS=0 PGPU_DICT_GATHERS=1"
BENCH_ARGS="--workload c2 --segments-per-gpu 100" bash scripts/ab_env.sh || exit 1
BENCH_ARGS="--workload c1 --segments-per-gpu 1" bash scripts/ab_env.sh || exit 1
BENCH_ARGS="--workload c5 --segments-per-gpu 100" STEPS=10 bash scripts/ab_env.sh
