#!/bin/bash
# r05 session c: K8c staged write-out (part_pass_kernel<true, 1|2>) -- the partition / hash-partition / workload
# parity tests, then A/B against the library built without it (PGPU_PART_NO_STAGE) on C5 and c5_hash, then C5's
# kernel summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_hash_partition_gpu.py tests/test_workloads_gpu.py \
  tests/test_timeout_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_nostage.so" BENCH_ARGS="--workload c5 --segments-per-gpu 100" \
  bash scripts/ab_lib.sh || exit 1
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_nostage.so" BENCH_ARGS="--workload c5_hash --segments-per-gpu 100" \
  bash scripts/ab_lib.sh || exit 1
WL="c5:100" PMC=1 WL_TIMEOUT=500 bash scripts/gpu_profiles.sh
