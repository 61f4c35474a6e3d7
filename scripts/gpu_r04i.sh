#!/bin/bash
# r04 session i: tests of this session's hash-path changes, c5_hash with the re-shaped partitions, then the round's
# profiles part 1 (C3, C2, C1, indexed C3: bench lines with PMC traffic + serialized kernel summaries).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out/i
timeout -k 10 600 python -u -m pytest tests/test_hash_partition_gpu.py tests/test_workloads_gpu.py \
  tests/test_combine_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/i/suite.log 2>&1
rc=$?
tail -3 gpurun_out/i/suite.log
[ $rc -eq 0 ] || exit $rc
STEPS=10 VARIANTS="PGPU_X=0 PGPU_X=1" BENCH_ARGS="--workload c5_hash --no-bytes" bash scripts/ab_env.sh || exit 1
bash scripts/gpu_r04d.sh
