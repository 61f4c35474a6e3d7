#!/bin/bash
# r04 session f: the -m gpu files from the hashed partitions on (the earlier files passed in session b), then the rest
# of session b (transient diagnosis, SADDR A/B, multi-rank rehearsal).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_hash_partition_gpu.py tests/test_multi_rank_gpu.py \
  tests/test_orderby_gpu.py tests/test_raw_columns_gpu.py tests/test_startree_gpu.py tests/test_timeout_gpu.py \
  tests/test_workloads_gpu.py tests/test_combine_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/r04f_suite.log 2>&1
rc=$?
tail -5 gpurun_out/r04f_suite.log
[ $rc -eq 0 ] || exit $rc
SKIP_TESTS=1 bash scripts/gpu_r04b.sh
