#!/bin/bash
# r04 session za: K8c with its 16 cursor reservations issued together -- partition parity, then C5 / c5_hash profiles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out/za
timeout -k 10 900 python -u -m pytest tests/test_hash_partition_gpu.py tests/test_workloads_gpu.py tests/test_gpu_parity.py \
  tests/test_multi_rank_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/za/suite.log 2>&1
rc=$?
tail -3 gpurun_out/za/suite.log
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/profiles
WL="c5:100 c5_hash:100" PMC=1 WL_TIMEOUT=600 bash scripts/gpu_profiles.sh
