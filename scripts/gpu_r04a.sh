#!/bin/bash
# r04 session: the new tests first (combine over RCCL / host transport, indexed leaves, cancellation, the hash
# workload), then the whole -m gpu suite, the transient diagnosis of the driver's bench command, the multi-rank
# rehearsal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_combine_gpu.py tests/test_multi_rank_gpu.py tests/test_workloads_gpu.py tests/test_gpu_parity.py tests/test_timeout_gpu.py -k "combine or multi_rank or inverted or cancel or c5_hash" -x -v --timeout 300 --timeout-method thread > gpurun_out/r04a_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r04a_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04a_suite.log 2>&1
rc=$?
tail -5 gpurun_out/r04a_suite.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_transient.sh || exit 1
bash scripts/gpu_mr_bench.sh
