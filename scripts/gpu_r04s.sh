#!/bin/bash
# r04 session s: the index + scan pair as its own kernel instance -- parity of the scan paths, the driver's command,
# then the C3 and indexed C3 profile lines again (final library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out/s
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_workloads_gpu.py tests/test_concurrency_gpu.py \
  tests/test_timeout_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s/suite.log 2>&1
rc=$?
tail -3 gpurun_out/s/suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s/driver.log 2>&1 || { tail -5 gpurun_out/s/driver.log; exit 1; }
tail -1 gpurun_out/s/driver.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('driver', d['ms_per_step'], r['kernel_us'], r['frac'], d['parity']['ok'])"
WL="adanalytics:1000 adanalytics_inv:1000" PMC=1 WL_TIMEOUT=500 bash scripts/gpu_profiles.sh
