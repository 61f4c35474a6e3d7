#!/bin/bash
# r04 session l: the timeout / cancellation tests after the finalize-buffer change, the rest of the -m gpu files from
# test_timeout on, the indexed C3 line with the BITDIR prefetch, c5_hash with (hashed key, value) mid records,
# the C1 profile line over 200 steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out/l
timeout -k 10 600 python -u -m pytest tests/test_timeout_gpu.py tests/test_hash_partition_gpu.py tests/test_workloads_gpu.py \
  tests/test_combine_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/l/suite.log 2>&1
rc=$?
tail -3 gpurun_out/l/suite.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload adanalytics_inv --steps 20 --warmup 5 --no-pmc --no-cpu-baseline \
    > gpurun_out/l/inv_$i.log 2>&1 || { tail -5 gpurun_out/l/inv_$i.log; exit 1; }
  tail -1 gpurun_out/l/inv_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('inv', d['ms_per_step'], r['kernel_us'], r['frac'])"
done
STEPS=10 VARIANTS="PGPU_X=0 PGPU_NO_MID_PAIR=1" BENCH_ARGS="--workload c5_hash --no-bytes" bash scripts/ab_env.sh || exit 1
WL="c1:1" STEPS=200 PMC=1 bash scripts/gpu_profiles.sh
