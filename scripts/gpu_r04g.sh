#!/bin/bash
# r04 session g: the hashed-partition / compact-hash-result tests, the driver's bench command (warm-up extended),
# and the c5_hash A/B (hashed partitions against the global hash table, partition bits, LDS budget).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out/g
timeout -k 10 600 python -u -m pytest tests/test_hash_partition_gpu.py tests/test_workloads_gpu.py \
  tests/test_combine_gpu.py tests/test_multi_rank_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/g/suite.log 2>&1
rc=$?
tail -3 gpurun_out/g/suite.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --step-trace gpurun_out/g/steps20_$i.json \
    > gpurun_out/g/driver_$i.log 2>&1 || { tail -5 gpurun_out/g/driver_$i.log; exit 1; }
  tail -1 gpurun_out/g/driver_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('driver', d['ms_per_step'], d.get('warmup_run'), d['roofline']['kernel_us'], d['roofline']['frac'], d.get('parity', {}).get('ok'))"
done
STEPS=10 VARIANTS="PGPU_X=0 PGPU_NO_PART_HASH=1 PGPU_PART_HASH_PBITS=14 PGPU_PART_HASH_LDS_KB=40" \
  BENCH_ARGS="--workload c5_hash --no-bytes" bash scripts/ab_env.sh || exit 1
