#!/bin/bash
# r04 session p: the whole -m gpu suite on the current tree, the driver's command twice, C5 (compaction ranges
# without same-address atomics) and c5_hash through the global hash table (compaction reservations per workgroup).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out/p
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/p/suite.log 2>&1
rc=$?
tail -3 gpurun_out/p/suite.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/p/driver_$i.log 2>&1 || { tail -5 gpurun_out/p/driver_$i.log; exit 1; }
  tail -1 gpurun_out/p/driver_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('driver', d['ms_per_step'], r['kernel_us'], r['frac'], d['parity']['ok'])"
done
STEPS=10 VARIANTS="PGPU_X=0 PGPU_NO_PART_HASH=1" BENCH_ARGS="--workload c5_hash --no-bytes" bash scripts/ab_env.sh || exit 1
VARIANTS="PGPU_X=0" BENCH_ARGS="--workload c5" bash scripts/ab_env.sh || exit 1
