#!/bin/bash
# r05 session d: K8c with its own LDS (cursors of num_coarse, not K8a's histogram) -- partition tests, the staged /
# unstaged A/B on c5_hash and C5, their profiles with traffic; then 2 vs 3 queries in flight on C3 (1000 and 125
# segments) under the driver's step counts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_hash_partition_gpu.py tests/test_workloads_gpu.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_nostage.so" BENCH_ARGS="--workload c5_hash --segments-per-gpu 100" \
  bash scripts/ab_lib.sh || exit 1
WL="c5_hash:100 c5:100" PMC=1 WL_TIMEOUT=500 bash scripts/gpu_profiles.sh || exit 1
for segs in 1000 125; do
  for f in 2 3; do
    timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --segments-per-gpu $segs --no-cpu-baseline --no-pmc \
      --parity-segments 0 --inflight $f > $O/c3_${segs}_if$f.log 2>&1 || { tail -5 $O/c3_${segs}_if$f.log; exit 1; }
    tail -1 $O/c3_${segs}_if$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 $segs inflight $f', d['ms_per_step'], d['latency_ms_per_query'], d['roofline']['kernel_us'], d['roofline']['frac'])"
  done
done
