#!/bin/bash
# r05 session j: table-global value arrays with threshold maps (no memory access per lookup): parity tests, C2 A/B
# against the per-segment arrays, C3 (records grew) and the workgroup-time diagnostics (gpu_r05i.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05j
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_workloads_gpu.py tests/test_hash_partition_gpu.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_noglobal.so" \
  BENCH_ARGS="--workload c2 --segments-per-gpu 100 --parity-segments 0" bash scripts/ab_lib.sh || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc > $O/c3.log 2>&1 || { tail -5 $O/c3.log; exit 1; }
tail -1 $O/c3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['ms_per_step'], d['roofline']['kernel_us'], d['parity'])"
bash scripts/gpu_r05i.sh
