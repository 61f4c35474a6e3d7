#!/bin/bash
# r05 session h: the whole GPU suite with the table-global value arrays (and the indexed leaf's directory entry cached
# per 65536-doc block); C2 A/B against the per-segment value arrays; indexed C3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_noglobal.so" \
  BENCH_ARGS="--workload c2 --segments-per-gpu 100 --parity-segments 0" bash scripts/ab_lib.sh || exit 1
timeout -k 10 300 python -u bench.py --workload adanalytics_inv --steps 50 --warmup 5 --no-cpu-baseline --no-pmc \
  > $O/inv.log 2>&1 || { tail -5 $O/inv.log; exit 1; }
tail -1 $O/inv.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('inv', d['ms_per_step'], d['roofline'])"
