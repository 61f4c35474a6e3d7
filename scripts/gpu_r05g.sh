#!/bin/bash
# r05 session g: a rank whose own combine step fails fails every rank (two ranks, host transport); C2 with one shared
# dictionary array for md (diagnostic build: the access pattern a table-global dval array would have) against the
# per-segment dictionaries and against no gathers at all.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_multi_rank_gpu.py -k "rank_failure" -m gpu -x -q --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_shareddval.so pinot_amd/libpinotgpu_ab_nodval.so" \
  BENCH_ARGS="--workload c2 --segments-per-gpu 100 --parity-segments 0" bash scripts/ab_lib.sh || exit 1
