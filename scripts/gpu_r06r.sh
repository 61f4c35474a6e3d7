#!/bin/bash
# r06 session r: LDS MIN / MAX read before the atomic (an atomic only where the value changes the word) against
# always-atomic (libpinotgpu_mmatomic): the parity suite's dense / MIN-MAX tests, then C2 and C1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06r
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_workloads_gpu.py -x -q --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for spec in "c2:--workload c2" "c1:--workload c1"; do
  n=${spec%%:*}; a=${spec#*:}
  echo "== $n"
  LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_mmatomic.so" BENCH_ARGS="$a" timeout -k 10 500 bash scripts/ab_lib.sh || exit 1
done
