#!/bin/bash
# r06 session n: the star-tree metric tests and the suite's star / workload tests on the reverted layout (statistics
# after the table again, 8-byte star metrics), then the new library against libpinotgpu_prev on C4 star, C3 at 125
# segments and C1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_startree_gpu.py tests/test_workloads_gpu.py tests/test_timeout_gpu.py -x -q \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for spec in "c4:--workload c4" "c3_125:--segments-per-gpu 125" "c1:--workload c1"; do
  n=${spec%%:*}; a=${spec#*:}
  echo "== $n"
  LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_prev.so" BENCH_ARGS="$a" timeout -k 10 500 bash scripts/ab_lib.sh || exit 1
done
