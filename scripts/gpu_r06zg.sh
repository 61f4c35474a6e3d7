#!/bin/bash
# r06 session zg: the first matching lane's entry difference by one readlane instead of two ballots (leap2_entries):
# statistics / parity GPU tests, then C3 at 1000 and 125 segments against the previous library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06zg
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_workloads_gpu.py tests/test_range_index_gpu.py -x -q \
  --timeout 250 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for spec in "c3_1000:" "c3_125:--segments-per-gpu 125"; do
  n=${spec%%:*}; a=${spec#*:}
  echo "== $n"
  LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_prev.so" BENCH_ARGS="$a" timeout -k 10 500 bash scripts/ab_lib.sh || exit 1
done
