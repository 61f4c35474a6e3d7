#!/bin/bash
# r06 session ze: the leap-frog scanner state by one addition instead of a 5-step segmented fill (leap2_entries): the
# parity / statistics GPU tests, then C3 at 1000 and 125 segments against the previous library and the no-statistics
# diagnostics build (the bound on what the statistics can still give).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06ze
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log
[ $rc -ne 0 ] && exit $rc
for spec in "c3_1000:" "c3_125:--segments-per-gpu 125"; do
  n=${spec%%:*}; a=${spec#*:}
  echo "== $n"
  LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_prev.so pinot_amd/libpinotgpu_noleap.so" BENCH_ARGS="$a" timeout -k 10 500 bash scripts/ab_lib.sh || exit 1
done
