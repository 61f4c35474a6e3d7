#!/bin/bash
# r06 session zd: what the leap-frog statistics cost the C3 scan (diagnostics build PGPU_DIAG_NO_LEAP: the two-scan
# entries count skipped -- wrong statistics, same groups), C3 at 1000 and 125 segments.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
for spec in "c3_1000:" "c3_125:--segments-per-gpu 125"; do
  n=${spec%%:*}; a=${spec#*:}
  echo "== $n"
  LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_noleap.so" BENCH_ARGS="$a" timeout -k 10 500 bash scripts/ab_lib.sh || exit 1
done
