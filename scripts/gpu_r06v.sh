#!/bin/bash
# r06 session v: issue priority by dispatch slot (libpinotgpu_prio: s_setprio 0..3 by blockIdx quarter) against the
# default, each with the slot weights (default step) and with equal shares (slot_weight_step=0): C3 at 125 / 1000
# segments, indexed C3, C2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
for spec in "c3_125:--segments-per-gpu 125" "c3_1000:" "c3inv:--workload adanalytics_inv" "c2:--workload c2"; do
  n=${spec%%:*}; a=${spec#*:}
  echo "== $n"
  LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_prio.so" BENCH_ARGS="$a" timeout -k 10 500 bash scripts/ab_lib.sh || exit 1
  echo "-- equal shares"
  LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_prio.so" BENCH_ARGS="$a --config slot_weight_step=0.0" timeout -k 10 500 bash scripts/ab_lib.sh || exit 1
done
