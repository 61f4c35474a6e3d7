#!/bin/bash
# r06 session m: which half of the star-tree change costs K6 (175 -> 270 us): int32 metric arrays (nonarrow: 8-byte
# arrays again) or the metric-sector count (nosec), against the library before both (prev), C4 star path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_nonarrow.so pinot_amd/libpinotgpu_nosec.so pinot_amd/libpinotgpu_prev.so" \
  BENCH_ARGS="--workload c4" timeout -k 10 800 bash scripts/ab_lib.sh
