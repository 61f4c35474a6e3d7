#!/bin/bash
# r05 session w: C3 (the driver's configuration) with 2 vs 4 docs per lane batch in the sparse instances, interleaved
# on one box; C4 scan alike.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_lane2.so" STEPS=100 BENCH_ARGS="--parity-segments 0" bash scripts/ab_lib.sh || exit 1
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_lane2.so" STEPS=100 BENCH_ARGS="--parity-segments 0" bash scripts/ab_lib.sh || exit 1
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_lane2.so" BENCH_ARGS="--workload c4 --no-star-tree" bash scripts/ab_lib.sh || exit 1
