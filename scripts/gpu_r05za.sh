#!/bin/bash
# r05 session za: the sparse scans' tile order -- contiguous runs per workgroup (as built) vs XCD-interleaved tiles
# (A/B build) on C3 at 125 and 1000 segments, indexed C3 and the C4 scan path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_inter.so" STEPS=200 BENCH_ARGS="--segments-per-gpu 125" bash scripts/ab_lib.sh || exit 1
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_inter.so" STEPS=100 BENCH_ARGS="--parity-segments 0" bash scripts/ab_lib.sh || exit 1
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_inter.so" BENCH_ARGS="--workload adanalytics_inv --parity-segments 0" bash scripts/ab_lib.sh || exit 1
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_inter.so" BENCH_ARGS="--workload c4 --no-star-tree" bash scripts/ab_lib.sh || exit 1
