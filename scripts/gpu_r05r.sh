#!/bin/bash
# r05 session r: 4 matched docs per lane batch (lane-group path of the scans) against 2: C4 scan path, C2, C3, C1;
# then the C4 star-tree profile line again (session o's box had a loaded host).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_lane4.so" BENCH_ARGS="--workload c4 --no-star-tree" bash scripts/ab_lib.sh || exit 1
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_lane4.so" BENCH_ARGS="--workload c2" bash scripts/ab_lib.sh || exit 1
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_lane4.so" BENCH_ARGS="--segments-per-gpu 250" bash scripts/ab_lib.sh || exit 1
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_lane4.so" STEPS=200 BENCH_ARGS="--workload c1" bash scripts/ab_lib.sh || exit 1
rm -rf gpurun_out/profiles
PMC=1 WL="c4:64" bash scripts/gpu_profiles.sh
