#!/bin/bash
# r04 session q: C3 with / without the index + scan pair compiled in (code-layout check), then the round's final
# profiles part 1 (C3, indexed C3, C2; C1 over 200 steps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_nopair.so" BENCH_ARGS="--workload adanalytics" bash scripts/ab_lib.sh || exit 1
rm -rf gpurun_out/profiles
WL="adanalytics:1000 adanalytics_inv:1000 c2:100" PMC=1 WL_TIMEOUT=500 bash scripts/gpu_profiles.sh || exit 1
WL="c1:1" STEPS=200 PMC=1 bash scripts/gpu_profiles.sh
