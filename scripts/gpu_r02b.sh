#!/bin/bash
# Full GPU test suite, then the default bench (C3) and C2 without PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so  # the prebuilt library is current: no rebuild on the box
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -8 gpurun_out/gpu_tests.log
[ $rc -le 1 ] || exit $rc
STEPS=20 LIBS="pinot_amd/libpinotgpu.so" bash scripts/ab_lib.sh || exit 1
LIBS="pinot_amd/libpinotgpu.so" BENCH_ARGS="--workload c2 --segments-per-gpu 100" bash scripts/ab_lib.sh
