#!/bin/bash
# Full GPU test suite, then an A/B of the scan kernel's deadline check (libpinotgpu_ab0: no check, 108 VGPRs; ab1:
# check without the 4-wave launch bound; default: check + 4-wave bound) on C3 and C2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so  # the prebuilt libraries are current: no rebuild on the box
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -8 gpurun_out/gpu_tests.log
[ $rc -le 1 ] || exit $rc
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab0.so pinot_amd/libpinotgpu_ab1.so" bash scripts/ab_lib.sh || exit 1
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab0.so" BENCH_ARGS="--workload c2 --segments-per-gpu 100" bash scripts/ab_lib.sh
