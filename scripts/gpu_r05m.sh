#!/bin/bash
# r05 session m: the dense scan instance at 4 waves per SIMD (launch bound 4: 128 VGPRs, spills) against 3 on C2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_dense4.so" \
  BENCH_ARGS="--workload c2 --parity-segments 100" bash scripts/ab_lib.sh || exit 1
