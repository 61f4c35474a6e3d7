#!/bin/bash
# r05 session zd: K8a / K8c at 4 waves per SIMD as built: the partition / hash-partition / workload / multi-rank tests,
# then the C5 and c5_hash profile lines (CPU baselines, FETCH_SIZE traffic, kernel summaries).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05zd
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/profiles
PMC=1 WL="c5:100 c5_hash:100" bash scripts/gpu_profiles.sh
