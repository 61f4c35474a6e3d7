#!/bin/bash
# r05 session zb: interleaved tiles for the 4-doc-batch sparse instance's plans: the whole GPU suite, then the C4 scan
# path's profile line (CPU baseline, traffic, kernel summary).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05zb
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/profiles
PMC=1 WL="c4:64:scan:--no-star-tree" bash scripts/gpu_profiles.sh
