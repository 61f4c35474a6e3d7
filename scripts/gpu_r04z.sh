#!/bin/bash
# r04 session z: the whole GPU suite on the final tree (dense-instance threshold 1/4), then the C4 scan path's profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out/z
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/z/suite.log 2>&1
rc=$?
tail -3 gpurun_out/z/suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
rm -rf gpurun_out/profiles
WL="c4:64:scan:--no-star-tree" PMC=1 WL_TIMEOUT=500 bash scripts/gpu_profiles.sh
