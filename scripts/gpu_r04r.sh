#!/bin/bash
# r04 session r: the round's final profiles part 2 (C4 star-tree and scan paths, C5, c5_hash).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
WL="c4:64 c4:64:scan:--no-star-tree c5:100 c5_hash:100" PMC=1 WL_TIMEOUT=600 bash scripts/gpu_profiles.sh
