#!/bin/bash
# r05 session o: final profiles part 2 -- C4 star-tree and scan paths, C5, c5_hash (bench lines with CPU baselines and
# FETCH_SIZE traffic, serialized rocprofv3 kernel summaries).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PMC=1 WL="c4:64 c4:64:scan:--no-star-tree c5:100 c5_hash:100" bash scripts/gpu_profiles.sh
