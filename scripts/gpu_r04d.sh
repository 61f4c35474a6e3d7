#!/bin/bash
# r04 profiles, part 1: per-configuration bench lines (roofline + PMC traffic, full-size parity, CPU baseline) and
# serialized rocprofv3 kernel summaries -> gpurun_out/profiles (then scripts/collect_profiles.sh r04).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
WL="${WL:-adanalytics:1000 c2:100 c1:1 adanalytics_inv:1000}" PMC=1 WL_TIMEOUT=500 bash scripts/gpu_profiles.sh
