#!/bin/bash
# r06 session o: the profile set's bench lines again with their CPU baseline and full-size parity legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NOCPU="" BENCH_ONLY=1 ONLY="adanalytics_inv:--workload adanalytics_inv;c1:--workload c1;c2:--workload c2;c4:--workload c4;c4_scan:--workload c4 --no-star-tree;adanalytics_seg125:--segments-per-gpu 125" \
  bash scripts/gpu_r06_final.sh
