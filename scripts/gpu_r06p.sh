#!/bin/bash
# r06 session p: as session o for C5 and c5_hash (and the per-rank shares of C4 / C5).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NOCPU="" BENCH_ONLY=1 ONLY="c5:--workload c5;c5_hash:--workload c5_hash;c5_seg13:--workload c5 --segments-per-gpu 13;c4_seg8:--workload c4 --segments-per-gpu 8;c4_scan_seg8:--workload c4 --no-star-tree --segments-per-gpu 8" \
  bash scripts/gpu_r06_final.sh
