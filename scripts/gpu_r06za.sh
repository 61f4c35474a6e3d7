#!/bin/bash
# r06 session za: the C5 profile lines again after session z (bench lines with CPU baseline + parity, kernel stats).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NOCPU="" ONLY="c5:--workload c5;c5_seg13:--workload c5 --segments-per-gpu 13" bash scripts/gpu_r06_final.sh
