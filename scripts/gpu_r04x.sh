#!/bin/bash
# r04 session x: existing launch knobs on the two latency-bound dense scans -- chunked tile order, the sparse instance,
# the general dense instance for the C4 scan path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
VARIANTS="PGPU_X=0 PGPU_TILE_ORDER=1 PGPU_NO_DENSE=1" BENCH_ARGS="--workload c2" bash scripts/ab_env.sh || exit 1
VARIANTS="PGPU_X=0 PGPU_TILE_ORDER=1 PGPU_NO_SIMPLE=1 PGPU_NO_DENSE=1" BENCH_ARGS="--workload c4 --segments-per-gpu 64 --no-star-tree" bash scripts/ab_env.sh || exit 1
