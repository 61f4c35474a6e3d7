#!/bin/bash
# r06 session y: queries in flight (2 / 3 / 4 / 6) at 125 and 1000 C3 segments, 20 and 200 steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
V="--inflight 2;--inflight 3;--inflight 4;--inflight 6"
echo "== 125, 20 steps"; VARIANTS="$V" BENCH_ARGS="--segments-per-gpu 125" timeout -k 10 500 bash scripts/ab_args.sh || exit 1
echo "== 125, 200 steps"; STEPS=200 VARIANTS="$V" BENCH_ARGS="--segments-per-gpu 125" timeout -k 10 500 bash scripts/ab_args.sh || exit 1
echo "== 1000, 20 steps"; VARIANTS="--inflight 3;--inflight 4" timeout -k 10 600 bash scripts/ab_args.sh || exit 1
