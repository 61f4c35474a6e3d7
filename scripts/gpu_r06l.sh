#!/bin/bash
# r06 session l: where the C4 star path's time went (0.17 -> 0.28 ms/step in session k): the current library, the
# one before the int32 star metrics (libpinotgpu_prev: after the slot weights) and round 5's, interleaved; then the
# per-kernel statistics of the current one.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06l
mkdir -p $O
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_prev.so pinot_amd/libpinotgpu_r05.so" BENCH_ARGS="--workload c4" \
  timeout -k 10 600 bash scripts/ab_lib.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py \
  --workload c4 --steps 20 --warmup 3 --no-cpu-baseline --no-pmc --parity-segments 0 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name run_kernel_stats.csv)
cut -d, -f1-8 $f | head -12
