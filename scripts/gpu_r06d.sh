#!/bin/bash
# r06 session d: the execution's timing events (six hipEventRecord marker packets between the dependent dispatches of
# a query) against a library build without them (PGPU_NO_TIMING_EVENTS), on C3 at 125 and 1000 segments (step and
# one-query latency), then the kernel / copy timeline of the event-free build at 125 segments.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
for spec in "c3_125:--segments-per-gpu 125" "c3_1000:"; do
  n=${spec%%:*}; a=${spec#*:}
  echo "== $n"
  LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_noev.so" BENCH_ARGS="$a --parity-segments 0" \
    timeout -k 10 600 bash scripts/ab_lib.sh || exit 1
done
PGPU_LIB=pinot_amd/libpinotgpu_noev.so timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
  -d $O/prof -o run -- python3 -u bench.py --segments-per-gpu 125 --steps 10 --warmup 2 --inflight 1 --no-cpu-baseline \
  --no-pmc --no-bytes --parity-segments 0 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name run_kernel_trace.csv | head -1)
python3 tools/timeline.py $(dirname $f) > $O/timeline125_noev.txt && tail -12 $O/timeline125_noev.txt
