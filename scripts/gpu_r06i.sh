#!/bin/bash
# r06 session i: the GPU suite with the statistics ring (one fill per 256 executions) and the epilogue's export of
# small tables to pinned host memory (no copy launch), then an interleaved A/B against the previous library on C3
# at 125 / 1000 segments, C1 and C2 (ms/step, scan, frac, latency), and the serialized 125-segment timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log
[ $rc -ne 0 ] && exit $rc
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_prev.so"
for spec in "c3_125:--segments-per-gpu 125" "c1:--workload c1" "c3_1000:" "c2:--workload c2"; do
  n=${spec%%:*}; a=${spec#*:}
  echo "== $n"
  LIBS="$LIBS" BENCH_ARGS="$a" timeout -k 10 600 bash scripts/ab_lib.sh || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/prof -o run -- \
  python3 -u bench.py --segments-per-gpu 125 --steps 10 --warmup 2 --inflight 1 --roofline-steps 1 --no-cpu-baseline \
  --no-pmc --no-bytes --parity-segments 0 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name run_kernel_trace.csv)
python3 tools/timeline.py $(dirname $f) filter_groupby 2 2 > $O/timeline125.txt && tail -16 $O/timeline125.txt
