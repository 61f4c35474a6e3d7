#!/bin/bash
# r06 session u: K5 with one wave per frontier entry and its children over the lanes, against the previous library
# (libpinotgpu_prev): star-tree GPU tests, then C4 star at 64 and 8 segments.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06u
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_startree_gpu.py tests/test_workloads_gpu.py -x -q --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for spec in "c4:--workload c4" "c4_8:--workload c4 --segments-per-gpu 8"; do
  n=${spec%%:*}; a=${spec#*:}
  echo "== $n"
  LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_prev.so" BENCH_ARGS="$a" timeout -k 10 500 bash scripts/ab_lib.sh || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py \
  --workload c4 --steps 20 --warmup 5 --inflight 1 --no-pmc --no-cpu-baseline --parity-segments 0 > $O/prof.log 2>&1 || exit 1
grep -h "startree" $(find $O/prof -name run_kernel_stats.csv) | cut -d, -f1-4
