#!/bin/bash
# r06 session zi: K6 loads a lane's 16 pre-aggregated metrics as one 128-B line (8 16-byte loads when any matched,
# arrays 16-B aligned and padded at pin) instead of 16 conditional 8-byte loads: star-tree / workload GPU tests, then
# C4 star at 64 and 8 segments against the previous library, and K6's duration alone (rocprof, one query at a time).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06zi
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
for lib in libpinotgpu libpinotgpu_prev; do
  PGPU_LIB=pinot_amd/$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$lib -o run -- \
    python3 -u bench.py --workload c4 --steps 20 --warmup 5 --inflight 1 --no-pmc --no-cpu-baseline --parity-segments 0 \
    > $O/prof_$lib.log 2>&1 || exit 1
  echo "$lib $(grep -h 'startree' $(find $O/p_$lib -name run_kernel_stats.csv) | python3 -c "import sys,csv; [print(r[0][6:30], round(float(r[3])/1e3,1), end='; ') for r in csv.reader(sys.stdin)]")"
done
