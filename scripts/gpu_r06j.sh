#!/bin/bash
# r06 session j: which half of session i's change costs the latency -- the statistics ring, the epilogue's export, both,
# neither (libpinotgpu_noexp / _noring / the new one / _prev) on C1 and C3 at 125 segments, then PGPU_TRACE=1 host
# phases of C1 one query at a time for the new and the previous library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_noexp.so pinot_amd/libpinotgpu_noring.so pinot_amd/libpinotgpu_prev.so"
for spec in "c1:--workload c1" "c3_125:--segments-per-gpu 125"; do
  n=${spec%%:*}; a=${spec#*:}
  echo "== $n"
  LIBS="$LIBS" BENCH_ARGS="$a" timeout -k 10 600 bash scripts/ab_lib.sh || exit 1
done
for lib in libpinotgpu libpinotgpu_prev; do
  PGPU_LIB=pinot_amd/$lib.so PGPU_TRACE=1 timeout -k 10 300 python3 -u bench.py --workload c1 --steps 20 --warmup 3 \
    --inflight 1 --no-cpu-baseline --no-pmc --parity-segments 0 --host-profile > $O/trace_$lib.log 2>&1 || exit 1
  echo "== $lib"; grep "finalize:\|execute:" $O/trace_$lib.log | tail -4
  tail -1 $O/trace_$lib.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['latency_ms_per_query'], d.get('host_profile'))" | cut -c1-600
done
