#!/bin/bash
# r06 session t: host phases of one C5 / c5_hash query at a time (PGPU_TRACE=1: create_execute split, finalize's
# wait / copy / decode) and bench's own host profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06t
mkdir -p $O
for w in c5 c5_hash; do
  PGPU_TRACE=1 timeout -k 10 300 python3 -u bench.py --workload $w --steps 6 --warmup 2 --warmup-ms 0 --inflight 1 \
    --no-cpu-baseline --no-pmc --parity-segments 0 --host-profile > $O/trace_$w.log 2>&1 || { tail -5 $O/trace_$w.log; exit 1; }
  echo "== $w"; grep "finalize:\|create_execute\|execute:" $O/trace_$w.log | tail -4
  tail -1 $O/trace_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['latency_ms_per_query'], d.get('host_profile_us'))"
done
