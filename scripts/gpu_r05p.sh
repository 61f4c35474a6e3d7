#!/bin/bash
# r05 session p: host-side trace of C4 star-tree queries (PGPU_TRACE=1) with 1 and 3 queries in flight; the star
# path's step at 1 / 2 / 3 in flight.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
O=gpurun_out/r05p
mkdir -p $O
PGPU_TRACE=1 timeout -k 10 300 python -u bench.py --workload c4 --steps 6 --warmup 3 --warmup-ms 0 --inflight 3 \
  --no-cpu-baseline --no-pmc --no-bytes --parity-segments 0 --roofline-steps 2 > $O/c4_trace3.log 2>&1 || { tail -5 $O/c4_trace3.log; exit 1; }
grep "\[pgpu\]" $O/c4_trace3.log | tail -18
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --workload c4 --steps 50 --warmup 5 --inflight $i --no-cpu-baseline --no-pmc \
    --parity-segments 0 --host-profile > $O/c4_if$i.log 2>&1 || { tail -5 $O/c4_if$i.log; exit 1; }
  tail -1 $O/c4_if$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('inflight', $i, d['ms_per_step'], d['host_profile_us'])"
done
