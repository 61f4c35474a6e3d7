#!/bin/bash
# r05 session t: where C4's one long execute (3 queries in flight, third query of a run) spends its host time:
# the library's execution marks (PGPU_TRACE=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
O=gpurun_out/r05t
mkdir -p $O
PGPU_TRACE=1 timeout -k 10 300 python -u bench.py --workload c4 --steps 30 --warmup 5 --inflight 3 --no-cpu-baseline \
  --no-pmc --parity-segments 0 --host-profile > $O/c4_if3.log 2>&1 || { tail -5 $O/c4_if3.log; exit 1; }
tail -1 $O/c4_if3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('traced inflight 3', d['ms_per_step'], d['host_profile_us'])"
grep -n -A14 "execute: [0-9]\{4,\}" $O/c4_if3.log | head -40
