#!/bin/bash
# r06 session s: where one C3 query's host time goes at 125 segments (PGPU_TRACE=1,marks: every execution's marks,
# the create_execute split, finalize's wait / copy / decode), one query at a time.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06s
mkdir -p $O
PGPU_TRACE=1,marks timeout -k 10 300 python3 -u bench.py --segments-per-gpu 125 --steps 20 --warmup 3 --inflight 1 \
  --no-cpu-baseline --no-pmc --parity-segments 0 > $O/trace125.log 2>&1 || { tail -5 $O/trace125.log; exit 1; }
grep "\[pgpu\]" $O/trace125.log | tail -24
