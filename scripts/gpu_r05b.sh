#!/bin/bash
# r05 session b: the whole GPU suite, then where a 125-segment C3 query's host time goes (one rank's share at N=8):
# PGPU_TRACE per-phase times and the bench's host profile, then 1-4 queries in flight; c5_hash without the key sort.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
PGPU_TRACE=1 timeout -k 10 300 python3 -u bench.py --steps 200 --warmup 5 --segments-per-gpu 125 --no-cpu-baseline \
  --no-pmc --no-bytes --host-profile > $O/seg125_trace.log 2>&1 || { tail -5 $O/seg125_trace.log; exit 1; }
tail -1 $O/seg125_trace.log | cut -c1-2000
grep "^\[pgpu\]" $O/seg125_trace.log | tail -12
for f in 1 2 3 4; do
  timeout -k 10 300 python3 -u bench.py --steps 200 --warmup 5 --segments-per-gpu 125 --no-cpu-baseline --no-pmc \
    --no-bytes --host-profile --inflight $f > $O/seg125_if$f.log 2>&1 || { tail -5 $O/seg125_if$f.log; exit 1; }
  tail -1 $O/seg125_if$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('inflight $f', d['ms_per_step'], d['latency_ms_per_query'], d['roofline'], d['host_profile_us'])"
done
# c5_hash with the unsorted finalize (no rocPRIM sort, slot ranges from K8h's partitions)
WL="c5_hash:100" PMC=1 WL_TIMEOUT=500 bash scripts/gpu_profiles.sh
