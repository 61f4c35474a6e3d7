#!/bin/bash
# r05 session u: star-tree records uploaded only when they change (per scratch): the star / scan parity tests, then
# C4 at 3 in flight with the library's marks, and plain 20-step lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
O=gpurun_out/r05u
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_startree_gpu.py tests/test_workloads_gpu.py tests/test_concurrency_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
PGPU_TRACE=1 timeout -k 10 300 python -u bench.py --workload c4 --steps 30 --warmup 5 --inflight 3 --no-cpu-baseline \
  --no-pmc --parity-segments 0 --host-profile > $O/c4_if3.log 2>&1 || { tail -5 $O/c4_if3.log; exit 1; }
tail -1 $O/c4_if3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('traced inflight 3', d['ms_per_step'], d['host_profile_us'])"
grep -n -A14 "execute: [0-9]\{4,\}" $O/c4_if3.log | head -30
for i in 3 3 2; do
  timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 5 --inflight $i --no-cpu-baseline --no-pmc \
    --parity-segments 64 --host-profile > $O/c4.log 2>&1 || { tail -5 $O/c4.log; exit 1; }
  tail -1 $O/c4.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('inflight', $i, d['ms_per_step'], d['host_profile_us'], d['parity']['ok'])"
done
