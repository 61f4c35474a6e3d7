#!/bin/bash
# r05 session s: where the C4 star path's step goes at 3 queries in flight -- per-query host timestamps (--step-trace)
# beside the library's own create_execute / finalize times (PGPU_TRACE=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
O=gpurun_out/r05s
mkdir -p $O
for i in 3 2; do
PGPU_TRACE=1 timeout -k 10 300 python -u bench.py --workload c4 --steps 30 --warmup 5 --inflight $i --no-cpu-baseline \
  --no-pmc --parity-segments 0 --host-profile --step-trace $O/steps_if$i.json > $O/c4_if$i.log 2>&1 || { tail -5 $O/c4_if$i.log; exit 1; }
tail -1 $O/c4_if$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('inflight', $i, d['ms_per_step'], d['host_profile_us'])"
done
# the sparse instances' 4-doc lane batches as built (C4 scan path, C3, indexed C3, C1)
for a in "--workload c4 --no-star-tree" "--workload adanalytics_inv" "--workload c1 --steps 200" ""; do
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-pmc $a > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  tail -1 $O/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a', d['ms_per_step'], d['roofline']['kernel_us'], d['roofline']['frac'], d['parity'] and d['parity']['ok'])"
done
