#!/bin/bash
# Kernel time of query variants over one workload's table: SQLS="q1|q2|..." WLD=c2 NSEG=100
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS='|' read -ra QS <<< "${SQLS}"
i=0
for sql in "${QS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --workload ${WLD:-c2} --segments-per-gpu ${NSEG:-100} --steps 10 --warmup 2 --no-pmc --no-cpu-baseline ${EXTRA} --sql "$sql" > gpurun_out/probe_$i.log 2>&1 || { tail -5 gpurun_out/probe_$i.log; exit 1; }
  echo "== $sql"; tail -1 gpurun_out/probe_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline'] or {}; print('kernel_us', r.get('kernel_us'), 'frac', r.get('frac'), 'ms/step', d['ms_per_step'])"
done
