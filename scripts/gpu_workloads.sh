#!/bin/bash
# One bench line per workload on one GPU: WL="c1:1 c2:100 c5:100 adanalytics:1000" (workload:segments).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in ${WL:-c1:1 c2:100 c5:100}; do
  w=${spec%%:*}; n=${spec##*:}
  timeout -k 10 ${WL_TIMEOUT:-400} python -u bench.py --workload $w --segments-per-gpu $n --steps ${STEPS:-10} --warmup 2 --no-pmc --host-profile ${EXTRA} > gpurun_out/wl_$w.log 2>&1 || { echo "$w failed"; tail -5 gpurun_out/wl_$w.log; exit 1; }
  echo "== $w"; tail -1 gpurun_out/wl_$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_us'], r['frac'], r['bytes_alg_per_launch'], d['config']['groups'], d['host_profile_us'], (d['cpu_baseline'] or {}).get('value'))"
done
