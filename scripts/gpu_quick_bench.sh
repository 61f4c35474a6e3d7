#!/bin/bash
# Quick per-workload bench lines (no CPU baseline, no PMC): WL="adanalytics:1000 c2:100 c1:1".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/quick
mkdir -p $OUT
for spec in ${WL:-adanalytics:1000 c2:100 c1:1}; do
  w=${spec%%:*}; n=${spec##*:}
  timeout -k 10 ${WL_TIMEOUT:-300} python -u bench.py --workload $w --segments-per-gpu $n --steps ${STEPS:-20} --warmup 3 --no-pmc --no-cpu-baseline --host-profile ${EXTRA} > $OUT/${w}.log 2>&1 || { echo "$w failed"; tail -5 $OUT/${w}.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/${w}.log').read().strip().splitlines()[-1]); r=d['roofline'] or {}; print('$w', d['ms_per_step'], r.get('kernel_us'), r.get('frac'), d.get('host_profile_us'))"
done
