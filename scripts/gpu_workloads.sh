#!/bin/bash
# One bench line per workload (C1, C2, C5; C3 = default) on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "c1 1" "c2 100" "c5 100" "adanalytics 1000"; do
  set -- $spec
  timeout -k 10 400 python -u bench.py --workload $1 --segments-per-gpu $2 --steps 10 --warmup 2 --no-pmc --host-profile ${EXTRA} > gpurun_out/wl_$1.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/wl_$1.log; exit 1; }
  echo "== $1"; tail -1 gpurun_out/wl_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_us'], r['frac'], r['bytes_alg_per_launch'], d['config']['groups'], d['host_profile_us'], (d['cpu_baseline'] or {}).get('value'))"
done
