#!/bin/bash
# Scan-kernel time vs segment count (C3): bench lines without CPU baseline / PMC.  SEGS="125 250 500 1000".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/series
touch pinot_amd/libpinotgpu*.so
for n in ${SEGS:-125 250 500 1000}; do
  timeout -k 10 300 python -u bench.py --workload ${WL:-adanalytics} --segments-per-gpu $n --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-pmc ${ARGS} > gpurun_out/series/${WL:-adanalytics}_$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/series/${WL:-adanalytics}_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/series/${WL:-adanalytics}_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['ms_per_step'], r['kernel_us'], r['frac'])")"
done
