#!/bin/bash
# r05 session v: final profiles after the lane-batch / star-record changes -- the driver's command twice, then C3,
# indexed C3, C1, C4 star and scan paths (CPU baselines, FETCH_SIZE traffic, serialized rocprofv3 summaries).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05v
mkdir -p $O
for run in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/driver_$run.log 2>&1 || { tail -5 $O/driver_$run.log; exit 1; }
  tail -1 $O/driver_$run.log > $O/driver_$run.json
  python -c "import json; d=json.load(open('$O/driver_$run.json')); r=d['roofline']; print('driver', d['ms_per_step'], d['latency_ms_per_query'], r['kernel_us'], r['frac'], r['traffic'], d['parity']['ok'], d['cpu_baseline']['value'])"
done
rm -rf gpurun_out/profiles
PMC=1 WL="adanalytics:1000 adanalytics_inv:1000 c1:1 c4:64 c4:64:scan:--no-star-tree" bash scripts/gpu_profiles.sh
