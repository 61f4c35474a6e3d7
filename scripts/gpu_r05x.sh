#!/bin/bash
# r05 session x: 4-doc lane batches only in a pure-AND sparse instance of its own (plans of estimated selectivity >=
# 1/16): parity tests, then the driver's command twice and the final profile lines of C3, indexed C3, C1 and the C4
# scan path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05x
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
for run in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/driver_$run.log 2>&1 || { tail -5 $O/driver_$run.log; exit 1; }
  tail -1 $O/driver_$run.log > $O/driver_$run.json
  python -c "import json; d=json.load(open('$O/driver_$run.json')); r=d['roofline']; print('driver', d['ms_per_step'], d['latency_ms_per_query'], r['kernel_us'], r['frac'], r['traffic'], d['parity']['ok'], d['cpu_baseline']['value'])"
done
rm -rf gpurun_out/profiles
PMC=1 WL="adanalytics:1000 adanalytics_inv:1000 c1:1 c4:64:scan:--no-star-tree" bash scripts/gpu_profiles.sh
