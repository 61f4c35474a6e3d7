#!/bin/bash
# r05 final session: smoke() on the box, the driver's command twice and the C3 profile line of the final tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so oracle/*.so 2>/dev/null
export TMPDIR=/tmp
O=gpurun_out/r05final
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
for run in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/driver_$run.log 2>&1 || { tail -5 $O/driver_$run.log; exit 1; }
  tail -1 $O/driver_$run.log > $O/driver_$run.json
  python -c "import json; d=json.load(open('$O/driver_$run.json')); r=d['roofline']; print('driver', d['ms_per_step'], d['latency_ms_per_query'], r['kernel_us'], r['frac'], r['traffic'], d['parity']['ok'], d['cpu_baseline']['value'])"
done
rm -rf gpurun_out/profiles
PMC=1 WL="adanalytics:1000" bash scripts/gpu_profiles.sh
