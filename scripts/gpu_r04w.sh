#!/bin/bash
# r04 session w: the final tree -- the whole GPU suite, smoke, the driver's bench command twice, then C3 / indexed C3
# profiles with the pure-AND instance.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out/w
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/w/suite.log 2>&1
rc=$?
tail -3 gpurun_out/w/suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for i in 1 2; do
  timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/w/driver_$i.log 2>&1 || { tail -5 gpurun_out/w/driver_$i.log; exit 1; }
  tail -1 gpurun_out/w/driver_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('driver', d['ms_per_step'], r.get('kernel_us'), r['frac'], r.get('traffic'), d['parity']['ok'])"
done
WL="adanalytics:1000 adanalytics_inv:1000" PMC=1 WL_TIMEOUT=500 bash scripts/gpu_profiles.sh
