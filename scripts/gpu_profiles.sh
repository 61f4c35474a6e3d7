#!/bin/bash
# Per-workload bench line (with CPU baseline) + rocprofv3 kernel-trace summary, for profiles/.
# WL="c1:1 c2:100 c4:64 c5:100" (workload:segments per GPU); PMC=1 adds the FETCH_SIZE traffic passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
touch pinot_amd/libpinotgpu*.so  # the prebuilt library is current
PMCFLAG=--no-pmc
[ -n "$PMC" ] && PMCFLAG=""

OUT=gpurun_out/profiles
mkdir -p $OUT
for spec in ${WL:-c1:1 c2:100 c4:64 c5:100}; do
  w=${spec%%:*}; n=${spec##*:}
  timeout -k 10 ${WL_TIMEOUT:-400} python -u bench.py --workload $w --segments-per-gpu $n --steps ${STEPS:-20} --warmup 3 $PMCFLAG --host-profile > $OUT/${w}_bench.log 2>&1 || { echo "$w bench failed"; tail -5 $OUT/${w}_bench.log; exit 1; }
  tail -1 $OUT/${w}_bench.log > $OUT/${w}_bench.json
  echo "== $w $(python -c "import json; d=json.load(open('$OUT/${w}_bench.json')); r=d['roofline'] or {}; print(d['value'], d['ms_per_step'], r.get('kernel_us'), r.get('frac'), (d['cpu_baseline'] or {}).get('value'))")"
  timeout -k 10 ${WL_TIMEOUT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$w -o run -- python3 -u bench.py --workload $w --segments-per-gpu $n --steps 10 --warmup 2 --no-pmc --no-cpu-baseline --no-bytes > $OUT/${w}_prof.log 2>&1 || { echo "$w rocprof failed"; tail -5 $OUT/${w}_prof.log; exit 1; }
done
