#!/bin/bash
# Per-workload bench line (with CPU baseline) + rocprofv3 kernel-trace summary, for profiles/.
# WL="c1:1 c2:100 c4:64 c5:100" -- each spec is workload:segments[:tag[:flags]], flags with '+' for spaces and
# ENV=VALUE words exported for that run only (e.g. "c4:64:scan:--no-star-tree", "adanalytics:1000:nocache:PGPU_PLAN_CACHE=0").
# PMC=1 adds the FETCH_SIZE traffic passes; NOPROF=1 skips the rocprofv3 run, which runs one query at a time
# (--inflight 1) so its kernel durations are the serialized ones the roofline uses.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
touch pinot_amd/libpinotgpu*.so  # the prebuilt library is current
PMCFLAG=--no-pmc
[ -n "$PMC" ] && PMCFLAG=""

OUT=gpurun_out/profiles
mkdir -p $OUT
for spec in ${WL:-c1:1 c2:100 c4:64 c5:100}; do
  IFS=: read -r w n tag flags <<< "$spec"
  name=$w${tag:+_$tag}
  args=()
  envs=()
  for f in ${flags//+/ }; do
    if [[ $f == *=* && $f != --* ]]; then envs+=("$f"); else args+=("$f"); fi
  done
  (
    for e in "${envs[@]}"; do export "$e"; done
    timeout -k 10 ${WL_TIMEOUT:-400} python -u bench.py --workload $w --segments-per-gpu $n --steps ${STEPS:-20} --warmup ${WARMUP:-5} $PMCFLAG --host-profile "${args[@]}" > $OUT/${name}_bench.log 2>&1 || { echo "$name bench failed"; tail -5 $OUT/${name}_bench.log; exit 1; }
    tail -1 $OUT/${name}_bench.log > $OUT/${name}_bench.json
    echo "== $name $(python -c "import json; d=json.load(open('$OUT/${name}_bench.json')); r=d['roofline'] or {}; print(d['value'], d['ms_per_step'], r.get('kernel_us'), r.get('frac'), (d['cpu_baseline'] or {}).get('value'))")"
    [ -n "$NOPROF" ] && exit 0
    timeout -k 10 ${WL_TIMEOUT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$name -o run -- python3 -u bench.py --workload $w --segments-per-gpu $n --steps 10 --warmup 2 --inflight 1 --no-pmc --no-cpu-baseline --no-bytes "${args[@]}" > $OUT/${name}_prof.log 2>&1 || { echo "$name rocprof failed"; tail -5 $OUT/${name}_prof.log; exit 1; }
    exit 0
  ) || exit 1
done
