#!/bin/bash
# r06 profile set: per workload one bench line (PMC traffic passes included) and a rocprofv3 kernel-statistics run of
# the same command (--no-pmc), into gpurun_out/final/.  PART=1: the driver's command (C3, 1000 segments, CPU baseline
# and full-size parity), C3 at 125 segments, indexed C3, C1, C2; PART=2: C4 star / scan (64 and 8 segments), C5
# (100 and 13 segments), c5_hash.  PROF_ONLY=1: the kernel-statistics runs only;
# BENCH_ONLY=1: the bench lines only; NOCPU="": every line with its CPU baseline and full-size parity.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NOCPU=${NOCPU---no-cpu-baseline}
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
if [ -n "$ONLY" ]; then
  SPECS="$ONLY"
elif [ "${PART:-1}" = 1 ]; then
  SPECS="adanalytics:;adanalytics_seg125:--segments-per-gpu 125 $NOCPU;adanalytics_inv:--workload adanalytics_inv $NOCPU;c1:--workload c1 $NOCPU;c2:--workload c2 $NOCPU"
else
  SPECS="c4:--workload c4 $NOCPU;c4_scan:--workload c4 --no-star-tree $NOCPU;c4_seg8:--workload c4 --segments-per-gpu 8 $NOCPU;c4_scan_seg8:--workload c4 --no-star-tree --segments-per-gpu 8 $NOCPU;c5:--workload c5 $NOCPU;c5_seg13:--workload c5 --segments-per-gpu 13 $NOCPU;c5_hash:--workload c5_hash $NOCPU"
fi
IFS=';' read -ra SL <<< "$SPECS"
for spec in "${SL[@]}"; do
  n=${spec%%:*}; a=${spec#*:}
  if [ -z "$PROF_ONLY" ]; then
    timeout -k 10 420 python -u bench.py $a --steps 20 --warmup 5 > $O/${n}_bench.log 2>&1 || { tail -5 $O/${n}_bench.log; exit 1; }
    tail -1 $O/${n}_bench.log > $O/r06_${n}_1gpu_bench.json
  fi
  [ -n "$BENCH_ONLY" ] && { echo "== $n $(tail -c 300 $O/r06_${n}_1gpu_bench.json)"; continue; }
  # one query in flight: each kernel's duration is its own (the bench line's kernel_us comes from such a pass)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$n -o run -- python3 -u bench.py $a \
    --steps 20 --warmup 5 --inflight 1 --no-pmc --parity-segments 0 > $O/${n}_prof.log 2>&1 || { tail -5 $O/${n}_prof.log; exit 1; }
  cp $(find $O/prof_$n -name run_kernel_stats.csv) $O/r06_${n}_1gpu_kernel_stats.csv
  echo "== $n $(python3 -c "import json; d=json.load(open('$O/r06_${n}_1gpu_bench.json')); r=d['roofline'] or {}; print(d['ms_per_step'], d.get('latency_ms_per_query'), r.get('kernel_us'), r.get('frac'), r.get('traffic'), r.get('bytes_alg_per_launch'), (d.get('parity') or {}).get('ok'), (d.get('cpu_baseline') or {}).get('value'))")"
done
