#!/bin/bash
# A/B of bench argument variants on one workload, interleaved.  VARIANTS is ';'-separated:
# VARIANTS="--config slot_weight_step=0.0;--config slot_weight_step=0.11" BENCH_ARGS="--workload c2"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
IFS=';' read -ra VS <<< "${VARIANTS:- }"
for rep in 1 2; do
  for v in "${VS[@]}"; do
    name=$(echo "${BENCH_ARGS}_$v" | tr -c 'A-Za-z0-9_=.,-' '_')_$rep
    timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-pmc ${BENCH_ARGS} $v > gpurun_out/ab/$name.log 2>&1 || { tail -5 gpurun_out/ab/$name.log; exit 1; }
    echo "[$v] $rep $(tail -1 gpurun_out/ab/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline'] or {}; print(d['ms_per_step'], r.get('kernel_us'), r.get('frac'), (d['parity'] or {}).get('ok'), 'latency', d.get('latency_ms_per_query'))")"
  done
done
