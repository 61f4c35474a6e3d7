#!/bin/bash
# A/B of environment settings of one library on one bench workload, interleaved.
# ENVS="PGPU_SLOT_WEIGHTS=1 PGPU_X=0" BENCH_ARGS="--workload c2"  (PGPU_X=0: an unused variable -- the defaults)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for e in ${ENVS:-PGPU_X=0}; do
    name=$(echo "${BENCH_ARGS}_$e" | tr -c 'A-Za-z0-9_=.,-' '_')_$rep
    env $e timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-pmc ${BENCH_ARGS} > gpurun_out/ab/$name.log 2>&1 || { tail -5 gpurun_out/ab/$name.log; exit 1; }
    echo "$e $rep $(tail -1 gpurun_out/ab/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline'] or {}; print(d['ms_per_step'], r.get('kernel_us'), r.get('frac'), (d['parity'] or {}).get('ok'), 'latency', d.get('latency_ms_per_query'))")"
  done
done
