#!/bin/bash
# A/B of table executor settings (bench.py --config, pgpu_config fields) on one bench workload, interleaved.
# CONFIGS="scan_dynamic_pct=0 scan_dynamic_pct=30" BENCH_ARGS="--workload c2 --segments-per-gpu 100" TAG=x
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abc
for rep in 1 2; do
  for cfg in ${CONFIGS}; do
    name=${TAG:-ab}_$(echo $cfg | tr ',=' '__')_$rep
    timeout -k 10 300 python -u bench.py --steps ${STEPS:-50} --warmup 3 --no-cpu-baseline --no-pmc --config $cfg \
      ${BENCH_ARGS} > gpurun_out/abc/$name.log 2>&1 || { tail -5 gpurun_out/abc/$name.log; exit 1; }
    echo "$name $(tail -1 gpurun_out/abc/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline'] or {}; print(d['ms_per_step'], r.get('kernel_us'), d['parity'] and d['parity'].get('ok'))")"
  done
done
