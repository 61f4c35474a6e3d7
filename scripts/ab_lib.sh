#!/bin/bash
# A/B of library variants (pinot_amd/build.py build(defines=..., out=...)) on one bench workload, interleaved.
# LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab0.so" BENCH_ARGS="--workload c2 --segments-per-gpu 100"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for lib in ${LIBS:-pinot_amd/libpinotgpu.so}; do
    name=$(basename $lib .so)_$rep
    PGPU_LIB=$lib timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-pmc ${BENCH_ARGS} > gpurun_out/ab/$name.log 2>&1 || { tail -5 gpurun_out/ab/$name.log; exit 1; }
    echo "$name $(tail -1 gpurun_out/ab/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline'] or {}; print(d['ms_per_step'], r.get('kernel_us'), (d['parity'] or {}).get('ok'), 'latency', d.get('latency_ms_per_query'))")"
  done
done
