#!/bin/bash
# A/B of environment knobs on one bench workload, interleaved twice:
# VARIANTS="PGPU_DICT_GATHERS=0 PGPU_DICT_GATHERS=1" BENCH_ARGS="--workload c2 --segments-per-gpu 100"
# (a variant may set several variables joined by commas: "A=1,B=2")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
touch pinot_amd/libpinotgpu*.so
tag=$(echo "${BENCH_ARGS:-default}" | tr -c 'a-zA-Z0-9' '_')
for rep in 1 2; do
  for v in ${VARIANTS}; do
    name=${tag}_${v}_$rep
    env ${v//,/ } timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-pmc ${BENCH_ARGS} > gpurun_out/ab/$name.log 2>&1 || { tail -5 gpurun_out/ab/$name.log; exit 1; }
    echo "$name $(tail -1 gpurun_out/ab/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline'] or {}; print(d['ms_per_step'], r.get('kernel_us'), r.get('frac'))")"
  done
done
