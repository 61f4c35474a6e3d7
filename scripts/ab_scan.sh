#!/bin/bash
# A/B of the staged (LDS-DMA) scan kernel against the register-direct kernel on the default bench workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 1 0; do
  PGPU_SCAN=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --host-profile ${BENCH_ARGS} > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  echo "scan=$v"; tail -1 gpurun_out/ab_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline'], d['host_profile_us'])"
done
