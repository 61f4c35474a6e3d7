#!/bin/bash
# A/B of host planning parallelism / streamed launches on C3 (whole-query ms per step).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "X=0" "PGPU_PLAN_CHUNK_SEGS=250" "PGPU_PLAN_CHUNK_SEGS=125" "PGPU_STREAM_CHUNKS=2" "PGPU_STREAM_CHUNKS=4"; do
  env $cfg timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-pmc --no-cpu-baseline --no-bytes --host-profile > gpurun_out/ab_plan.log 2>&1 || { tail -5 gpurun_out/ab_plan.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/ab_plan.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['host_profile_us'])")"
done
