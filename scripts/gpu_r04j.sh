#!/bin/bash
# r04 session j: C1's host path (three 200-step runs with per-phase host times), then the round's profiles part 2
# (C4 star-tree and scan paths, C5, c5_hash).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out/j
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --workload c1 --steps 200 --warmup 5 --no-pmc --no-cpu-baseline --no-bytes \
    --host-profile > gpurun_out/j/c1_$i.log 2>&1 || { tail -5 gpurun_out/j/c1_$i.log; exit 1; }
  tail -1 gpurun_out/j/c1_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1', d['ms_per_step'], d['host_profile_us'])"
done
bash scripts/gpu_r04e.sh
