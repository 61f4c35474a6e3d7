#!/bin/bash
# r04 session h: queries in flight on the driver's command (C3), the c5_hash K8h table size / partition bits, a
# c5_hash kernel trace, then session c (C2 dense LDS forms, C5 record packing, C4 scan-path COUNT packing).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out/h
for rep in 1 2; do
  for inf in 2 3 4; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-bytes --no-cpu-baseline --inflight $inf \
      > gpurun_out/h/inflight${inf}_$rep.log 2>&1 || { tail -5 gpurun_out/h/inflight${inf}_$rep.log; exit 1; }
    echo "inflight $inf $(tail -1 gpurun_out/h/inflight${inf}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")"
  done
done
STEPS=10 VARIANTS="PGPU_X=0 PGPU_PART_HASH_LDS_KB=20,PGPU_PART_HASH_PBITS=14 PGPU_PART_HASH_LDS_KB=24 PGPU_PART_HASH_LDS_KB=56" \
  BENCH_ARGS="--workload c5_hash --no-bytes" bash scripts/ab_env.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/h/prof_c5h \
  -o run -- python3 -u bench.py --workload c5_hash --steps 5 --warmup 2 --warmup-ms 0 --no-bytes --no-pmc \
  --no-cpu-baseline --inflight 1 > gpurun_out/h/prof_c5h.log 2>&1 || { tail -5 gpurun_out/h/prof_c5h.log; exit 1; }
SKIP_TESTS=1 bash scripts/gpu_r04c.sh
