#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for sql in "SELECT COUNT(*) FROM t WHERE f < 500 GROUP BY d" "SELECT SUM(mi) FROM t WHERE f < 500 GROUP BY d" "SELECT SUM(md) FROM t WHERE f < 500 GROUP BY d" "SELECT COUNT(*), SUM(mi), MIN(mi), MAX(mi), SUM(md) FROM t WHERE f < 5 GROUP BY d" "SELECT COUNT(*) FROM t WHERE f < 500 GROUP BY mi"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --workload c2 --segments-per-gpu 100 --steps 10 --warmup 2 --no-pmc --no-cpu-baseline --sql "$sql" > gpurun_out/c2p_$i.log 2>&1 || { tail -5 gpurun_out/c2p_$i.log; exit 1; }
  echo "== $sql"; tail -1 gpurun_out/c2p_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(r['kernel_us'], r['frac'], r['bytes_alg_per_launch'])"
done
