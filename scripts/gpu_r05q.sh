#!/bin/bash
# r05 session q: C4 star-tree step of the round-4 tree (_r04tree, built from commit 5cd5ffb) against this tree, same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so _r04tree/pinot_amd/libpinotgpu*.so
O=$PWD/gpurun_out/r05q
mkdir -p $O
for rep in 1 2; do
  (cd _r04tree && timeout -k 10 300 python -u bench.py --workload c4 --steps 50 --warmup 5 --no-cpu-baseline --no-pmc \
    --parity-segments 0 > $O/r04_$rep.log 2>&1) || { tail -5 $O/r04_$rep.log; exit 1; }
  tail -1 $O/r04_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('r04', d['ms_per_step'], d['roofline']['kernel_us'], d['config'].get('queries_in_flight'))"
  timeout -k 10 300 python -u bench.py --workload c4 --steps 50 --warmup 5 --no-cpu-baseline --no-pmc \
    --parity-segments 0 --inflight 2 > $O/r05_$rep.log 2>&1 || { tail -5 $O/r05_$rep.log; exit 1; }
  tail -1 $O/r05_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('r05', d['ms_per_step'], d['roofline']['kernel_us'], d['config'].get('queries_in_flight'))"
done
