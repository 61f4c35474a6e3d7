#!/bin/bash
# r05 session zh: queries in flight, 3 (the bench default) against 4 (= GPU_MAX_HW_QUEUES, one hardware queue each),
# interleaved, under the driver's step counts: C3 at 1 000 and 125 segments, C2, C4 (star-tree), C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05zh
mkdir -p $O
for spec in "c3:" "c3s125:--segments-per-gpu 125" "c2:--workload c2" "c4:--workload c4" "c5:--workload c5"; do
  n=${spec%%:*}; a=${spec#*:}
  for rep in 1 2; do
    for q in 3 4; do
      timeout -k 10 300 python -u bench.py $a --steps 20 --warmup 5 --inflight $q --no-pmc --no-cpu-baseline \
        --parity-segments 0 > $O/${n}_q${q}_$rep.log 2>&1 || { tail -5 $O/${n}_q${q}_$rep.log; exit 1; }
      tail -1 $O/${n}_q${q}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', 'inflight $q', d['ms_per_step'], d['latency_ms_per_query'])"
    done
  done
done
