#!/bin/bash
# Rehearsal of bench.py's multi-rank step on one GPU: `bench.py --gpus 2` starts its two ranks itself and the C ABI
# combine runs over the host transport (RCCL refuses two ranks per device).  Each line carries the N>1 parity leg
# (per-rank oracle results merged as the broker merges server responses): dense all-reduce (C3, C2, C4 star-tree),
# reduce-scatter (C5), hash-mode all-to-all (c5_hash), numGroupsLimit row exchange (C5 with a binding limit).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/mr
export PGPU_BENCH_BACKEND=host
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --gpus 2 --steps 3 --warmup 1 --warmup-ms 0 --no-cpu-baseline --no-pmc \
    --verify "$@" > gpurun_out/mr/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  grep '^{' gpurun_out/mr/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['parity']; print(' ', d['n_gpus'], d['ms_per_step'], d['config']['combine'], d['config']['groups'], 'parity', p['ok'], p['groups'], p.get('mismatch'))" || tail -5 gpurun_out/mr/$name.log
  return $rc
}
run c3 --workload adanalytics --rows-total 8000000 &&
run c2 --workload c2 --rows-total 4000000 &&
run c4 --workload c4 --rows-total 4000000 &&
run c5_rs --workload c5 --rows-total 4000000 &&
run c5_hash --workload c5_hash --rows-total 4000000 &&
run limit --workload c5 --rows-total 2000000 --num-groups-limit 100000
