#!/bin/bash
# Rehearsal of bench.py's multi-rank step on one GPU (2 ranks, the C ABI combine over the host transport):
# dense all-reduce (C2), reduce-scatter (C5), hash-mode all-to-all (C5 key + m: 10^10 keys), numGroupsLimit row
# exchange (C1 by filt, metric: 10^7 keys per segment).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PGPU_BENCH_BACKEND=host
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29600 + RANDOM % 200)) bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-bytes \
    --verify "$@" > gpurun_out/mr_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep '^{' gpurun_out/mr_$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['config']['combine'], d['config']['groups'])" || tail -5 gpurun_out/mr_$name.log
  return $rc
}
run dense --workload c2 --rows-total 4000000 &&
run rs --workload c5 --rows-total 2000000 &&
run hash --workload c5 --rows-total 2000000 --num-groups-limit 1000000000 --sql "SELECT SUM(m), COUNT(*) FROM t GROUP BY k1, k3, m" &&
run limit --workload c5 --rows-total 2000000 --sql "SELECT SUM(m), COUNT(*) FROM t GROUP BY k1, k2, k3, m" &&
run rows --workload c1 --rows-total 2000000 --sql "SELECT SUM(metric), COUNT(*) FROM t GROUP BY filt, metric"
