#!/bin/bash
# r06 session g: chunked scans weighted by CU slot (KParams.slot_w) -- the diagnostics build's per-workgroup loop ends
# with the default weights, then an interleaved A/B of the weights (PGPU_SLOT_WEIGHTS; "1" = equal shares) on C3 at
# 125 / 1000 segments and indexed C3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
run() {  # name, bench args
  local name=$1; shift
  PGPU_LIB=pinot_amd/libpinotgpu_diag_wgt.so PGPU_TRACE=wgtimes PGPU_WGTIMES_OUT=$O/$name.wg timeout -k 10 300 \
    python -u bench.py --steps 4 --warmup 2 --warmup-ms 0 --inflight 1 --roofline-steps 1 --no-cpu-baseline --no-pmc \
    --no-bytes --parity-segments 0 "$@" > $O/$name.log 2>&1 || { tail -5 $O/$name.log; return 1; }
  echo "== $name"; grep wgtimes $O/$name.log | tail -2 | cut -c1-300
}
run c3_125 --segments-per-gpu 125 && run c3_1000 || exit 1
ENVS="PGPU_SLOT_WEIGHTS=1 PGPU_X=0 PGPU_SLOT_WEIGHTS=1.4,1.25,1.1,1 PGPU_SLOT_WEIGHTS=1.15,1.1,1.05,1"
for spec in "c3_125:--segments-per-gpu 125" "c3_1000:" "c3inv:--workload adanalytics_inv"; do
  n=${spec%%:*}; a=${spec#*:}
  echo "== $n"
  ENVS="$ENVS" BENCH_ARGS="$a" timeout -k 10 900 bash scripts/ab_env.sh || exit 1
done
