#!/bin/bash
# r05 session i: workgroup start / loop-end / end times of the scan launches (diagnostics build
# PGPU_DIAG_WG_TIMES, PGPU_TRACE=wgtimes): how much of a C3 launch at 125 and 1000 segments is ramp, tail and
# static-split imbalance; C2 and the C4 scan path alike.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
run() {  # name, bench args
  local name=$1; shift
  PGPU_LIB=pinot_amd/libpinotgpu_diag_wgt.so PGPU_TRACE=wgtimes timeout -k 10 300 python -u bench.py --steps 4 \
    --warmup 2 --warmup-ms 0 --inflight 1 --roofline-steps 2 --no-cpu-baseline --no-pmc --no-bytes \
    --parity-segments 0 "$@" > $O/$name.log 2>&1 || { tail -5 $O/$name.log; return 1; }
  echo "== $name"; grep wgtimes $O/$name.log | tail -4
}
run c3_125 --segments-per-gpu 125 && run c3_1000 && run c2 --workload c2 --segments-per-gpu 100 && \
  run c4_scan --workload c4 --no-star-tree && run inv --workload adanalytics_inv
