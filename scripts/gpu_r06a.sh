#!/bin/bash
# r06 session a: where a C3 launch's workgroups end (diagnostics build PGPU_DIAG_WG_TIMES, PGPU_TRACE=wgtimes: per
# XCD end times and the loop-end spread) at 125 and 1000 segments, then the driver's command on the round's first tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
run() {  # name, bench args
  local name=$1; shift
  PGPU_LIB=pinot_amd/libpinotgpu_diag_wgt.so PGPU_TRACE=wgtimes timeout -k 10 300 python -u bench.py --steps 6 \
    --warmup 2 --warmup-ms 0 --inflight 1 --roofline-steps 2 --no-cpu-baseline --no-pmc --no-bytes \
    --parity-segments 0 "$@" > $O/$name.log 2>&1 || { tail -5 $O/$name.log; return 1; }
  echo "== $name"; grep wgtimes $O/$name.log | tail -6
}
run c3_125 --segments-per-gpu 125 && run c3_1000 && \
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/driver.log 2>&1 && tail -1 $O/driver.log | cut -c1-400
