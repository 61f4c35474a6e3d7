#!/bin/bash
# r05 session k: the scan's dynamic tail (claimed wave-tiles): the whole GPU suite, A/B of scan_dynamic_pct on
# C3 (1000 and 125 segments), indexed C3, C2 and the C4 scan path, workgroup end times with the tail.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
CONFIGS="scan_dynamic_pct=0 scan_dynamic_pct=20 scan_dynamic_pct=30 scan_dynamic_pct=45" TAG=c3 STEPS=100 \
  BENCH_ARGS="--parity-segments 1000" bash scripts/ab_cfg.sh || exit 1
CONFIGS="scan_dynamic_pct=0 scan_dynamic_pct=30 scan_dynamic_pct=45" TAG=c3s125 STEPS=200 \
  BENCH_ARGS="--segments-per-gpu 125" bash scripts/ab_cfg.sh || exit 1
CONFIGS="scan_dynamic_pct=0 scan_dynamic_pct=30" TAG=inv BENCH_ARGS="--workload adanalytics_inv" bash scripts/ab_cfg.sh || exit 1
CONFIGS="scan_dynamic_pct=0 scan_dynamic_pct=30" TAG=c2 BENCH_ARGS="--workload c2" bash scripts/ab_cfg.sh || exit 1
CONFIGS="scan_dynamic_pct=0 scan_dynamic_pct=30" TAG=c4s BENCH_ARGS="--workload c4 --no-star-tree" bash scripts/ab_cfg.sh || exit 1
PGPU_LIB=pinot_amd/libpinotgpu_diag_wgt.so PGPU_TRACE=wgtimes timeout -k 10 300 python -u bench.py --steps 4 \
    --warmup 2 --warmup-ms 0 --inflight 1 --roofline-steps 2 --no-cpu-baseline --no-pmc --no-bytes \
    --parity-segments 0 > $O/wgt_c3.log 2>&1 || { tail -5 $O/wgt_c3.log; exit 1; }
grep wgtimes $O/wgt_c3.log | tail -3
