#!/bin/bash
# r05 session l: scan grid oversubscription (pgpu_config.scan_grid_factor): parity tests, then A/B of the factor on
# C3 (1000 / 125 segments), indexed C3, C2, the C4 scan path and C1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_workloads_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
CONFIGS="scan_grid_factor=1 scan_grid_factor=2 scan_grid_factor=4 scan_grid_factor=8" TAG=c3 STEPS=100 \
  BENCH_ARGS="--parity-segments 1000" bash scripts/ab_cfg.sh || exit 1
CONFIGS="scan_grid_factor=1 scan_grid_factor=2 scan_grid_factor=4" TAG=c3s125 STEPS=200 \
  BENCH_ARGS="--segments-per-gpu 125" bash scripts/ab_cfg.sh || exit 1
CONFIGS="scan_grid_factor=1 scan_grid_factor=2 scan_grid_factor=4" TAG=inv BENCH_ARGS="--workload adanalytics_inv" bash scripts/ab_cfg.sh || exit 1
CONFIGS="scan_grid_factor=1 scan_grid_factor=2 scan_grid_factor=4" TAG=c2 BENCH_ARGS="--workload c2" bash scripts/ab_cfg.sh || exit 1
CONFIGS="scan_grid_factor=1 scan_grid_factor=2" TAG=c4s BENCH_ARGS="--workload c4 --no-star-tree" bash scripts/ab_cfg.sh || exit 1
CONFIGS="scan_grid_factor=1 scan_grid_factor=2" TAG=c1 STEPS=200 BENCH_ARGS="--workload c1" bash scripts/ab_cfg.sh || exit 1
