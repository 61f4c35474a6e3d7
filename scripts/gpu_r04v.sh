#!/bin/bash
# r04 session v: dense instance with staged columns (LDS-DMA at the tile's start) -- parity, then C2 and the C4 scan
# path against PGPU_NO_STAGE=1, then C2's full-size parity line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out/v
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_workloads_gpu.py tests/test_orderby_gpu.py \
  tests/test_startree_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v/suite.log 2>&1
rc=$?
tail -3 gpurun_out/v/suite.log
[ $rc -eq 0 ] || exit $rc
VARIANTS="PGPU_X=0 PGPU_NO_STAGE=1" BENCH_ARGS="--workload c2" bash scripts/ab_env.sh || exit 1
VARIANTS="PGPU_X=0 PGPU_NO_STAGE=1" BENCH_ARGS="--workload c4 --segments-per-gpu 64 --no-star-tree" bash scripts/ab_env.sh || exit 1
timeout -k 10 600 python -u bench.py --workload c2 --no-pmc > gpurun_out/v/c2_full.log 2>&1 || { tail -5 gpurun_out/v/c2_full.log; exit 1; }
tail -1 gpurun_out/v/c2_full.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 full', d['ms_per_step'], d['roofline']['frac'], d.get('parity'))"
