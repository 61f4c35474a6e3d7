#!/bin/bash
# r04 session y: the dense-instance threshold (parity, C4 scan A/B), then SQ counter passes of the C3 scan (pure-AND instance), the indexed C3 scan (pair instance) and C5's
# partition pipeline -- where the next round's time goes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out/y
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_workloads_gpu.py tests/test_orderby_gpu.py \
  tests/test_startree_gpu.py tests/test_concurrency_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/y/suite.log 2>&1
rc=$?
tail -3 gpurun_out/y/suite.log
[ $rc -eq 0 ] || exit $rc
# the dense-instance threshold (1/4) against the previous 1/16
VARIANTS="PGPU_X=0 PGPU_DENSE_SEL=0.0625" BENCH_ARGS="--workload c4 --segments-per-gpu 64 --no-star-tree" bash scripts/ab_env.sh || exit 1
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_BUSY_CYCLES"
TAG=c3 KREGEX=filter_groupby ARGS="--workload adanalytics --segments-per-gpu 250" PASSES="$P1;$P2" bash scripts/pmc_kernel.sh > gpurun_out/pmc_c3.txt 2>&1 || { tail -5 gpurun_out/pmc_c3.txt; exit 1; }
TAG=c3i KREGEX=filter_groupby ARGS="--workload adanalytics_inv --segments-per-gpu 250" PASSES="$P1;$P2" bash scripts/pmc_kernel.sh > gpurun_out/pmc_c3i.txt 2>&1 || { tail -5 gpurun_out/pmc_c3i.txt; exit 1; }
TAG=c5 KREGEX=part_ ARGS="--workload c5" PASSES="$P1;$P2" bash scripts/pmc_kernel.sh > gpurun_out/pmc_c5.txt 2>&1 || { tail -5 gpurun_out/pmc_c5.txt; exit 1; }
cat gpurun_out/pmc_c3.txt gpurun_out/pmc_c3i.txt gpurun_out/pmc_c5.txt
