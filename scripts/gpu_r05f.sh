#!/bin/bash
# r05 session f: K8d's COUNT + SUM word table in 32 KB of LDS (four workgroups per CU), chunked -- partition tests,
# then A/B against the full-LDS build (PGPU_PART_CS_FULL_LDS) on C5, then SQ counters of C5's four kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_hash_partition_gpu.py tests/test_workloads_gpu.py \
  tests/test_timeout_gpu.py tests/test_multi_rank_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_csfull.so" BENCH_ARGS="--workload c5 --segments-per-gpu 100" \
  bash scripts/ab_lib.sh || exit 1
TAG=c5sq KREGEX="part_" ARGS="--workload c5 --segments-per-gpu 100 --inflight 1 --no-bytes --parity-segments 0" \
  PASSES="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
  bash scripts/pmc_kernel.sh > $O/c5_sq.txt 2>&1; tail -40 $O/c5_sq.txt
# C2: L2 hits / misses and memory read requests of the dense scan, with and without the md dictionary gathers
for lib in libpinotgpu libpinotgpu_ab_nodval; do
  PGPU_LIB=pinot_amd/$lib.so TAG=c2_$lib KREGEX="filter_groupby" \
    ARGS="--workload c2 --segments-per-gpu 100 --inflight 1 --no-bytes --parity-segments 0" \
    PASSES="TCC_HIT_sum TCC_MISS_sum;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum;SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD" \
    bash scripts/pmc_kernel.sh > $O/c2_tcc_$lib.txt 2>&1; tail -12 $O/c2_tcc_$lib.txt
done
