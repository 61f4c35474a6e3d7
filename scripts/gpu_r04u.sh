#!/bin/bash
# r04 session u: where C2's and C4-scan's dense scans spend their wave cycles (SQ counters, two passes each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_BUSY_CYCLES"
TAG=c2 KREGEX=filter_groupby ARGS="--workload c2" PASSES="$P1;$P2" bash scripts/pmc_kernel.sh > gpurun_out/pmc_c2.txt 2>&1 || { tail -5 gpurun_out/pmc_c2.txt; exit 1; }
TAG=c4s KREGEX=filter_groupby ARGS="--workload c4 --segments-per-gpu 64 --no-star-tree" PASSES="$P1;$P2" bash scripts/pmc_kernel.sh > gpurun_out/pmc_c4s.txt 2>&1 || { tail -5 gpurun_out/pmc_c4s.txt; exit 1; }
cat gpurun_out/pmc_c2.txt gpurun_out/pmc_c4s.txt
