#!/bin/bash
# r04 session y: SQ counter passes of the C3 scan (pure-AND instance), the indexed C3 scan (pair instance) and C5's
# partition pipeline -- where the next round's time goes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_BUSY_CYCLES"
TAG=c3 KREGEX=filter_groupby ARGS="--workload adanalytics --segments-per-gpu 250" PASSES="$P1;$P2" bash scripts/pmc_kernel.sh > gpurun_out/pmc_c3.txt 2>&1 || { tail -5 gpurun_out/pmc_c3.txt; exit 1; }
TAG=c3i KREGEX=filter_groupby ARGS="--workload adanalytics_inv --segments-per-gpu 250" PASSES="$P1;$P2" bash scripts/pmc_kernel.sh > gpurun_out/pmc_c3i.txt 2>&1 || { tail -5 gpurun_out/pmc_c3i.txt; exit 1; }
TAG=c5 KREGEX=part_ ARGS="--workload c5" PASSES="$P1;$P2" bash scripts/pmc_kernel.sh > gpurun_out/pmc_c5.txt 2>&1 || { tail -5 gpurun_out/pmc_c5.txt; exit 1; }
cat gpurun_out/pmc_c3.txt gpurun_out/pmc_c3i.txt gpurun_out/pmc_c5.txt
