#!/bin/bash
# r06 session zj: SQ counters of the scan kernel on the round's last tree (rocprofv3 --pmc, one pass each): C2's dense
# instance and C3's sparse one (wave cycles waiting / issuing, VALU / VMEM / LDS instructions, LDS bank conflicts).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r06_c2 KREGEX="filter_groupby" ARGS="--workload c2" timeout -k 10 300 bash scripts/pmc_kernel.sh > gpurun_out/r06_c2_pmc_sq.txt 2>&1 || { tail -5 gpurun_out/r06_c2_pmc_sq.txt; exit 1; }
cat gpurun_out/r06_c2_pmc_sq.txt | cut -c1-150
TAG=r06_c3 KREGEX="filter_groupby" ARGS="--workload adanalytics --segments-per-gpu 250" timeout -k 10 300 bash scripts/pmc_kernel.sh > gpurun_out/r06_c3_pmc_sq.txt 2>&1 || { tail -5 gpurun_out/r06_c3_pmc_sq.txt; exit 1; }
cat gpurun_out/r06_c3_pmc_sq.txt | cut -c1-150
