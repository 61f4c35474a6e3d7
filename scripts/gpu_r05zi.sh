#!/bin/bash
# r05 session zi: SQ counters (one pass each) of the scan kernel on the round's last tree: C3, indexed C3, C2, the C4
# scan path -- wave cycles waiting / issuing, VMEM / LDS instructions, LDS bank conflicts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for spec in "c3:" "c3inv:--workload adanalytics_inv" "c2:--workload c2" "c4s:--workload c4 --no-star-tree"; do
  n=${spec%%:*}; a=${spec#*:}
  TAG=r05zi_$n KREGEX="filter_groupby" ARGS="$a --parity-segments 0" timeout -k 10 300 bash scripts/pmc_kernel.sh \
    > gpurun_out/r05zi_$n.txt 2>&1 || { tail -5 gpurun_out/r05zi_$n.txt; exit 1; }
  grep -E "SQ_WAVE_CYCLES|SQ_WAIT_ANY|SQ_LDS_BANK" gpurun_out/r05zi_$n.txt | head -6
done
