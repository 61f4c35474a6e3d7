#!/bin/bash
# The GPU suite, then the multi-rank bench rehearsal (scripts/gpu_mr_bench.sh); the first failure stops.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/suite.log; grep -E "FAILED|Error" gpurun_out/suite.log | head -5
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_mr_bench.sh
