#!/bin/bash
# The GPU suite (PYTEST_K selects) then, if SEGS is set, the C3 series (scripts/gpu_series.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -2 gpurun_out/suite.log; grep -E "FAILED|Error" gpurun_out/suite.log | head -5
[ $rc -eq 0 ] || exit $rc
[ -z "$SEGS" ] || bash scripts/gpu_series.sh
