#!/bin/bash
# Concurrency tests only (diagnostics run): PYTEST_K selects, e.g. "table"; PGPU_TRACE=crash prints native frames.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -s -v -x --timeout 120 --timeout-method thread tests/test_concurrency_gpu.py -m gpu ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/conc.log 2>&1
rc=$?; echo "conc rc=$rc"; grep -E "PASSED|FAILED|Error|mismatch|launch check|\[pgpu\]" gpurun_out/conc.log | head -60; exit $rc
