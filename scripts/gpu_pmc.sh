#!/bin/bash
# HBM traffic of the scan kernel from PMC counters: FETCH_SIZE on the bench query and on a calibration query whose
# algorithmic bytes are all one fully-read column (accountId = rarest id: ~no matches), each in its own pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SEGS=${SEGS:-1000}
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_main -o main -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --segments-per-gpu $SEGS > gpurun_out/pmc_main.log 2>&1 || { tail -5 gpurun_out/pmc_main.log; exit 1; }
tail -1 gpurun_out/pmc_main.log
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_calib -o calib -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --segments-per-gpu $SEGS --sql "SELECT sum(clicks) FROM AdAnalyticsTable WHERE accountId = 4699963 GROUP BY daysSinceEpoch" > gpurun_out/pmc_calib.log 2>&1 || { tail -5 gpurun_out/pmc_calib.log; exit 1; }
tail -1 gpurun_out/pmc_calib.log
find gpurun_out/pmc_main gpurun_out/pmc_calib -name '*.csv' | head
