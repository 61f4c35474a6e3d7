#!/bin/bash
# r06 session e: the whole GPU suite on the split runtime with opt-in timing events (PGPU_OPT_TIMING), the driver's
# default bench command, C3 at 125 segments (bench line with PMC traffic + rocprofv3 kernel statistics).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > $O/driver.log 2>&1 || { tail -5 $O/driver.log; exit 1; }
tail -1 $O/driver.log | cut -c1-400
timeout -k 10 300 python -u bench.py --segments-per-gpu 125 --steps 20 --warmup 3 --no-cpu-baseline \
  > $O/c3_125.log 2>&1 || { tail -5 $O/c3_125.log; exit 1; }
tail -1 $O/c3_125.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof125 -o run -- python3 -u bench.py --segments-per-gpu 125 \
  --steps 20 --warmup 3 --no-cpu-baseline --no-pmc > $O/prof125.log 2>&1 || { tail -5 $O/prof125.log; exit 1; }
f=$(find $O/prof125 -name "run_kernel_stats.csv")
head -6 $f | cut -c1-200
