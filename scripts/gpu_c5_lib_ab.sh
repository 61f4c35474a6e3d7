#!/bin/bash
# C5: partition parity with the current library, then library A/B (LIBS) with per-kernel times of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c5
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_workloads_gpu.py -k "high_cardinality or finalize_key_range or c5" > gpurun_out/c5/tests.log 2>&1 || { tail -30 gpurun_out/c5/tests.log; exit 1; }
tail -1 gpurun_out/c5/tests.log
for lib in ${LIBS}; do
  n=$(basename $lib .so)
  PGPU_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5/prof_$n -o run -- python3 -u bench.py --workload c5 --segments-per-gpu 100 --steps 10 --warmup 2 --no-pmc --no-cpu-baseline --no-bytes > gpurun_out/c5/prof_$n.log 2>&1 || { tail -5 gpurun_out/c5/prof_$n.log; exit 1; }
  echo "== $n $(tail -1 gpurun_out/c5/prof_$n.log | cut -c1-200)"
  python3 - $n <<'PY'
import csv, glob, sys
f = glob.glob("gpurun_out/c5/prof_%s/**/*kernel_stats.csv" % sys.argv[1], recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "part" in r["Name"]: print("   %-50s avg %.1f us" % (r["Name"][:50], float(r["AverageNs"]) / 1e3))
PY
done
