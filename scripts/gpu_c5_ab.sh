#!/bin/bash
# C5 partition pipeline: parity of the partitioned paths, env A/B, and a kernel-trace summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c5
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_workloads_gpu.py -k "high_cardinality or finalize_key_range or c5" > gpurun_out/c5/tests.log 2>&1 || { tail -30 gpurun_out/c5/tests.log; exit 1; }
tail -2 gpurun_out/c5/tests.log
VARIANTS="${VARIANTS:-PGPU_PART_VAL64=1 PGPU_X=0}" BENCH_ARGS="--workload c5 --segments-per-gpu 100" STEPS=10 bash scripts/ab_env.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5/prof -o run -- python3 -u bench.py --workload c5 --segments-per-gpu 100 --steps 10 --warmup 2 --no-pmc --no-cpu-baseline --no-bytes > gpurun_out/c5/prof.log 2>&1 || { tail -5 gpurun_out/c5/prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/c5/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if float(r["Percentage"]) > 1: print("%-60s %8s calls avg %.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
