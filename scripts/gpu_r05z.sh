#!/bin/bash
# r05 session z: leap-frog statistics summed per block before the one atomic (was one per segment): tests that assert
# the statistic, the C3 epilogue time at 125 / 1000 segments (rocprofv3), and the driver's command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05z
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_workloads_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for n in 125 1000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$n -o run -- python3 -u bench.py \
    --segments-per-gpu $n --steps 20 --warmup 3 --inflight 1 --no-pmc --no-cpu-baseline --no-bytes --parity-segments 0 > $O/p_$n.log 2>&1 || { tail -5 $O/p_$n.log; exit 1; }
  python - "$O/p_$n" <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0])))
keep = [r for r in rows if any(k in r["Name"] for k in ("filter_groupby", "epilogue"))]
print(sys.argv[1], " | ".join("%s x%s %.1f" % (r["Name"][:28], r["Calls"], float(r["AverageNs"]) / 1000) for r in keep))
PY
done
for run in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/driver_$run.log 2>&1 || { tail -5 $O/driver_$run.log; exit 1; }
  tail -1 $O/driver_$run.log > $O/driver_$run.json
  python -c "import json; d=json.load(open('$O/driver_$run.json')); r=d['roofline']; print('driver', d['ms_per_step'], d['latency_ms_per_query'], r['kernel_us'], r['frac'], r['traffic'], d['parity']['ok'], d['cpu_baseline']['value'])"
done
timeout -k 10 300 python -u bench.py --segments-per-gpu 125 --steps 20 --warmup 5 --no-cpu-baseline --no-pmc > $O/s125.log 2>&1 || { tail -5 $O/s125.log; exit 1; }
tail -1 $O/s125.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('125 segments', d['ms_per_step'], d['roofline']['kernel_us'], d['parity']['ok'])"
