#!/bin/bash
# r05 session zf: the slab fold with 128 lanes per table word (one round of loads for 1 024 slabs): the whole GPU suite,
# the C3 epilogue at 125 / 1000 segments and the C4 scan path's (rocprofv3), the driver's command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05zf
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
for spec in "125:--segments-per-gpu 125" "1000:--segments-per-gpu 1000" "c4s:--workload c4 --no-star-tree" "c2:--workload c2"; do
  n=${spec%%:*}; a=${spec#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$n -o run -- python3 -u bench.py \
    $a --steps 20 --warmup 3 --inflight 1 --no-pmc --no-cpu-baseline --no-bytes --parity-segments 0 > $O/p_$n.log 2>&1 || { tail -5 $O/p_$n.log; exit 1; }
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
timeout -k 10 300 python -u bench.py --segments-per-gpu 125 --steps 200 --warmup 5 --no-cpu-baseline --no-pmc > $O/s125.log 2>&1 || { tail -5 $O/s125.log; exit 1; }
tail -1 $O/s125.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('125 segments, 200 steps', d['ms_per_step'], d['roofline']['kernel_us'])"
