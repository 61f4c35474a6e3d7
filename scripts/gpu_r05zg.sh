#!/bin/bash
# r05 session zg: confirmation on the round's last tree -- the whole GPU suite, smoke(), the driver's command twice
# (with its rocprofv3 kernel summary), C3 at 125 segments (200 steps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05zg
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for run in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/driver_$run.log 2>&1 || { tail -5 $O/driver_$run.log; exit 1; }
  tail -1 $O/driver_$run.log > $O/driver_$run.json
  python -c "import json; d=json.load(open('$O/driver_$run.json')); r=d['roofline']; print('driver', d['ms_per_step'], d['latency_ms_per_query'], r['kernel_us'], r['frac'], r['traffic'], d['parity']['ok'], d['cpu_baseline']['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py \
  --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --parity-segments 0 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
cp "$(find $O/prof -name run_kernel_stats.csv | head -1)" $O/driver_kernel_stats.csv
timeout -k 10 300 python -u bench.py --segments-per-gpu 125 --steps 200 --warmup 5 --no-cpu-baseline --no-pmc > $O/s125.log 2>&1 || { tail -5 $O/s125.log; exit 1; }
tail -1 $O/s125.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('125 segments, 200 steps', d['ms_per_step'], d['roofline']['kernel_us'])"
