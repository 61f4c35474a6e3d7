#!/bin/bash
# r06 session zf: confirmation on the round's final tree after sessions z-ze (the GPU suite ran in session ze on the
# same library): smoke(), the driver's command, C3's 125-segment share with parity.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so oracle/*.so
export TMPDIR=/tmp
O=gpurun_out/r06zf
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > $O/driver.log 2>&1 || { tail -5 $O/driver.log; exit 1; }
tail -1 $O/driver.log > $O/r06_final2_driver20_bench.json
timeout -k 10 400 python -u bench.py --segments-per-gpu 125 --steps 20 --warmup 5 > $O/c125.log 2>&1 || { tail -5 $O/c125.log; exit 1; }
tail -1 $O/c125.log > $O/r06_final2_adanalytics_seg125_1gpu_bench.json
for f in $O/r06_final2_*.json; do python3 -c "import json; d=json.load(open('$f')); r=d['roofline']; print('$f', d['ms_per_step'], d['latency_ms_per_query'], r['kernel_us'], r['frac'], r['traffic'], d['parity']['ok'], d['cpu_baseline']['value'])"; done
