#!/bin/bash
# r06 session w: confirmation on the round's final tree -- the whole GPU suite, smoke(), and the driver's command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so oracle/*.so
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > $O/driver.log 2>&1 || { tail -5 $O/driver.log; exit 1; }
tail -1 $O/driver.log > $O/r06_final_driver20_bench.json
python3 -c "import json; d=json.load(open('$O/r06_final_driver20_bench.json')); r=d['roofline']; print(d['ms_per_step'], d['latency_ms_per_query'], r['kernel_us'], r['frac'], r['traffic'], d['parity']['ok'], d['cpu_baseline']['value'])"
