#!/bin/bash
# Parity tests + one bench line (+ optional staged-kernel A/B).  Stops at the first failing GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E 'FAILED|Error|assert' gpurun_out/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --host-profile ${BENCH_ARGS} > gpurun_out/bench_q.log 2>&1 || { tail -5 gpurun_out/bench_q.log; exit 1; }
tail -1 gpurun_out/bench_q.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline'], d['host_profile_us'])"
