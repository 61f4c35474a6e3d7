#!/bin/bash
# The driver's bench command with per-query host timestamps, then the same command under a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
mkdir -p gpurun_out/tr
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --step-trace gpurun_out/tr/steps20.json ${BENCH_ARGS} > gpurun_out/tr/b20.log 2>&1 || exit 1
tail -1 gpurun_out/tr/b20.log | cut -c1-300
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 200 --warmup 5 --no-pmc --no-cpu-baseline --no-bytes --step-trace gpurun_out/tr/steps200.json ${BENCH_ARGS} > gpurun_out/tr/b200.log 2>&1 || exit 1
tail -1 gpurun_out/tr/b200.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/tr/prof -o run -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-bytes --step-trace gpurun_out/tr/steps20_prof.json ${BENCH_ARGS} > gpurun_out/tr/prof.log 2>&1
echo prof rc=$?
