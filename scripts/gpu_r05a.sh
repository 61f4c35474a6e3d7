#!/bin/bash
# r05 session a: bench.py's own rank launcher (--gpus 2 over the host transport, with the N>1 parity leg), the
# fail-fast path (--gpus 8 on a 1-GPU box), C3 at 125 segments (one rank's share at N=8) under the driver's command
# with its GPU timeline, then the whole GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
PGPU_BENCH_BACKEND=host timeout -k 10 400 python3 -u bench.py --gpus 2 --workload c2 --rows-total 4000000 \
  --steps 20 --warmup 5 > $O/mr_c2.log 2>&1
rc=$?; echo "mr c2 rc=$rc"; tail -2 $O/mr_c2.log | cut -c1-1500
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u bench.py --gpus 8 > $O/gpus8.log 2>&1
echo "gpus8 rc=$? (expected non-zero)"; tail -2 $O/gpus8.log
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --segments-per-gpu 125 --no-cpu-baseline \
  > $O/seg125.log 2>&1 || { tail -5 $O/seg125.log; exit 1; }
tail -1 $O/seg125.log | cut -c1-1500
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tl -o run -- python3 -u bench.py \
  --steps 20 --warmup 5 --segments-per-gpu 125 --no-cpu-baseline --no-pmc --no-bytes > $O/tl.log 2>&1
echo "timeline rc=$?"
python3 tools/timeline.py $(dirname $(find $O/tl -name run_kernel_trace.csv | head -1)) > $O/timeline.txt 2>&1; tail -30 $O/timeline.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; exit $rc
