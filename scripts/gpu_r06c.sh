#!/bin/bash
# r06 session c: the new GPU tests (range-index leaves, communicator recreate, hash-result trims), the host / device
# timeline of one C3 query at 125 segments (PGPU_TRACE=1 marks, rocprofv3 kernel + copy trace), and the dense
# instance at 4 waves per SIMD (PGPU_DENSE_MIN_WAVES=4: 128 VGPRs, 18 spilled, since the record reads became scalar)
# against 3 on C2 and the C4 scan path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_range_index_gpu.py tests/test_hash_partition_gpu.py \
  "tests/test_multi_rank_gpu.py::test_comm_recreate_after_rank_failure" -x -q --timeout 200 --timeout-method thread \
  > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
PGPU_TRACE=1 timeout -k 10 300 python3 -u bench.py --segments-per-gpu 125 --steps 20 --warmup 3 --inflight 1 \
  --no-cpu-baseline --no-pmc --parity-segments 0 --host-profile > $O/trace125.log 2>&1 || exit 1
tail -1 $O/trace125.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/prof -o run -- \
  python3 -u bench.py --segments-per-gpu 125 --steps 10 --warmup 2 --inflight 1 --no-cpu-baseline --no-pmc --no-bytes \
  --parity-segments 0 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name run_kernel_trace.csv | head -1)
python3 tools/timeline.py $(dirname $f) > $O/timeline125.txt && tail -25 $O/timeline125.txt
for spec in "c2:--workload c2" "c4s:--workload c4 --no-star-tree"; do
  n=${spec%%:*}; a=${spec#*:}
  echo "== $n"
  LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_dense4.so" BENCH_ARGS="$a" timeout -k 10 600 bash scripts/ab_lib.sh || exit 1
done
