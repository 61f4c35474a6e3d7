#!/bin/bash
# r06 session z (and zb: the compact scatter with every round's words loaded up front): K8d writes the ordered compaction's chunk counts and ranges (C5: partitions == compaction chunks), so
# finalize skips compact_count_kernel: partitioned / workload GPU tests, then C5 at 100 and 13 segments against the
# previous library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06z
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_workloads_gpu.py tests/test_hash_partition_gpu.py \
  tests/test_multi_rank_gpu.py -x -q --timeout 250 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for spec in "c5:--workload c5" "c5_13:--workload c5 --segments-per-gpu 13"; do
  n=${spec%%:*}; a=${spec#*:}
  echo "== $n"
  LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_prev.so" BENCH_ARGS="$a" timeout -k 10 500 bash scripts/ab_lib.sh || exit 1
done
