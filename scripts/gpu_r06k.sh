#!/bin/bash
# r06 session k: star-tree metric arrays pinned as int32 when integral (half the bytes per star document) and the
# kernel's count of metric sectors holding a matched doc (the line-granular bytes model): the star-tree GPU tests,
# then C4 star path / scan path lines (64 segments, PMC traffic) and the 8-segment per-rank share.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_startree_gpu.py tests/test_workloads_gpu.py -x -q --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for spec in "c4:--workload c4" "c4_scan:--workload c4 --no-star-tree" "c4_8seg:--workload c4 --segments-per-gpu 8" \
            "c4_scan_8seg:--workload c4 --no-star-tree --segments-per-gpu 8"; do
  n=${spec%%:*}; a=${spec#*:}
  timeout -k 10 400 python -u bench.py $a --steps 20 --warmup 5 > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  echo "== $n"; tail -1 $O/$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['ms_per_step'], d['latency_ms_per_query'], {k: r.get(k) for k in ('kernel_us','frac','traffic','bytes_alg_per_launch','star_metric_bytes','bytes_per_star_doc','star_docs_read')}, (d.get('parity') or {}).get('ok'))"
done
