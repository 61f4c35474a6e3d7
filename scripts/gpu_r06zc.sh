#!/bin/bash
# r06 session zc: compact_dense_scatter_kernel's duration, new (rounds loaded up front) vs previous library, C5 at 13
# segments one query at a time (rocprofv3 kernel statistics), twice each, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06zc
mkdir -p $O
for rep in 1 2; do
  for lib in libpinotgpu libpinotgpu_prev; do
    PGPU_LIB=pinot_amd/$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_${lib}_$rep -o run -- \
      python3 -u bench.py --workload c5 --segments-per-gpu 13 --steps 20 --warmup 3 --inflight 1 --no-pmc --no-cpu-baseline \
      --parity-segments 0 > $O/${lib}_$rep.log 2>&1 || { tail -5 $O/${lib}_$rep.log; exit 1; }
    echo "$lib $rep $(grep -h 'compact_dense_scatter\|compact_minmax\|part_aggregate' $(find $O/p_${lib}_$rep -name run_kernel_stats.csv) | awk -F'","|",' '{print $1}' | cut -c2-40 | tr '\n' ' ') $(grep -h 'compact_dense_scatter\|part_aggregate' $(find $O/p_${lib}_$rep -name run_kernel_stats.csv) | python3 -c "import sys,csv; [print(round(float(r[3])/1e3,1), end=' ') for r in csv.reader(sys.stdin)]") $(tail -1 $O/${lib}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['latency_ms_per_query'])")"
  done
done
