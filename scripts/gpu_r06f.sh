#!/bin/bash
# r06 session f: per-workgroup start / loop-end / end times with the CU (HW_ID) and XCD (XCC_ID) that ran each
# workgroup (diagnostics build PGPU_DIAG_WG_TIMES, raw rows via PGPU_WGTIMES_OUT) for C3 at 125 and 1000 segments;
# then the kernel + copy timeline of C3 at 125 segments as the bench runs it (3 queries in flight) with kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
run() {  # name, bench args
  local name=$1; shift
  PGPU_LIB=pinot_amd/libpinotgpu_diag_wgt.so PGPU_TRACE=wgtimes PGPU_WGTIMES_OUT=$O/$name.wg timeout -k 10 300 \
    python -u bench.py --steps 4 --warmup 2 --warmup-ms 0 --inflight 1 --roofline-steps 1 --no-cpu-baseline --no-pmc \
    --no-bytes --parity-segments 0 "$@" > $O/$name.log 2>&1 || { tail -5 $O/$name.log; return 1; }
  echo "== $name"; grep wgtimes $O/$name.log | tail -3 | cut -c1-300
}
run c3_125 --segments-per-gpu 125 && run c3_1000 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 -u bench.py --segments-per-gpu 125 --steps 20 --warmup 3 --roofline-steps 1 --no-cpu-baseline --no-pmc \
  --no-bytes --parity-segments 0 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name run_kernel_trace.csv)
python3 tools/timeline.py $(dirname $f) filter_groupby 2 8 > $O/timeline125_pipelined.txt && tail -45 $O/timeline125_pipelined.txt
