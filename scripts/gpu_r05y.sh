#!/bin/bash
# r05 session y: the C3 epilogue's two parts (slab fold, leap-frog statistics) at 125 and 1000 segments: kernel
# summaries of the C3 query and of a one-leaf variant (no leap-frog statistics, fold only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05y
mkdir -p $O
ONE="SELECT sum(clicks), sum(impressions) FROM AdAnalyticsTable WHERE daysSinceEpoch BETWEEN 17849 AND 17856 GROUP BY daysSinceEpoch TOP 100"
for n in 125 1000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$n -o run -- python3 -u bench.py \
    --segments-per-gpu $n --steps 20 --warmup 3 --inflight 1 --no-pmc --no-cpu-baseline --no-bytes --parity-segments 0 > $O/p_$n.log 2>&1 || { tail -5 $O/p_$n.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/q_$n -o run -- python3 -u bench.py \
    --segments-per-gpu $n --steps 20 --warmup 3 --inflight 1 --no-pmc --no-cpu-baseline --no-bytes --parity-segments 0 --sql "$ONE" > $O/q_$n.log 2>&1 || { tail -5 $O/q_$n.log; exit 1; }
done
for f in $O/p_125 $O/q_125 $O/p_1000 $O/q_1000; do
  python - "$f" <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0])))
keep = [r for r in rows if any(k in r["Name"] for k in ("filter_groupby", "epilogue", "copyBuffer", "fillBuffer", "expand"))]
print(sys.argv[1], " | ".join("%s x%s %.1f" % (r["Name"][:28], r["Calls"], float(r["AverageNs"]) / 1000) for r in keep))
PY
done
