#!/bin/bash
# r05 session zc: K8a / K8c held to 4 waves per SIMD (launch bound: 128 VGPRs; the staged K8c had 130, 3 waves) vs as
# built, on C5 and c5_hash.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_pp4.so" BENCH_ARGS="--workload c5 --parity-segments 100" bash scripts/ab_lib.sh || exit 1
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_pp4.so" BENCH_ARGS="--workload c5_hash --parity-segments 100" bash scripts/ab_lib.sh || exit 1
for l in pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_pp4.so; do
  PGPU_LIB=$l timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/zc/$(basename $l .so) -o run -- python3 -u bench.py \
    --workload c5 --steps 10 --warmup 2 --inflight 1 --no-pmc --no-cpu-baseline --no-bytes --parity-segments 0 > gpurun_out/zc_$(basename $l .so).log 2>&1 || exit 1
  python - "gpurun_out/zc/$(basename $l .so)" <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0])))
keep = [r for r in rows if "part_" in r["Name"]]
print(sys.argv[1], " | ".join("%s %.1f" % (r["Name"][10:40], float(r["AverageNs"]) / 1000) for r in keep))
PY
done
