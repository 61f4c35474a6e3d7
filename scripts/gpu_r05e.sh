#!/bin/bash
# r05 session e: the whole GPU suite (pgpu_config in place of the environment knobs), smoke, then C2's traffic with
# and without the md dictionary gathers (diagnostic build: which share of C2's 1.85x traffic they are), then the C3
# scan time against the segment count (the per-launch intercept).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
for lib in libpinotgpu libpinotgpu_ab_nodval; do
  PGPU_LIB=pinot_amd/$lib.so timeout -k 10 500 python3 -u bench.py --workload c2 --segments-per-gpu 100 --steps 20 \
    --warmup 5 --no-cpu-baseline --parity-segments 0 > $O/c2_$lib.log 2>&1 || { tail -5 $O/c2_$lib.log; exit 1; }
  tail -1 $O/c2_$lib.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c2 $lib', d['ms_per_step'], r['kernel_us'], r['frac'], r['traffic'], r['bytes_alg_per_launch'], r.get('traffic_pmc'))"
done
for segs in 32 125 500; do
  timeout -k 10 300 python3 -u bench.py --steps 50 --warmup 5 --segments-per-gpu $segs --no-cpu-baseline --no-pmc \
    --parity-segments 0 --roofline-steps 20 > $O/c3_seg$segs.log 2>&1 || { tail -5 $O/c3_seg$segs.log; exit 1; }
  tail -1 $O/c3_seg$segs.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c3 segs $segs', d['ms_per_step'], d['latency_ms_per_query'], r['kernel_us'], r['frac'])"
done
bash scripts/gpu_mr_bench.sh || exit 1
# K8e one-word split (part_split_words_kernel) vs the general split
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_nosplitw.so" BENCH_ARGS="--workload c5 --segments-per-gpu 100" \
  bash scripts/ab_lib.sh || exit 1
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_ab_nosplitw.so" BENCH_ARGS="--workload c5_hash --segments-per-gpu 100" \
  bash scripts/ab_lib.sh || exit 1
