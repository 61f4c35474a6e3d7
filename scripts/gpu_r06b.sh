#!/bin/bash
# r06 session b: the whole GPU suite on the tree with run-time tile claims and constant-address-space record reads,
# then an interleaved A/B of three libraries -- claims (default), the same without claims (PGPU_NO_CLAIM), and the
# round-5 library -- on C3 at 125 / 1000 segments, indexed C3, C2 and the C4 scan path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log
[ $rc -ne 0 ] && exit $rc
LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_noclaim.so pinot_amd/libpinotgpu_r05.so"
for spec in "c3_125:--segments-per-gpu 125" "c3_1000:" "c3inv:--workload adanalytics_inv" "c2:--workload c2" \
            "c4s:--workload c4 --no-star-tree"; do
  n=${spec%%:*}; a=${spec#*:}
  echo "== $n"
  LIBS="$LIBS" BENCH_ARGS="$a" timeout -k 10 600 bash scripts/ab_lib.sh || exit 1
done
