#!/bin/bash
# r06 session q: contiguous tile runs for the dense and wide plans too (libpinotgpu_chunkall: their gathers now read
# table-global value arrays, so the interleaved order's L2 argument may be gone; chunked runs also take the slot
# weights on a solo launch) against the default, on C2, the C4 scan path and C1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
for spec in "c2:--workload c2" "c4s:--workload c4 --no-star-tree" "c1:--workload c1"; do
  n=${spec%%:*}; a=${spec#*:}
  echo "== $n"
  LIBS="pinot_amd/libpinotgpu.so pinot_amd/libpinotgpu_chunkall.so" BENCH_ARGS="$a" timeout -k 10 500 bash scripts/ab_lib.sh || exit 1
done
