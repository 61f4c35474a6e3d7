#!/bin/bash
# r04 session c: A/B of this round's kernel forms (env knobs, interleaved) -- C2 dense LDS forms and SADDR gathers,
# C5 record packing, hashed partitions against the global hash table on c5_hash -- and the indexed C3 line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
VARIANTS="PGPU_X=0 PGPU_NO_DENSE_NARROW=1 PGPU_NO_PACK_COUNT=1" BENCH_ARGS="--workload c2 --no-bytes" bash scripts/ab_env.sh || exit 1
VARIANTS="PGPU_X=0 PGPU_NO_CS_PACK=1 PGPU_NO_FINE_PACK=1" BENCH_ARGS="--workload c5 --no-bytes" bash scripts/ab_env.sh || exit 1
VARIANTS="PGPU_X=0 PGPU_NO_PACK_COUNT=1" BENCH_ARGS="--workload c4 --no-star-tree --no-bytes" bash scripts/ab_env.sh || exit 1
WL="adanalytics_inv:1000 c5_hash:100" NOPROF=1 bash scripts/gpu_profiles.sh
