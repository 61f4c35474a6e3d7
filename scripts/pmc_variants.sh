#!/bin/bash
# PMC passes (scripts/pmc_kernel.sh) of one workload under several environment variants (library builds:
# PGPU_LIB=pinot_amd/libpinotgpu_ab_x.so): VARIANTS="A=0 B=1|A=1" (| between
# variants, spaces inside one), TAGP=prefix, plus pmc_kernel.sh's KREGEX / ARGS / SQL / PASSES.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
IFS='|' read -ra VS <<< "${VARIANTS:-PGPU_X=0}"
i=0
for v in "${VS[@]}"; do
  i=$((i+1))
  echo "=== variant $i: $v"
  ( for e in $v; do export "$e"; done; TAG=${TAGP:-v}$i bash scripts/pmc_kernel.sh ) || exit 1
done
