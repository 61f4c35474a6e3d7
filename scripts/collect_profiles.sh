#!/bin/bash
# Copies a gpu_profiles.sh session's outputs (gpurun_out/profiles/) into profiles/ under a round prefix:
#   <name>_bench.json -> profiles/<round>_<name>_1gpu_bench.json
#   prof_<name>/run_kernel_stats.csv -> profiles/<round>_<name>_1gpu_kernel_stats.csv
# usage: bash scripts/collect_profiles.sh r04
cd "$(dirname "$0")/.."
round=${1:?round prefix, e.g. r04}
for j in gpurun_out/profiles/*_bench.json; do
  [ -s "$j" ] || continue
  name=$(basename "$j" _bench.json)
  cp "$j" "profiles/${round}_${name}_1gpu_bench.json"
  k="gpurun_out/profiles/prof_${name}/run_kernel_stats.csv"
  [ -s "$k" ] && cp "$k" "profiles/${round}_${name}_1gpu_kernel_stats.csv"
  echo "$name"
done
