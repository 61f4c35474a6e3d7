#!/bin/bash
# r06 session h: the GPU suite with slot weights as a pgpu_config field (slot_weight_step) applied to solo launches
# only (table->scans_inflight), then an interleaved A/B of the step (0 = equal shares) on C3 at 1000 / 125 segments
# and indexed C3: the pipelined step must not lose, the serialized scan should gain.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
touch pinot_amd/libpinotgpu*.so
export TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log
[ $rc -ne 0 ] && exit $rc
V="--config slot_weight_step=0.0;--config slot_weight_step=0.11;--config slot_weight_step=0.15"
for spec in "c3_1000:" "c3inv:--workload adanalytics_inv" "c3_125:--segments-per-gpu 125"; do
  n=${spec%%:*}; a=${spec#*:}
  echo "== $n"
  VARIANTS="$V" BENCH_ARGS="$a" timeout -k 10 700 bash scripts/ab_args.sh || exit 1
done
