#!/bin/bash
# SQL="..." overrides the workload query.
# PMC passes over one kernel of a bench run: KREGEX="startree_scan" ARGS="--workload c4 --segments-per-gpu 64"
# PASSES="A B C;D E" (passes separated by ;).  Each pass is its own rocprofv3 run (counter slots per pass are limited); CSVs under gpurun_out/pmc/<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
touch pinot_amd/libpinotgpu*.so  # the prebuilt library is current
TAG=${TAG:-k}
OUT=gpurun_out/pmc/$TAG
mkdir -p $OUT
i=0
IFS=';' read -ra PLIST <<< "${PASSES:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT}"
for pass in "${PLIST[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/p$i -o p -- \
    python3 bench.py $ARGS ${SQL:+--sql "$SQL"} --steps 3 --warmup 1 --no-pmc --no-cpu-baseline > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
for f in $(find $OUT -name "*counter_collection.csv"); do
  python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    agg[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print("%-60s %-24s mean %.4g  n=%d" % (k, c, sum(v) / len(v), len(v)))
PY
done
