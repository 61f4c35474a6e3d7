#!/bin/bash
# PMC counters of the scan kernel for a set of queries (one rocprofv3 pass per counter group per query).
# Q1..Qn via SQLS (|-separated), workload WLD (default c2), segments NSEG.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
WLD=${WLD:-c2}; NSEG=${NSEG:-100}
PASSES=("SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
        "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_FLAT")
IFS='|' read -ra QS <<< "${SQLS:-SELECT COUNT(*) FROM t WHERE f < 500 GROUP BY d|SELECT SUM(mi) FROM t WHERE f < 500 GROUP BY d}"
qi=0
for q in "${QS[@]}"; do
  qi=$((qi+1)); pi=0
  for pass in "${PASSES[@]}"; do
    pi=$((pi+1))
    timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/pmc/q${qi}_p${pi} -o run -- \
      python3 -u bench.py --workload $WLD --segments-per-gpu $NSEG --steps 2 --warmup 1 --no-bytes --no-cpu-baseline --no-pmc --sql "$q" \
      > gpurun_out/pmc/q${qi}_p${pi}.log 2>&1 || { echo "pass $qi/$pi failed"; tail -5 gpurun_out/pmc/q${qi}_p${pi}.log; exit 1; }
    echo "q$qi p$pi done"
  done
done
python3 - <<'PY'
import csv, glob, os, collections
for d in sorted(glob.glob("gpurun_out/pmc/q*_p*")):
    if not os.path.isdir(d): continue
    fs = [os.path.join(r, f) for r, _, ff in os.walk(d) for f in ff if f.endswith("counter_collection.csv")]
    if not fs: continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(fs[0])):
        if "filter_groupby_kernel" in r["Kernel_Name"] or "scan_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(d, {k: "%.4g" % (sum(v) / len(v)) for k, v in sorted(acc.items())})
PY
