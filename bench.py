"""Benchmark: the README AdAnalytics filtered GROUP BY (BASELINE.json configs[2], C3) on synthetic segments
pinned in HBM, one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload adanalytics|c1|c2|c4|c5]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

--gpus N > 1 without a launcher starts the N rank processes itself (before this process touches the GPU) and exits
with the first failing rank's code; under a launcher WORLD_SIZE must equal --gpus.  RCCL takes one GPU per rank, so
more ranks than visible GPUs fail at once (PGPU_BENCH_BACKEND=host rehearses N ranks on fewer GPUs).

A step is one whole query on every rank: plan (per-segment predicate translation; a plan-cache hit for a repeated
query), the fused scan kernel over all local segments, the dense group-table merge across ranks (RCCL all-reduce
over xGMI) and the compacted result copied back to the host.  By default the workload's BASELINE row count is split
across the ranks (strong scaling: C3 = 1 000 segments of 1M docs = 1B rows over 1/2/4/8 GPUs, "1B rows sharded
1/2/4/8 GPUs"); --segments-per-gpu S instead pins S segments on every rank (weak scaling).  Queries are pipelined
--inflight deep (default 3, each in flight on its own stream and group table): query k+1 is planned and launched
before query k's result is finalized, as a server overlaps concurrent queries -- the GPU does not idle while the
host finalizes.  Kernel durations for the roofline come from a separate serialized pass (--inflight 1 semantics).
Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SHARD_BYTES = 16 << 20  # group tables at least this large are reduce-scattered across ranks, not all-reduced
# Rows of each workload's BASELINE.json configuration: the default strong-scaling total.
DEFAULT_ROWS = {"adanalytics": 1_000_000_000, "adanalytics_inv": 1_000_000_000, "c1": 1_000_000, "c2": 100_000_000,
                "c4": 64_000_000, "c5": 100_000_000, "c5_hash": 100_000_000}
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md "Chip-level parameters"


def log(msg):
    """Progress to stderr (long phases: segment generation, bytes_alg pass, CPU baseline)."""
    print("[bench %s] %s" % (time.strftime("%H:%M:%S"), msg), file=sys.stderr, flush=True)


def parse_args():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)  # sub-millisecond steps: a long enough timed region
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--warmup-ms", type=float, default=60.0,
                   help="after the W warm-up steps, keep warming up (untimed) until this much wall time of sustained "
                        "queries has passed: the per-step trace of the driver's command shows query time decaying "
                        "750 -> 670 us over the first ~20 ms of load (the GPU's clocks ramping), which a 5-step warm-up "
                        "leaves inside the timed region; 0 = exactly W steps")
    p.add_argument("--workload", default="adanalytics")
    p.add_argument("--sql", default=None, help="override the workload's query (same table)")
    p.add_argument("--rows-total", type=int, default=None,
                   help="strong scaling: this many rows split across the ranks (default: the workload's BASELINE rows)")
    p.add_argument("--segments-per-gpu", type=int, default=None,
                   help="weak scaling: this many segments on every rank (overrides --rows-total)")
    p.add_argument("--inflight", type=int, default=3,
                   help="queries in flight (1 = strictly one after another); 3: C3 at 125 segments per rank (one rank's "
                        "share at N=8) 0.116 -> 0.104 ms per query against 2, 1000 segments 0.676 -> 0.672")
    p.add_argument("--roofline-steps", type=int, default=10, help="serialized steps timing the scan kernel")
    p.add_argument("--docs-per-segment", type=int, default=1_000_000)
    p.add_argument("--cpu-sample-segments", type=int, default=None, help="default: the workload's sample size")
    p.add_argument("--cpu-target-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--parity-segments", type=int, default=None,
                   help="segments of the full-size parity check against the oracle (default: all; 0 = skip)")
    p.add_argument("--no-bytes", action="store_true", help="skip the bytes_alg measurement pass")
    p.add_argument("--verify", action="store_true", help="check every step's result equals the first")
    p.add_argument("--host-profile", action="store_true", help="report host time per phase of a step")
    p.add_argument("--step-trace", default=None, help="write per-query host timestamps of the timed region (JSON)")
    p.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 FETCH_SIZE passes (roofline.traffic)")
    p.add_argument("--no-star-tree", action="store_true", help="query option useStarTree=false (scan path)")
    p.add_argument("--num-groups-limit", type=int, default=None, help="query option numGroupsLimit (default: the "
                   "workload's)")
    p.add_argument("--config", default=None, help="table executor settings, field=value[,field=value] "
                   "(pgpu_config fields, e.g. dense_selectivity=0.5)")
    return p.parse_args()


def parse_config(text):
    """--config: "field=value,field=value" -> {field: int or float} (pgpu_config, include/pinotgpu.h)."""
    out = {}
    for item in filter(None, (text or "").split(",")):
        k, _, v = item.partition("=")
        out[k.strip()] = float(v) if "." in v else int(v)
    return out


def compulsory_bytes(table, handles, query, docs_per_segment, inverted_columns=()):
    """bytes_alg (compulsory-traffic form): full forward-index bytes of every filter column, plus
    the 128-B lines of every other referenced column's forward index that hold >= 1 matched doc, plus the 128-B
    lines of the group-by / aggregated columns' dictionaries that hold >= 1 matched dictId.  A filter column whose
    predicates are all inverted-index leaves (EQ / NOT_EQ / IN / NOT_IN on a column with a bitmap inverted index)
    costs the scan kernel its materialised docId bitmap, N/8 bytes, instead of its forward index."""
    from pinot_amd.query import EQ, IN, NOT_EQ, NOT_IN
    preds = []
    if query.filter is not None:
        query.filter.postfix(preds, [])
    filter_cols = sorted({p.column for p in preds})
    bitmap_cols = {c for c in filter_cols if c in inverted_columns and
                   all(p.type in (EQ, NOT_EQ, IN, NOT_IN) for p in preds if p.column == c)}
    other_cols = [c for c in query.columns() if c not in filter_cols]
    dict_cols = [c for c in query.group_by] + [c for _, c in query.aggregations if c != "*"]
    dict_cols = sorted(set(dict_cols))
    width = {n: (4 if t in ("INT", "FLOAT") else 8) for n, t in zip(table.names, [None] * len(table.names))}
    for i, n in enumerate(table.names):
        width[n] = 4 if table.types[i] in (0, 2) else 8
    total = 0
    matched_total = 0
    with table.plan(handles, query) as plan:
        scanned = plan.scanned_segments()
    for h, sc in zip(handles, scanned):
        if not sc:  # filter folded to always-false: the segment is not read (EmptyFilterOperator)
            continue
        bm = table.filter_bitmap(h, query, docs_per_segment)
        bits = np.unpackbits(bm.view(np.uint8), bitorder="little")[:docs_per_segment]
        docs = np.nonzero(bits)[0].astype(np.int64)
        matched_total += len(docs)
        info = {}
        for c in set(filter_cols) | set(other_cols):
            card, b, dlen, flen = _col_info(table, h, c)
            info[c] = (card, b, flen)
        for c in filter_cols:
            total += ((docs_per_segment + 31) // 32) * 4 if c in bitmap_cols else info[c][2]
        for c in other_cols:
            b = info[c][1]
            if len(docs):
                first = (docs * b) >> 10          # 1024 bits = one 128-B line
                last = (docs * b + b - 1) >> 10
                total += len(np.union1d(first, last)) * 128
        for c in dict_cols:
            if len(docs):
                ids = table.read_dict_ids(h, c, docs.astype(np.int32)).astype(np.int64)
                total += len(np.unique((ids * width[c]) >> 7)) * 128
    return total, matched_total


def _col_info(table, h, c):
    import ctypes
    from pinot_amd import _lib as L
    card, bits = ctypes.c_int32(), ctypes.c_int32()
    dl, fl = ctypes.c_int64(), ctypes.c_int64()
    L.check(table.lib.pgpu_segment_column_info(table.handle, h, table.index[c], ctypes.byref(card),
                                               ctypes.byref(bits), ctypes.byref(dl), ctypes.byref(fl)))
    return card.value, bits.value, dl.value, fl.value


# Calibration query per workload: every segment is scanned, no document matches, and the only bytes read are the
# full forward index of one column (two contradicting EQ leaves on it), so its bytes_alg is exact.
CALIB_SQL = {
    "adanalytics": "SELECT COUNT(*) FROM t WHERE daysSinceEpoch = 17532 AND daysSinceEpoch = 17533 GROUP BY daysSinceEpoch",
    "adanalytics_inv": "SELECT COUNT(*) FROM t WHERE daysSinceEpoch = 17532 AND daysSinceEpoch = 17533 GROUP BY daysSinceEpoch",
    "c1": "SELECT COUNT(*) FROM t WHERE filt = 1 AND filt = 2 GROUP BY dim",
    "c2": "SELECT COUNT(*) FROM t WHERE f = 1 AND f = 2 GROUP BY d",
    "c5": "SELECT COUNT(*) FROM t WHERE k1 = 1 AND k1 = 2 GROUP BY k2",
    "c5_hash": "SELECT COUNT(*) FROM t WHERE k1 = 1 AND k1 = 2 GROUP BY k2",
    # C4: the calibration runs on the scan path (--no-star-tree in its child); the factor is the counter's (the gfx950
    # half count of wide streaming reads), so it applies to the star-tree kernels' FETCH_SIZE alike
    "c4": "SELECT COUNT(*) FROM t WHERE d1 = 1 AND d1 = 2 GROUP BY d2",
}
SCAN_KERNELS = ("filter_groupby_kernel", "part_pass_kernel", "part_split_kernel", "part_aggregate_kernel",
                "part_hash_aggregate_kernel", "startree_traverse_kernel", "startree_scan_kernel")
# the kernel that opens one scan launch (the partitioned group-by is a pipeline of four kernels per launch; a
# star-tree launch is the traversal, then the pre-aggregated document scan)
LAUNCH_KERNELS = ("filter_groupby_kernel", "part_pass_kernel<false", "startree_traverse_kernel")
# the launcher's and torch.distributed.run's variables: a profiled child run is one rank of its own
DIST_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE",
            "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID", "TORCHELASTIC_RESTART_COUNT",
            "TORCHELASTIC_MAX_RESTARTS", "PGPU_BENCH_PMC")


def _fetch_per_launch(csv_path):
    """FETCH_SIZE of one scan launch: every kernel of the launch's pipeline summed, averaged over the launches."""
    import csv
    rows = [r for r in csv.DictReader(open(csv_path)) if r["Counter_Name"] == "FETCH_SIZE"]
    total = sum(float(r["Counter_Value"]) for r in rows if any(k in r["Kernel_Name"] for k in SCAN_KERNELS))
    launches = sum(1 for r in rows if any(k in r["Kernel_Name"] for k in LAUNCH_KERNELS))
    return total / launches * 1024.0 if launches else None


def pmc_traffic(args):
    """roofline.traffic: HBM bytes per launch of the scan kernel from rocprofv3 FETCH_SIZE (KB units), measured in
    two child runs of this script started before this process touches the GPU: the bench query, and a calibration
    query of known bytes (CALIB_SQL) in the same access pattern.  FETCH_SIZE under-counts wide streaming reads on
    gfx950 (MI355X_MICROARCH.md, HBM section); traffic = FETCH(main) x bytes_alg(calib) / FETCH(calib)."""
    import shutil
    import subprocess
    import tempfile
    rocprof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(rocprof) or args.workload not in CALIB_SQL:
        return None
    base = [sys.executable, "-u", os.path.abspath(__file__), "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
            "--no-pmc", "--workload", args.workload, "--segments-per-gpu", str(args.local_segments),
            "--docs-per-segment", str(args.docs_per_segment), "--inflight", "1", "--roofline-steps", "2",
            "--warmup-ms", "0", "--parity-segments", "0"]
    if args.num_groups_limit:
        base += ["--num-groups-limit", str(args.num_groups_limit)]
    if args.config:
        base += ["--config", args.config]
    env = {k: v for k, v in os.environ.items() if k not in DIST_ENV}
    res = {}
    with tempfile.TemporaryDirectory() as d:
        for name, sql in (("main", args.sql), ("calib", CALIB_SQL[args.workload])):
            extra = (["--sql", sql] if sql else []) + \
                (["--no-star-tree"] if args.no_star_tree or name == "calib" else [])
            cmd = [rocprof, "--pmc", "FETCH_SIZE", "--output-format", "csv", "-d", d, "-o", name, "--"] + base + extra
            try:
                p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300,
                                   env=env)
            except subprocess.TimeoutExpired:
                print("pmc pass %s timed out" % name, file=sys.stderr)
                return None
            line = [x for x in p.stdout.splitlines() if x.startswith("{")]
            csvs = [os.path.join(r, f) for r, _, fs in os.walk(d) for f in fs if f == name + "_counter_collection.csv"]
            if p.returncode != 0 or not line or not csvs:
                print("pmc pass %s failed (rc %d): %s" % (name, p.returncode, p.stdout[-2000:]), file=sys.stderr)
                return None
            res[name] = (json.loads(line[-1]), _fetch_per_launch(csvs[0]))
    (jm, fm), (jc, fc) = res["main"], res["calib"]
    if not fm or not fc:
        return None
    factor = jc["roofline"]["bytes_alg_per_launch"] / fc
    return {"traffic": fm * factor, "fetch_size_bytes": fm, "calib_factor": round(factor, 4),
            "calib_bytes_alg": jc["roofline"]["bytes_alg_per_launch"], "calib_fetch_size_bytes": fc}


def attach_star_trees(table, handles, workload, docs):
    """Builds each segment's star-tree on the host (pgpu_startree_build: BaseSingleTreeBuilder restatement) from
    the segment's Pinot bytes and pins it beside the segment (worker threads; the builder releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    from pinot_amd import _lib as L
    from pinot_amd.segment import ColumnData, SegmentBuffers
    from pinot_amd.startree import StarTree
    spec = workload.star_tree

    def build(seg):
        return StarTree.build(workload.schema, seg, spec["split_order"], spec["pairs"], spec["max_leaf_records"])

    handles = list(handles)
    with ThreadPoolExecutor(max_workers=8) as ex:
        for i in range(0, len(handles), 8):
            segs = []
            for h in handles[i:i + 8]:  # segment bytes back from HBM (the table's stream: one thread)
                cols = {}
                for name, typ in workload.schema:
                    card, bits, d, f = table.segment_column_bytes(h, name)
                    tcode = L.TYPE_NAMES[typ]
                    cols[name] = ColumnData(tcode, card, bits, 4 if tcode in (L.INT, L.FLOAT) else 8, d, f)
                segs.append(SegmentBuffers(docs, cols))
            for h, st in zip(handles[i:i + 8], ex.map(build, segs)):
                table.attach_startree(h, st)
                st.close()


def attach_inverted_indexes(table, handles, workload, docs):
    """Bitmap inverted indexes of the workload's columns: each segment's forward index is read back, the host
    creator (pgpu_build_inverted_index) writes Pinot's .bitmap.inv bytes, and pgpu_attach_inverted_index pins them."""
    from concurrent.futures import ThreadPoolExecutor
    from pinot_amd.segment_files import build_inverted_index_native

    def one(h):
        out = []
        for name in workload.inverted_columns:
            card, bits, _, fwd = table.segment_column_bytes(h, name)
            out.append((name, build_inverted_index_native(fwd, bits, docs, card)))
        return h, out

    with ThreadPoolExecutor(8) as ex:
        for h, out in ex.map(one, handles):
            for name, inv in out:
                table.attach_inverted_index(h, name, inv)


def host_segments(table, handles, workload, docs):
    """Each segment's Pinot bytes pulled back from HBM (what the oracle reads)."""
    from pinot_amd import _lib as L
    from pinot_amd.segment import ColumnData, SegmentBuffers
    segs = []
    for h in handles:
        cols = {}
        for name, typ in workload.schema:
            card, bits, d, f = table.segment_column_bytes(int(h), name)
            tcode = L.TYPE_NAMES[typ]
            cols[name] = ColumnData(tcode, card, bits, 4 if tcode in (L.INT, L.FLOAT) else 8, d, f)
        segs.append(SegmentBuffers(docs, cols))
    return segs


def attach_star_arrays(segs, workload):
    """Each host segment's star-tree (the same builder that made the pinned trees, so the same trees) as the oracle's
    input: seg.star_arrays, read by run_groupby(..., use_star_tree=True)."""
    from concurrent.futures import ThreadPoolExecutor
    from pinot_amd.startree import StarTree
    spec = workload.star_tree

    def tree(seg):
        st = StarTree.build(workload.schema, seg, spec["split_order"], spec["pairs"], spec["max_leaf_records"])
        a = st.arrays()
        st.close()
        return a
    with ThreadPoolExecutor(8) as ex:
        for seg, a in zip(segs, ex.map(tree, segs)):
            seg.star_arrays = a


def full_parity(table, handles, query, workload, docs, args):
    """The GPU answer of the benchmarked query over the first --parity-segments segments (default: all of this
    rank's) against the oracle's over the same bytes (pulled back from HBM): bit-exact for integer / count / dictId
    work, 1e-9 relative for FLOAT / DOUBLE sums (BASELINE north_star).  Star-tree plans are checked against the
    oracle's star-tree operator over the same trees, statistics included; inverted-index plans compare
    numDocsScanned only (the oracle restates the scan operator, whose numEntriesScannedInFilter differs by design)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle
    n = len(handles) if args.parity_segments is None else max(0, min(args.parity_segments, len(handles)))
    if n == 0:
        return None
    t0 = time.perf_counter()
    hs = np.ascontiguousarray(handles[:n], dtype=np.int64)
    segs = host_segments(table, hs, workload, docs)
    star = bool(workload.star_tree) and query.use_star_tree
    if star:  # the oracle's star-tree operator over the same trees (statistics = star-tree documents read)
        attach_star_arrays(segs, workload)
    orc = _oracle.run_groupby_arrays(workload.schema, segs, query, nthreads=host_cores(), use_star_tree=star)
    del segs
    r = table.execute_groupby(hs, query)
    cmp = _oracle.compare_result_arrays(table, r, orc, query, workload.schema,
                                        check_stats="docs" if workload.inverted_columns else True)
    cmp.update({"segments": n, "rows": n * docs, "seconds": round(time.perf_counter() - t0, 1),
                "against": "oracle/oracle.c over the same segment bytes"})
    return cmp


def multi_rank_parity(table, handles, query, workload, docs, res, world, rank, sharded):
    """Parity of an N-rank query (the check full_parity makes at N = 1): every rank runs the oracle over its own
    segments' bytes (pulled back from its HBM, the rank's cores split between the ranks of the box), rank 0 merges
    those per-server partial results as the broker merges server responses (_oracle.merge_partial_arrays, numpy --
    not the device combine it checks) and compares them with the GPU's merged answer: rank 0's table for an all-reduce,
    every rank's disjoint share gathered for reduce-scatter / hash / row combines.  Statistics are per rank on both
    sides (the combine merges groups, not statistics) and compared as sums.  Collective: every rank calls it; rank 0
    gets the verdict dict, the others None."""
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle
    t0 = time.perf_counter()
    hs = np.ascontiguousarray(handles, dtype=np.int64)
    segs = host_segments(table, hs, workload, docs)
    threads = max(1, host_cores() // world)
    star = bool(workload.star_tree) and query.use_star_tree
    err = None
    try:
        if star:
            attach_star_arrays(segs, workload)
        orc = _oracle.run_groupby_arrays(workload.schema, segs, query, nthreads=threads, use_star_tree=star)
    except Exception as e:  # every rank reaches the gather below, whatever failed here
        orc, err = None, "rank %d oracle: %s" % (rank, e)
    del segs
    gpu = _oracle.gpu_result_arrays(table, res, query) if (sharded or rank == 0) else None
    mine = {"rank": rank, "orc": orc, "gpu": gpu, "stats": tuple(res.stats.as_tuple()), "err": err,
            "segments": len(hs)}
    gathered = [None] * world if rank == 0 else None
    dist.gather_object(mine, gathered, dst=0)
    if rank != 0:
        return None
    errs = [g["err"] for g in gathered if g["err"]]
    if errs:
        return {"ok": False, "mismatch": "; ".join(errs), "ranks": world}
    merged = _oracle.merge_partial_arrays([g["orc"] for g in gathered], query.aggregations)
    gpu = _oracle.concat_arrays([g["gpu"] for g in gathered]) if sharded else gathered[0]["gpu"]
    gstats = tuple(int(sum(g["stats"][i] for g in gathered)) for i in range(4))
    out = _oracle.compare_arrays(gpu, gstats, merged, query, workload.schema,
                                 check_stats="docs" if workload.inverted_columns else True)
    nseg = sum(g["segments"] for g in gathered)
    out.update({"segments": nseg, "rows": nseg * docs, "ranks": world, "seconds": round(time.perf_counter() - t0, 1),
                "against": "oracle/oracle.c per rank over the same segment bytes, partial results merged as the "
                           "broker merges server responses (numpy)",
                "merged_from": "rank 0 (all-reduced table)" if not sharded else "every rank's disjoint share"})
    return out


def cpu_baseline(table, handles, query, workload, docs, args):
    """The oracle (C restatement of Pinot's per-segment operator + combine, one task per segment) timed on the
    host cores over a bounded sample of the same segments (bytes pulled back from HBM)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle
    nsample = args.cpu_sample_segments or max(workload.cpu_sample_segments, 2 * host_cores())
    sample = handles[:max(1, min(nsample, len(handles)))]
    segs = host_segments(table, sample, workload, docs)
    threads = host_cores()
    star = bool(workload.star_tree) and query.use_star_tree
    if star:  # the path Pinot's plan picks (StarTreeUtils.isFitForStarTree): the oracle's star-tree operator
        attach_star_arrays(segs, workload)
    _oracle.run_groupby(workload.schema, segs[:2], query, nthreads=threads, decode=False,
                        use_star_tree=star)  # warm-up
    reps, elapsed = 0, 0.0
    t0 = time.perf_counter()
    while True:
        _oracle.run_groupby(workload.schema, segs, query, nthreads=threads, decode=False, use_star_tree=star)
        reps += 1
        elapsed = time.perf_counter() - t0
        if elapsed >= args.cpu_target_seconds or reps >= 1000:
            break
    rows = reps * len(segs) * docs
    return {"value": rows / elapsed, "unit": "rows/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "nproc": os.cpu_count(),
            "sample": "%d segments x %d rows, %d repetitions, %.1f s, %d worker threads = every core this process may "
                      "run on (sched_getaffinity; the machine has %s) (oracle/oracle.c, one task per segment as "
                      "GroupByCombineOperator%s)" % (len(segs), docs, reps, elapsed, threads, os.cpu_count(),
                                                     "; star-tree path: StarTreeFilterOperator + "
                                                     "StarTreeGroupByExecutor over each segment's star-tree"
                                                     if star else "")}


def host_cores():
    """Cores this process may run on (the GPU box grants a share of the machine: os.cpu_count() shows all)."""
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        return max(1, os.cpu_count() or 1)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def launch_mode(gpus, environ, visible_gpus):
    """How this invocation runs, decided before anything touches the GPU:
    ("rank", N) -- one rank of N started by a launcher (torch.distributed.run or this script's own spawn): WORLD_SIZE
                   is set and must equal --gpus;
    ("single", 1) -- --gpus 1 without a launcher;
    ("spawn", N) -- --gpus N > 1 without a launcher: this process starts the N ranks itself (spawn_ranks).
    Raises SystemExit with the reason when the request cannot run: WORLD_SIZE != --gpus, or RCCL ranks (one GPU
    each) past the visible GPUs -- PGPU_BENCH_BACKEND=host rehearses N ranks sharing the visible GPUs."""
    if gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1 (got %d)" % gpus)
    ws = environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            raise SystemExit("bench.py: WORLD_SIZE=%s from the launcher but --gpus %d: the rank count and --gpus must "
                             "match" % (ws, gpus))
        return "rank", gpus
    if gpus == 1:
        return "single", 1
    if environ.get("PGPU_BENCH_BACKEND", "rccl") != "host" and visible_gpus < gpus:
        raise SystemExit("bench.py --gpus %d: %d GPU(s) visible, and RCCL takes one GPU per rank "
                         "(PGPU_BENCH_BACKEND=host rehearses %d ranks sharing the visible GPUs)"
                         % (gpus, visible_gpus, gpus))
    return "spawn", gpus


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def rank_env(environ, rank, world, port):
    """A spawned rank's environment: what torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 sets."""
    env = {k: v for k, v in environ.items() if k not in DIST_ENV}
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def spawn_ranks(world, argv, extra_env=None, poll_s=0.2, grace_s=20.0, script=None):
    """Starts `world` ranks of this script (child processes, never an exec) and waits for all of them.  The first rank
    that fails ends the others (terminate, then kill after `grace_s`: a rank left waiting in a collective for a dead
    peer never returns by itself).  Returns the exit code: 0, or the failed rank's (128 + signal for a signal)."""
    import signal
    import subprocess
    port = free_port()
    procs = []
    for r in range(world):
        env = rank_env(os.environ, r, world, port)
        if r == 0 and extra_env:
            env.update(extra_env)
        procs.append(subprocess.Popen([sys.executable, "-u", script or os.path.abspath(__file__)] + list(argv), env=env))
    rc, failed = 0, None
    live = set(range(world))
    t_fail = None
    while live:
        for r in sorted(live):
            x = procs[r].poll()
            if x is None:
                continue
            live.discard(r)
            if x != 0 and failed is None:
                failed, rc = r, (x if x > 0 else 128 - x)
                t_fail = time.monotonic()
                log("rank %d exited with %d: ending the other ranks" % (r, x))
                for q in live:
                    procs[q].send_signal(signal.SIGTERM)
        if live and t_fail is not None and time.monotonic() - t_fail > grace_s:
            for q in live:
                procs[q].kill()
            t_fail = float("inf")  # killed once
        time.sleep(poll_s)
    return rc


def main():
    args = parse_args()
    import torch

    how, _ = launch_mode(args.gpus, os.environ, torch.cuda.device_count())  # device_count() does not initialise HIP
    world = args.gpus if how != "single" else 1
    rank = int(os.environ.get("RANK", "0")) if how == "rank" else 0
    docs = args.docs_per_segment
    if args.segments_per_gpu:  # weak scaling
        seg_first, nseg = rank * args.segments_per_gpu, args.segments_per_gpu
        total_segments = args.segments_per_gpu * world
    else:  # strong scaling: the workload's rows split across the ranks
        rows = args.rows_total or DEFAULT_ROWS.get(args.workload, 1_000_000_000)
        total_segments = max(1, rows // docs)
        seg_first = rank * total_segments // world
        nseg = (rank + 1) * total_segments // world - seg_first
    args.local_segments = nseg
    pmc = None
    pmc_file = os.environ.get("PGPU_BENCH_PMC")
    if pmc_file is not None:  # rank 0 spawned by this script: the launcher measured it before starting the ranks
        if pmc_file:
            try:
                pmc = json.load(open(pmc_file))
            except (OSError, ValueError):
                pmc = None
    elif rank == 0 and not args.no_pmc and not args.no_bytes:
        # before this process initialises the GPU: the profiled runs are children, not exec'd (rank 0's share of the
        # segments, profiled as a one-rank run)
        from pinot_amd.build import build as _build
        _build()
        pmc = pmc_traffic(args)
    if how == "spawn":
        import tempfile
        extra = {}
        if pmc:
            fd, path = tempfile.mkstemp(prefix="pgpu_bench_pmc_", suffix=".json")
            with os.fdopen(fd, "w") as f:
                json.dump(pmc, f)
            extra["PGPU_BENCH_PMC"] = path
        else:
            extra["PGPU_BENCH_PMC"] = ""
        from pinot_amd.build import build as _build
        _build()  # once, before the ranks (each rank's build() then finds the library current)
        log("starting %d ranks (%s)" % (world, os.environ.get("PGPU_BENCH_BACKEND", "rccl")))
        rc = spawn_ranks(world, sys.argv[1:], extra)
        if extra.get("PGPU_BENCH_PMC"):
            os.unlink(extra["PGPU_BENCH_PMC"])
        sys.exit(rc)
    import torch.distributed as dist
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # The combine across ranks is the C ABI's (pgpu_comm + pgpu_plan_combine): RCCL over xGMI, one GPU per rank.
    # PGPU_BENCH_BACKEND=host rehearses the same combine code on a box with fewer GPUs than ranks (ranks share
    # devices, collectives staged through host memory).  torch.distributed (gloo, CPU) only hands the communicator
    # id to the ranks and brackets the timed region (barrier, max over ranks).
    backend = os.environ.get("PGPU_BENCH_BACKEND", "rccl")
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        local_rank = local_rank % max(1, torch.cuda.device_count()) if backend == "host" else local_rank
        torch.cuda.set_device(local_rank)
        dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)
    device = local_rank if world > 1 else 0

    from pinot_amd import _lib as L
    from pinot_amd.build import build
    from pinot_amd.combine import (Communicator, combine_mode, combine_plan, combine_result_rows,
                                   union_dictionaries_comm)
    from pinot_amd.executor import GpuTable
    from pinot_amd.query import parse_query
    from pinot_amd.workloads import WORKLOADS

    if rank == 0:
        build()
    if world > 1:
        dist.barrier()
    L.load()
    w = WORKLOADS[args.workload]()
    if args.sql:
        w.sql = args.sql
    q = parse_query(w.sql, num_groups_limit=args.num_groups_limit or w.num_groups_limit)
    if args.no_star_tree:
        q.use_star_tree = False
    table = GpuTable(w.schema, device=device, config=parse_config(args.config) or None)
    t_gen = time.perf_counter()
    handles = []
    for i in range(nseg):
        global_seg = seg_first + i
        handles.append(table.generate_segment(w.gen, row0=global_seg * docs, num_docs=docs))
    t_gen = time.perf_counter() - t_gen
    log("rank %d: %d segments generated in %.1f s" % (rank, nseg, t_gen))
    if w.star_tree:
        t_st = time.perf_counter()
        attach_star_trees(table, handles, w, docs)
        log("rank %d: star-trees built and pinned in %.1f s" % (rank, time.perf_counter() - t_st))
    if w.inverted_columns:
        t_inv = time.perf_counter()
        attach_inverted_indexes(table, handles, w, docs)
        log("rank %d: inverted indexes built and pinned in %.1f s" % (rank, time.perf_counter() - t_inv))
    comm = None
    if world > 1:
        kind = L.COMM_HOST if backend == "host" else L.COMM_RCCL
        try:
            comm = Communicator.from_process_group(kind, device)
        except L.PinotGpuError as e:  # every rank fails alike (RCCL missing / bootstrap refused): same transport
            log("rank %d: RCCL communicator failed (%s); combining over the host transport" % (rank, e))
            backend = "host (RCCL failed)"
            comm = Communicator.from_process_group(L.COMM_HOST, device)
        union_dictionaries_comm(table, q.group_by, comm)
    handles = np.array(handles, dtype=np.int64)

    # Real streams (the default stream's handle 0 would mean "the table's own stream" to the C ABI, and the
    # collectives on torch's stream would not be ordered after the scan writing d_table): one per query in flight,
    # each with its own group table.
    inflight = max(1, args.inflight)
    streams = [torch.cuda.Stream() for _ in range(inflight)]
    torch.cuda.set_stream(streams[0])
    # how the ranks' results merge, agreed by every rank (pgpu_plan_combine_mode): dense tables element-wise
    # (all-reduce, or reduce-scatter by key range when large), hash-mode tables by a device all-to-all,
    # numGroupsLimit / ARRAY_MAP plans by their finalized rows
    probe = table.plan(handles, q)
    mode, kinds = combine_mode(probe, comm, SHARD_BYTES) if world > 1 else (L.COMBINE_LOCAL, None)
    try:
        nslots, nkeys, _ = probe.layout()
    except L.PinotGpuError:  # numGroupsLimit plan: its parts have their own tables
        nslots, nkeys = 1, 0
    probe_nslots = nslots
    probe.close()
    # PGPU_BENCH_CALLER_TABLE=1: plans write into caller-owned device tables instead of their scratch tables
    caller_table = nkeys > 0 and os.environ.get("PGPU_BENCH_CALLER_TABLE") == "1"
    d_tables = [torch.empty((nslots, max(nkeys, 1)) if caller_table else (1,), dtype=torch.int64, device="cuda")
                for _ in range(inflight)]
    sharded = mode in (L.COMBINE_REDUCE_SCATTER, L.COMBINE_HASH, L.COMBINE_ROWS)  # disjoint per-rank results

    trace = []  # per query: [k, launch start, launch end, finalize start, complete end] (perf_counter)
    phases = {"plan": 0.0, "merge": 0.0, "finalize": 0.0, "close": 0.0, "finalize_c": 0.0, "decode": 0.0}
    star_work = [0, 0, 0]
    star_mbytes = [-1]

    def launch(k):
        """Plan + execute query k on its stream (streamed: segment chunks launch while the rest is planned), then
        enqueue the cross-rank merge of its table on the same stream."""
        c0 = time.perf_counter()
        trace.append([k, c0, 0.0, 0.0, 0.0])
        s, dt = streams[k % inflight], d_tables[k % inflight]
        # the plan's own table by default (its statistics words follow it: one copy back instead of two); the
        # combine merges whichever table the plan wrote
        dptr = dt.data_ptr() if caller_table else None
        plan = table.plan_execute(handles, q, s.cuda_stream, dptr)
        c1 = time.perf_counter()
        if mode in (L.COMBINE_ALL_REDUCE, L.COMBINE_REDUCE_SCATTER, L.COMBINE_HASH):
            combine_plan(plan, comm, s.cuda_stream, mode, kinds, d_table=dptr)
        phases["plan"] += c1 - c0
        phases["merge"] += time.perf_counter() - c1
        trace[-1][2] = time.perf_counter()
        return plan, s, dt, len(trace) - 1

    def complete(item):
        """Finalize query k (waits for its stream only) and release its plan."""
        plan, s, dt, ti = item
        c0 = time.perf_counter()
        trace[ti][3] = c0
        if mode == L.COMBINE_ROWS:
            res = combine_result_rows(table, plan.finalize(s.cuda_stream), comm)
        else:  # a reduce-scattered / exchanged plan finalizes this rank's share
            res = plan.finalize(s.cuda_stream, dt.data_ptr() if caller_table else None)
        c1 = time.perf_counter()
        tm = (0.0, 0.0, 0.0, 0.0)
        if q.timing:  # the kernel-timing pass only: timing events are marker packets between dependent dispatches
            try:
                tm = plan.timing_us()
            except L.UnsupportedQueryError:  # numGroupsLimit plans time their parts separately
                pass
        if w.star_tree and not args.no_star_tree:  # star-tree plans: traversal + pre-aggregated document scan
            k_us = (tm[3], 1)
            star_work[:] = plan.star_work()
            star_mbytes[0] = plan.star_metric_bytes()
        else:
            k_us = (tm[1], max(int(tm[2]), 1))  # scan launches of this query: summed duration, count
        fc_us, dec_us = plan.finalize_us
        plan.close()
        phases["finalize"] += c1 - c0
        phases["close"] += time.perf_counter() - c1
        trace[ti][4] = time.perf_counter()
        phases["finalize_c"] += fc_us * 1e-6
        phases["decode"] += dec_us * 1e-6
        return res, k_us

    def run(n, depth, keep=1):
        """n queries, at most `depth` in flight; returns (results, kernel timings) in query order.  Only the first
        `keep` results are kept (all with --verify): a server hands each result on and frees it, and holding more of
        them (C5: 51 MB of pinned host memory each) would grow the result buffer pool inside the timed region."""
        from collections import deque
        pending, res, kus = deque(), [], []

        def done(item):
            r, k = complete(item)
            if keep is None or len(res) < keep:
                res.append(r)
            kus.append(k)

        for k in range(n):
            pending.append(launch(k))
            if len(pending) >= depth:
                done(pending.popleft())
        while pending:
            done(pending.popleft())
        return res, kus

    import gc
    # as timeit does: a collector pass inside a sub-millisecond step is the harness's cost, not the query's.  Collected
    # before the warm-up, so the GPU does not sit idle between the warm-up and the timed region (an idle gap lets the
    # clocks drop, and the first timed queries pay the ramp).
    gc.collect()
    gc.disable()
    first = None
    ngroups = 0
    warmup_run = 0
    if args.warmup:
        w0 = time.perf_counter()
        first = run(args.warmup, inflight)[0][0]
        warmup_run = args.warmup
        # sustained load until the clocks are at their steady state (--warmup-ms): the extra steps are estimated
        # from the W steps' pace and agreed across ranks (every rank runs the same queries: their combines meet)
        per_step = (time.perf_counter() - w0) / args.warmup
        extra = min(1000, max(0, int(np.ceil((args.warmup_ms * 1e-3 - per_step * args.warmup) / max(per_step, 1e-6)))))
        if world > 1:
            e = torch.tensor([extra], dtype=torch.int64)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            extra = int(e.item())
        if extra:
            run(extra, inflight, keep=0)
            warmup_run += extra
        ngroups = len(first)
        if not args.verify:
            first = None  # its pinned buffer back to the pool: the timed region holds no result
    for k in phases:
        phases[k] = 0.0
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    del trace[:]
    t0 = time.perf_counter()
    timed, _ = run(args.steps, inflight, keep=None if args.verify else (0 if args.warmup else 1))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    gc.enable()
    timed_trace = [[r[0]] + [round((x - t0) * 1e6, 1) for x in r[1:]] for r in trace[:args.steps]]
    if args.step_trace and rank == 0:
        with open(args.step_trace, "w") as f:
            json.dump({"elapsed_us": elapsed * 1e6, "queries": timed_trace,
                       "fields": ["k", "launch_start_us", "launch_end_us", "finalize_start_us", "complete_end_us"]}, f)
    if args.verify and first is not None:  # FLOAT/DOUBLE sums vary in their last bits (atomicAdd order): 1e-9
        ref = first.as_dict()
        for res in timed:
            got = res.as_dict()
            assert got.keys() == ref.keys(), "groups differ between steps"
            for k, v in got.items():
                assert all(x == y or abs(x - y) <= 1e-9 * max(abs(x), abs(y)) for x, y in zip(v, ref[k])), k
    if not args.warmup and timed:
        ngroups = len(timed[0])
    del timed, first
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    if sharded:  # disjoint per-rank shards: the query's groups are their sum
        g = torch.tensor([ngroups], dtype=torch.int64)
        dist.all_reduce(g)
        ngroups = int(g.item())
    total_rows = float(total_segments) * docs
    value = total_rows * args.steps / elapsed
    # The per-query latency: a serialized pass after the timed region, one query at a time, plan to result in host
    # memory (merge included), with no timing events (as the timed region).
    # The scan kernel's duration for the roofline: a second serialized pass (one query in flight, so no other query's
    # kernels share the GPU with the one being timed) whose queries record timing events (PGPU_OPT_TIMING).
    nser = max(1, args.roofline_steps)
    torch.cuda.synchronize()
    t_ser = time.perf_counter()
    run(nser, 1, keep=0)
    torch.cuda.synchronize()
    latency_ms = (time.perf_counter() - t_ser) / nser * 1e3
    q.timing = True
    kernel_us = run(nser, 1, keep=0)[1]
    q.timing = False
    torch.cuda.synchronize()
    if world > 1:
        e = torch.tensor([latency_ms], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        latency_ms = float(e.item())
    launches = kernel_us[0][1] if kernel_us else 1
    kernel_avg_us = float(np.mean([k for k, _ in kernel_us])) / launches if kernel_us else 0.0  # per launch

    log("timed region done: %.3f ms/step" % (elapsed / args.steps * 1e3))
    roofline = None
    if not args.no_bytes and w.star_tree and not args.no_star_tree and star_work[0] > 0:
        # star-tree bytes model (line-granular): nodes x 28 B + star-tree documents read x the bits of
        # the dimensions they are read for + the metric arrays' 64-B sectors that hold a matched document (counted by
        # the kernel: pgpu_plan_star_metric_bytes; without it, 8 B per document per pre-aggregated array)
        preds = []
        if q.filter is not None:
            q.filter.postfix(preds, [])
        dims = sorted(set(q.group_by) | {p.column for p in preds})
        dim_bits = sum(_col_info(table, int(handles[0]), c)[1] for c in dims)
        nslots = probe_nslots
        metric_bytes = star_mbytes[0] if star_mbytes[0] >= 0 else star_work[2] * 8.0 * nslots
        per_doc = dim_bits / 8.0 + metric_bytes / max(star_work[2], 1)
        bytes_alg = star_work[1] * 28 + star_work[2] * dim_bits / 8.0 + metric_bytes
        achieved = bytes_alg / (kernel_avg_us * 1e-6) / 1e9 if kernel_avg_us > 0 else 0.0
        roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": None,
                    "bytes_alg_per_launch": int(bytes_alg), "kernel_us": round(kernel_avg_us, 2),
                    "kernels": "startree_traverse_kernel + startree_scan_kernel",
                    "star_segments": int(star_work[0]), "star_nodes": int(star_work[1]),
                    "star_docs_read": int(star_work[2]), "bytes_per_star_doc": round(per_doc, 3),
                    "star_metric_bytes": int(metric_bytes),
                    "launches_per_query": 1, "kernel_us_per_query": round(kernel_avg_us, 2)}
    if not args.no_bytes and (not w.star_tree or args.no_star_tree):  # scan-path bytes model
        bytes_alg, matched = compulsory_bytes(table, handles, q, docs, w.inverted_columns)
        bytes_alg /= launches  # equal chunks of statistically identical segments: per-launch share
        achieved = bytes_alg / (kernel_avg_us * 1e-6) / 1e9 if kernel_avg_us > 0 else 0.0
        roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": None,
                    "bytes_alg_per_launch": int(bytes_alg), "kernel_us": round(kernel_avg_us, 2),
                    "matched_docs_per_gpu": int(matched), "launches_per_query": launches,
                    "kernel_us_per_query": round(kernel_avg_us * launches, 2)}
    if roofline is not None and pmc:
        roofline["traffic"] = round(pmc["traffic"], 0)
        roofline["traffic_pmc"] = {k: v for k, v in pmc.items() if k != "traffic"}
    cpu = parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("bytes_alg pass done; full-size parity")
        parity = full_parity(table, handles, q, w, docs, args)
        log("parity %s; CPU baseline" % (parity and parity["ok"]))
        cpu = cpu_baseline(table, handles, q, w, docs, args)
    elif world > 1 and args.parity_segments != 0:
        # the merged answer (this rank's share of it for sharded combines) of one more query, against the oracle
        res = run(1, 1, keep=1)[0][0]
        log("rank %d: multi-rank parity" % rank)
        parity = multi_rank_parity(table, handles, q, w, docs, res, world, rank, sharded)
        if rank == 0:
            log("parity %s" % parity["ok"])

    if rank == 0:
        line = {
            "metric": "rows/sec scanned+aggregated (node) & % HBM peak, AdAnalytics GROUP BY query",
            "value": round(value, 1),
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup, "warmup_run": warmup_run,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            # ms_per_step is a pipelined throughput (--inflight queries overlap); one query alone takes this long
            "latency_ms_per_query": round(latency_ms, 4),
            "higher_is_better": True,
            "scaling": "weak" if args.segments_per_gpu else "strong",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (BASELINE.md §3 generators, built on the device)",
            "config": {"workload": w.name, "query": w.sql, "segments_per_gpu": nseg, "docs_per_segment": docs,
                       "rows_per_gpu": nseg * docs, "global_rows": int(total_rows), "parallelism": "dp%d" % world,
                       "groups": ngroups, "setup_s": round(t_gen, 1), "queries_in_flight": inflight,
                       "combine": L.COMBINE_NAMES[mode] + (" (pgpu_plan_combine, %s)" % backend if world > 1 else ""),
                       **({"executor_config": parse_config(args.config)} if args.config else {})},
            "roofline": roofline,
            "host_profile_us": {k: round(v / args.steps * 1e6, 1) for k, v in phases.items()} if args.host_profile else None,
            "cpu_baseline": cpu,
            "parity": parity,
        }
        print(json.dumps(line), flush=True)
    table.close()
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
