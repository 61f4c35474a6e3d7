"""Aggregate queries/s of concurrent queries on one pinned table (the serving model: many queries at once over the
same segments, BaseCombineOperator.java:85-115).  Each of --threads host threads runs whole queries (plan from the
table's plan cache, scan, finalize into host memory) on its own HIP stream for --seconds; the line reports the
total queries/s and rows/s over all threads.

    python tools/qps.py --workload c1 --segments 1 --threads 1 4
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c1")
    ap.add_argument("--segments", type=int, default=1)
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--threads", type=int, nargs="+", default=[1, 4])
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--uncached", action="store_true", help="compile every plan afresh (PGPU_OPT_NO_PLAN_CACHE)")
    args = ap.parse_args()
    import torch
    from pinot_amd.executor import GpuTable
    from pinot_amd.query import parse_query
    from pinot_amd.workloads import WORKLOADS
    torch.cuda.set_device(0)
    w = WORKLOADS[args.workload]()
    t = GpuTable(w.schema)
    hs = [t.generate_segment(w.gen, row0=i * args.docs, num_docs=args.docs) for i in range(args.segments)]
    ref = t.execute_groupby(hs, parse_query(w.sql, num_groups_limit=w.num_groups_limit)).as_dict()
    out = {"workload": w.name, "query": w.sql, "segments": args.segments, "docs_per_segment": args.docs,
           "plan_cache": not args.uncached, "runs": []}
    for nt in args.threads:
        counts = [0] * nt
        bad = []
        stop = threading.Event()
        barrier = threading.Barrier(nt + 1)

        def worker(k):
            s = torch.cuda.Stream()
            q = parse_query(w.sql, num_groups_limit=w.num_groups_limit)
            q.no_plan_cache = args.uncached
            barrier.wait()
            while not stop.is_set():
                r = t.execute_groupby(hs, q, s.cuda_stream)
                if counts[k] == 0 and r.as_dict() != ref:
                    bad.append(k)
                counts[k] += 1

        ths = [threading.Thread(target=worker, args=(k,)) for k in range(nt)]
        for th in ths:
            th.start()
        barrier.wait()
        t0 = time.perf_counter()
        time.sleep(args.seconds)
        stop.set()
        for th in ths:
            th.join()
        dt = time.perf_counter() - t0
        n = sum(counts)
        out["runs"].append({"threads": nt, "queries": n, "seconds": round(dt, 3), "qps": round(n / dt, 1),
                            "rows_per_s": round(n * args.segments * args.docs / dt, 1),
                            "per_thread": counts, "results_match": not bad})
        print("[qps] %d threads: %.1f queries/s" % (nt, n / dt), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)
    t.close()


if __name__ == "__main__":
    main()
