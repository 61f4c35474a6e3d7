"""Concurrent queries on one table (Pinot's serving model: many queries at once over the same segments, one task per
segment each, BaseCombineOperator.java:85-115; SURVEY.md §8b threading).

Several host threads run a mix of C1- and C3-shaped queries (filtered group-by, aggregation-only, a large dense
table) on one pinned table at the same time -- through the plan cache and around it, on the table's stream and on
their own streams -- and every result must equal the oracle's.  Pinned state changes under running queries too: a
segment unpinned while a plan that references it is alive (the reference-counted SegmentDataManager contract), and
pins that grow a global dictionary while other threads' plans run on the old key space (dictionary snapshots: the
groups of a plan never get re-labelled)."""
import threading

import numpy as np
import pytest

from pinot_amd import _lib as L
from pinot_amd.executor import GpuTable
from pinot_amd.query import parse_query
from pinot_amd.segment import SegmentBuffers
from pinot_amd.workloads import WORKLOADS

pytestmark = pytest.mark.gpu
DOCS = 200_000
NSEG = 6
REL = 1e-9

QUERIES = [
    # C3 (the README AdAnalytics query)
    "SELECT sum(clicks), sum(impressions) FROM t WHERE daysSinceEpoch BETWEEN 17849 AND 17856 "
    "AND accountId IN (123456789) GROUP BY daysSinceEpoch",
    # C1-shaped: a 50 % range filter, one aggregate, a low-cardinality key
    "SELECT SUM(clicks) FROM t WHERE impressions BETWEEN 25000 AND 74999 GROUP BY daysSinceEpoch",
    # set leaf + range leaf, COUNT / MAX by the set column
    "SELECT COUNT(*), MAX(impressions), MIN(clicks) FROM t WHERE accountId IN (123456789, 1000037, 1000074) "
    "AND daysSinceEpoch >= 17800 GROUP BY accountId",
    # aggregation-only
    "SELECT SUM(impressions), MIN(clicks), COUNT(*) FROM t WHERE clicks < 100",
    # a dense global table (365 x 1000 keys)
    "SELECT COUNT(*), SUM(impressions) FROM t WHERE accountId <> 123456789 GROUP BY daysSinceEpoch, clicks",
]


def _oracle_segments(oracle, w, seg_ids):
    segs = []
    for i in seg_ids:
        cols = {}
        for (name, typ), g in zip(w.schema, w.gen):
            cols[name] = oracle.build_column(L.TYPE_NAMES[typ], oracle.gen_values(g, i * DOCS, DOCS))
        segs.append(SegmentBuffers(DOCS, cols))
    return segs


def _diff(got, exp):
    """None when equal, else a short description (never the whole group maps: pytest would render them)."""
    gk, ek = set(got), set(exp)
    missing, extra = ek - gk, gk - ek
    bad = []
    for k in ek & gk:
        gv, ev = got[k], exp[k]
        for x, y in zip(gv, ev):
            same = x == pytest.approx(y, rel=REL) if isinstance(y, float) and not float(y).is_integer() else x == y
            if not same:
                bad.append((k, gv, ev))
                break
    if not missing and not extra and not bad:
        return None
    return "groups %d vs %d, missing %d %s, extra %d %s, value diffs %d %s" % (
        len(got), len(exp), len(missing), sorted(missing)[:2], len(extra), sorted(extra)[:2], len(bad), bad[:2])


def _same(got, exp):
    d = _diff(got, exp)
    assert d is None, d


@pytest.fixture(scope="module")
def c3(oracle, gpu_lib):
    w = WORKLOADS["adanalytics"]()
    t = GpuTable(w.schema)
    hs = [t.generate_segment(w.gen, row0=i * DOCS, num_docs=DOCS) for i in range(NSEG)]
    segs = _oracle_segments(oracle, w, range(NSEG))
    expected = {}
    for qi, sql in enumerate(QUERIES):
        for sub in ("all", "half"):
            ss = segs if sub == "all" else segs[::2]
            o = oracle.run_groupby(w.schema, ss, parse_query(sql))
            expected[(qi, sub)] = o.groups
    yield w, t, hs, segs, expected
    t.close()


def test_queries_sequential(c3):
    """Every query of the mix, one at a time, on both segment subsets (the baseline the threads are held to)."""
    w, t, hs, segs, expected = c3
    for rep in range(2):  # the second round hits the plan cache (device-resident plan images)
        for qi, sql in enumerate(QUERIES):
            for sub in ("all", "half"):
                q = parse_query(sql)
                r = t.execute_groupby(hs if sub == "all" else hs[::2], q)
                d = _diff(r.as_dict(), expected[(qi, sub)])
                assert d is None, (rep, qi, sub, d)


def _run_threads(t, hs, expected, nthreads, per_thread, stream_mode, uncached_every):
    """nthreads x per_thread queries of the mix; returns the mismatches as (thread, query index, subset, uncached,
    stream kind, description)."""
    import torch
    errors = []
    start = threading.Barrier(nthreads)
    stop = threading.Event()  # the first mismatch stops every thread (nothing runs on a state already wrong)

    def worker(tid):
        try:
            own = stream_mode == "own" or (stream_mode == "mixed" and tid >= nthreads // 2)
            stream = torch.cuda.Stream() if own else None  # None: the table's own stream
            handle = stream.cuda_stream if stream is not None else None
            start.wait()
            for i in range(per_thread):
                if stop.is_set():
                    return
                qi = (tid + i) % len(QUERIES)
                sub = "all" if (i // len(QUERIES)) % 2 == 0 else "half"
                q = parse_query(QUERIES[qi])  # per-thread query objects (their C form is cached on them)
                q.no_plan_cache = uncached_every > 0 and (i + tid) % uncached_every == 0
                r = t.execute_groupby(hs if sub == "all" else hs[::2], q, handle)
                d = _diff(r.as_dict(), expected[(qi, sub)])
                if d:
                    errors.append((tid, qi, sub, q.no_plan_cache, "own" if own else "table", d))
                    stop.set()
        except Exception as e:  # noqa: BLE001 -- reported by the main thread
            errors.append((tid, -1, "", False, "", repr(e)))
            stop.set()

    threads = [threading.Thread(target=worker, args=(k,)) for k in range(nthreads)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=100)
    assert not any(th.is_alive() for th in threads), "a query thread hung"
    return errors


@pytest.mark.parametrize("stream_mode,uncached_every", [("table", 0), ("own", 0), ("mixed", 3)])
def test_concurrent_queries_one_table(c3, stream_mode, uncached_every):
    """4 threads x 20 queries, mixed shapes, segment subsets, cached and uncached plans, the table's stream and
    per-thread streams: every result equals the oracle's."""
    w, t, hs, segs, expected = c3
    errors = _run_threads(t, hs, expected, 4, 20, stream_mode, uncached_every)
    assert not errors, "%d mismatches, first: %s" % (len(errors), errors[:3])


def test_unpin_while_plan_alive(oracle, gpu_lib):
    """A plan keeps its segments alive: unpinning one after the plan is made (before it executes) defers the free,
    and the plan still answers over the segment set it was planned on."""
    w = WORKLOADS["adanalytics"]()
    t = GpuTable(w.schema)
    try:
        hs = [t.generate_segment(w.gen, row0=i * DOCS, num_docs=DOCS) for i in range(2)]
        segs = _oracle_segments(oracle, w, range(2))
        q = parse_query(QUERIES[1])
        exp = oracle.run_groupby(w.schema, segs, q).groups
        with t.plan(hs, q) as p:
            t.unpin_segment(hs[1])
            assert t.num_segments() == 1
            p.execute()
            _same(p.finalize().as_dict(), exp)
        with pytest.raises(L.PinotGpuError):
            t.execute_groupby(hs, q)  # the handle is gone for new plans
        _same(t.execute_groupby(hs[:1], q).as_dict(), oracle.run_groupby(w.schema, segs[:1], q).groups)
    finally:
        t.close()


def test_pins_grow_dictionaries_under_running_queries(oracle, gpu_lib):
    """While threads run group-by queries over the first segments, the main thread pins segments whose values
    extend the group-by columns' global dictionaries (new days, new clicks values below the old minimum: every old
    dictId shifts).  Plans made before a pin keep their LUTs and dictionary snapshot, so their groups are right;
    queries over every segment after the pins see the new values."""
    import torch
    w = WORKLOADS["adanalytics"]()
    t = GpuTable(w.schema)
    try:
        hs = [t.generate_segment(w.gen, row0=i * DOCS, num_docs=DOCS) for i in range(3)]
        segs = _oracle_segments(oracle, w, range(3))
        sqls = [QUERIES[1], "SELECT COUNT(*), SUM(impressions) FROM t WHERE impressions < 50000 GROUP BY clicks"]
        exp = [oracle.run_groupby(w.schema, segs, parse_query(s)).groups for s in sqls]
        shifted = [dict(g) for g in w.gen]
        shifted[0].update(lo=17000, hi=17600)   # days before the old minimum: every daysSinceEpoch id shifts
        shifted[2].update(lo=-500, hi=700)       # clicks below 0
        errors, stop = [], threading.Event()

        def worker(k):
            try:
                stream = torch.cuda.Stream()
                n = 0
                while not stop.is_set() or n < 4:
                    q = parse_query(sqls[k % 2])
                    q.no_plan_cache = n % 2 == 1
                    _same(t.execute_groupby(hs, q, stream.cuda_stream).as_dict(), exp[k % 2])
                    n += 1
            except Exception as e:  # noqa: BLE001
                errors.append((k, repr(e)))

        threads = [threading.Thread(target=worker, args=(k,)) for k in range(3)]
        for th in threads:
            th.start()
        new = [t.generate_segment(shifted, row0=(10 + i) * DOCS, num_docs=DOCS) for i in range(2)]
        stop.set()
        for th in threads:
            th.join(timeout=300)
        assert not any(th.is_alive() for th in threads)
        assert not errors, errors[:3]
        # every segment, after the pins: the new values are groups too
        ws = WORKLOADS["adanalytics"]()
        ws.gen = shifted
        all_segs = segs + _oracle_segments(oracle, ws, [10, 11])
        for s in sqls:
            q = parse_query(s)
            _same(t.execute_groupby(hs + new, q).as_dict(), oracle.run_groupby(w.schema, all_segs, q).groups)
    finally:
        t.close()


def test_init_shutdown_and_free_result(gpu_lib):
    """Process lifecycle entry points: pgpu_init brings up every visible device (idempotent),
    pgpu_free_result releases a result, pgpu_shutdown drains the devices."""
    import ctypes
    lib = L.load()
    n = lib.pgpu_init(0)
    assert n >= 1, L.last_error()
    assert lib.pgpu_init(1) == 1
    assert lib.pgpu_init(n + 1) == L.PGPU_ERR_INVALID_ARGUMENT
    w = WORKLOADS["c1"]()
    t = GpuTable(w.schema)
    try:
        h = t.generate_segment(w.gen, row0=0, num_docs=10000)
        q, keep = parse_query(w.sql).to_c(t.index)
        hs = (ctypes.c_int64 * 1)(h)
        r = ctypes.c_void_p()
        L.check(lib.pgpu_execute_groupby(t.handle, hs, 1, ctypes.byref(q), None, ctypes.byref(r)))
        ng = ctypes.c_int64()
        L.check(lib.pgpu_result_num_groups(r, ctypes.byref(ng)))
        assert ng.value == 16
        assert lib.pgpu_free_result(r) == 0
    finally:
        t.close()
    assert lib.pgpu_shutdown() == 0
