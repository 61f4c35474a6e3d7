"""Query deadlines on the GPU path (QueryContext.getEndTimeMs): the combine gives up at the end time and reports a
timeout instead of a result (BaseCombineOperator.java:193-203 for aggregation-only, GroupByCombineOperator.java:
193-203 for group-by).  Here: a deadline already past launches nothing; a deadline that passes while the scan runs
returns the timeout at the deadline (well before the scan would have finished; the device work left running keeps
its scratch until it completes, as Pinot's worker threads run to their next block); a generous deadline changes
nothing; the table stays usable after a timeout."""
import time

import pytest

from pinot_amd import _lib as L
from pinot_amd.executor import GpuTable
from pinot_amd.query import FilterContext, Predicate, QueryContext

pytestmark = pytest.mark.gpu

SCHEMA = [("a", "INT"), ("b", "INT"), ("m", "INT"), ("c", "INT")]
GEN = [{"kind": "UNIFORM", "column_index": 0, "lo": 0, "hi": 100_000},
       {"kind": "UNIFORM", "column_index": 1, "lo": 0, "hi": 100_000},
       {"kind": "UNIFORM", "column_index": 2, "lo": 0, "hi": 1000},
       {"kind": "UNIFORM", "column_index": 3, "lo": 0, "hi": 100}]
DOCS = 1_000_000


@pytest.fixture(scope="module")
def table():
    t = GpuTable(SCHEMA, device=0)
    handles = [t.generate_segment(GEN, row0=i * DOCS, num_docs=DOCS) for i in range(96)]
    yield t, handles
    t.close()


def _agg_query():
    return QueryContext([], [("COUNT", "*"), ("SUM", "m"), ("MAX", "a")],
                        filter=FilterContext.pred(Predicate.range("b", "1000", "89999")))


def _hash_query():
    # GROUP BY a, b: 10^10 keys -> the open-addressing hash table, one global atomic per doc (a slow scan)
    q = QueryContext(["a", "b"], [("COUNT", "*"), ("SUM", "m")], num_groups_limit=0)
    q.timing = True  # the tests size their deadlines from the scan's timing events (PGPU_OPT_TIMING)
    return q


def test_timing_events_are_opt_in(table):
    """Timing events only for a query with PGPU_OPT_TIMING; both forms share one cached plan and agree."""
    t, handles = table
    q = _agg_query()
    with t.plan_execute(handles, q) as p:
        untimed = p.finalize()
        with pytest.raises(L.PinotGpuError) as e:
            p.timing_us()
        assert e.value.code == L.PGPU_ERR_INVALID_ARGUMENT
    q.timing = True
    with t.plan_execute(handles, q) as p:
        timed = p.finalize()
        tm = p.timing_us()
    assert tm[0] >= tm[1] > 0 and tm[2] >= 1
    assert timed.values == untimed.values and timed.stats.as_tuple() == untimed.stats.as_tuple()


def test_deadline_already_past(table):
    t, handles = table
    q = _agg_query()
    q.end_time_ms = int(time.time() * 1000) - 5
    with pytest.raises(L.QueryTimeoutError) as e:
        t.execute_groupby(handles, q)
    assert "250" in e.value.message and "Timed out while polling results block" in e.value.message
    g = QueryContext(["m"], [("COUNT", "*")])
    g.end_time_ms = int(time.time() * 1000) - 5
    with pytest.raises(L.QueryTimeoutError) as e:
        t.execute_groupby(handles, g)
    assert "Timed out while combining group-by results" in e.value.message


def test_generous_deadline_same_result(table):
    t, handles = table
    base = t.execute_aggregation(handles, _agg_query())
    q = _agg_query().set_timeout(60_000)
    got = t.execute_aggregation(handles, q)
    assert got.values == base.values
    assert got.stats.as_tuple() == base.stats.as_tuple()
    assert base.stats.num_docs_scanned > 0


def test_deadline_stops_running_scan(table):
    t, handles = table
    q = _hash_query()
    with t.plan(handles, q) as p:  # device time of the whole scan, no finalize (tens of millions of groups)
        p.execute()
        full_us = p.timing_us()[1]
    assert full_us > 4_000, "the hash-table scan of %d docs took only %.0f us" % (len(handles) * DOCS, full_us)
    budget_ms = max(1, int(full_us / 1000 / 8))
    q.set_timeout(budget_ms)
    t0 = time.perf_counter()
    with pytest.raises(L.QueryTimeoutError):
        with t.plan(handles, q) as p:
            p.execute()
            p.finalize()
    elapsed_ms = (time.perf_counter() - t0) * 1000
    # returned at the deadline (plus planning and the wait's polling), far before the full scan
    assert elapsed_ms < budget_ms + 0.6 * full_us / 1000, (elapsed_ms, budget_ms, full_us)
    # the table stays usable: the next queries queue behind the abandoned scan on a fresh scratch
    after = t.execute_aggregation(handles, _agg_query())
    assert after.values == t.execute_aggregation(handles, _agg_query()).values
    assert after.stats.num_docs_scanned > 0


def test_deadline_partitioned_and_streamed(table):
    t, handles = table
    # GROUP BY a, c: 10^7 keys x 2 slots = a 160 MB dense table -> the partitioned group-by (K8a..K8d)
    q = QueryContext(["a", "c"], [("COUNT", "*"), ("SUM", "m")], num_groups_limit=0,
                     filter=FilterContext.pred(Predicate.range("m", "0", "499")))
    q.end_time_ms = int(time.time() * 1000) - 1
    with pytest.raises(L.QueryTimeoutError):
        t.execute_groupby(handles, q)
    with pytest.raises(L.QueryTimeoutError):
        with t.plan_execute(handles, q) as p:
            p.finalize()
    q.end_time_ms = 0
    r = t.execute_groupby(handles[:2], q)
    assert len(r) > 0


# ------------------------------------------------------------------------------------------------- cancellation
# pgpu_plan_cancel: the broker abandoned the query; Pinot's combine cancels its futures and each segment operator
# stops at its next block (BaseOperator.java:37-39 EarlyTerminationException, BaseCombineOperator.java:124-130).

def test_cancel_from_another_thread_ends_the_wait(table):
    import threading
    t, handles = table
    q = _hash_query()
    with t.plan(handles, q) as p:
        p.execute()
        full_us = p.timing_us()[1]
    assert full_us > 4_000, full_us
    box = {}
    with t.plan_execute(handles, q) as p:
        def canceller():
            time.sleep(full_us / 8 / 1e6)
            box["t"] = time.perf_counter()
            p.cancel()
        th = threading.Thread(target=canceller)
        t0 = time.perf_counter()
        th.start()
        with pytest.raises(L.QueryCancelledError) as e:
            p.finalize()
        t1 = time.perf_counter()
        th.join()
        assert "cancelled" in e.value.message
        # the waiting finalize returned right after the cancel, long before the scan could have finished
        assert (t1 - box["t"]) * 1e6 < 0.5 * full_us, (t1 - box["t"], full_us)
        assert (t1 - t0) * 1e6 < 0.75 * full_us
        with pytest.raises(L.QueryCancelledError):  # and so does any later finalize of the plan
            p.finalize()
    after = t.execute_aggregation(handles, _agg_query())
    assert after.values == t.execute_aggregation(handles, _agg_query()).values


def test_cancel_running_c3_scan_then_next_query_correct(oracle, gpu_lib):
    """The README AdAnalytics query (C3) over 64 segments of 1M rows: cancelled from another thread while its scan is
    queued / running on the GPU, the finalize reports PGPU_ERR_CANCELLED; the next query on the table -- on the plan
    cache's image and a fresh scratch -- equals the oracle's answer."""
    import threading
    import _oracle
    from pinot_amd.query import parse_query
    from pinot_amd.workloads import WORKLOADS
    w = WORKLOADS["adanalytics"]()
    q = parse_query(w.sql, num_groups_limit=w.num_groups_limit)
    t = GpuTable(w.schema, device=0)
    try:
        docs = 1_000_000
        hs = [t.generate_segment(w.gen, row0=i * docs, num_docs=docs) for i in range(64)]
        base = t.execute_groupby(hs, q)  # also fills the plan cache
        for _ in range(3):
            p = t.plan_execute(hs, q)
            th = threading.Thread(target=p.cancel)
            th.start()
            th.join()
            with pytest.raises(L.QueryCancelledError):
                p.finalize()
            p.close()
        p = t.plan(hs, q)  # cancelled before it runs: nothing is launched
        p.cancel()
        with pytest.raises(L.QueryCancelledError):
            p.execute()
        p.close()
        r = t.execute_groupby(hs, q)
        assert r.as_dict() == base.as_dict() and r.stats.as_tuple() == base.stats.as_tuple()
        r8 = t.execute_groupby(hs[:8], q)
        assert r8.as_dict() == _oracle.run_groupby(w.schema, _oracle.segments_from_table(t, hs[:8], w.schema, docs),
                                                   q).groups
    finally:
        t.close()
