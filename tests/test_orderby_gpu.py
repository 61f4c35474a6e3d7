"""SQL ORDER BY / LIMIT end to end on the GPU, pinned by the reference's own expected result tables
(InterSegmentOrderBySingleValueQueriesTest.orderBySQLResultTableProvider, extracted to tests/golden/kat_orderby_sql.json
by tests/golden/make_golden_orderby.py).

The flow is BaseQueriesTest.getBrokerResponse (BaseQueriesTest.java:209-242): one server runs the query over two
copies of the KAT segment (HIP scan + combine, then the SQL server trim, GroupByOrderByCombineOperator /
IndexedTable.finish), serializes its DataTable V3, and the broker reduces two copies of those bytes
(GroupByDataTableReducer): 4 x 30000 = 120000 documents.  Rows must match in order; SUM / MIN / AVG values are
compared to the printed doubles with 1e-12 relative tolerance (the reference prints e.g. 909380310.3521485), COUNT
and keys exactly; the statistics exactly.
"""
import json
import os

import pytest

import kat_common as K
from pinot_amd.executor import GpuTable, broker_reduce_sql
from pinot_amd.query import parse_query

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "kat_orderby_sql.json")))["cases"]


@pytest.fixture(scope="module")
def server(oracle, gpu_lib):
    seg = K.kat_segment(oracle, pairs=True)
    t = GpuTable(K.SCHEMA)
    hs = [t.pin_segment(seg), t.pin_segment(seg)]
    yield t, hs
    t.close()


def _same_value(got, exp):
    if isinstance(exp, str) or isinstance(exp, int) and not isinstance(exp, bool):
        return got == exp
    return got == pytest.approx(exp, rel=1e-12)


@pytest.mark.parametrize("case", CASES, ids=[c["query"][:90] for c in CASES])
def test_orderby_sql_kat(server, case):
    t, hs = server
    q = parse_query(case["query"])
    r = t.execute_groupby(hs, q)
    dt = r.trim_sql().datatable()
    resp = broker_reduce_sql([dt, dt], q)
    rt = resp["resultTable"]
    assert rt["dataSchema"]["columnNames"] == case["dataSchema"]["columnNames"]
    assert rt["dataSchema"]["columnDataTypes"] == case["dataSchema"]["columnDataTypes"]
    rows = rt["rows"]
    assert len(rows) == len(case["rows"]), (rows, case["rows"])
    for got, exp in zip(rows, case["rows"]):
        assert len(got) == len(exp)
        assert all(_same_value(g, e) for g, e in zip(got, exp)), (got, exp)
    got_stats = [resp["numDocsScanned"], resp["numEntriesScannedInFilter"], resp["numEntriesScannedPostFilter"],
                 resp["totalDocs"]]
    assert got_stats == case["stats"]


def test_trim_sql_keeps_order_by_prefix(server):
    """Server trim keeps the top max(limit * 5, minServerGroupTrimSize) groups: with the trim size lowered to 2 and
    LIMIT 1 the server keeps 5 groups, the first 5 of the full ORDER BY."""
    t, hs = server
    full = parse_query("SELECT column12, SUM(column1) FROM testTable GROUP BY column12 ORDER BY SUM(column1) DESC "
                       "LIMIT 100")
    small = parse_query("SELECT column12, SUM(column1) FROM testTable GROUP BY column12 ORDER BY SUM(column1) DESC "
                        "LIMIT 1")
    small.min_server_group_trim_size = 2
    r = t.execute_groupby(hs, full)
    a = r.trim_sql(full)
    b = r.trim_sql(small)
    assert len(a) == 9 and len(b) == 5
    assert b.keys == a.keys[:5]
    assert [v[0] for v in b.values] == [v[0] for v in a.values[:5]]
    sums = [v[0] for v in a.values]
    assert sums == sorted(sums, reverse=True)


def test_trim_pql_top_per_function(server):
    """AggregationGroupByTrimmingService: per function the top groups, MIN ascending, the others descending."""
    t, hs = server
    q = parse_query("SELECT SUM(column1), MIN(column6) FROM testTable GROUP BY column12 TOP 3")
    r = t.execute_groupby(hs, q)
    allg = r.as_dict()
    top = r.trim_pql(3, final=True)
    exp_sum = sorted(allg.items(), key=lambda kv: -kv[1][0])[:3]
    exp_min = sorted(allg.items(), key=lambda kv: kv[1][1])[:3]
    assert [v for _, v in top[0]] == [v[0] for _, v in exp_sum]
    assert [v for _, v in top[1]] == [v[1] for _, v in exp_min]
