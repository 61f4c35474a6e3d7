"""Pins the oracle to the reference's own known-answer tests on test_data-sv.avro (CPU only).

InnerSegmentAggregationSingleValueQueriesTest.java:119-219 (four group-by shapes, one per RawKeyHolder, with and
without the BaseSingleValueQueriesTest.java:73-74 filter) and InterSegmentOrderBySingleValueQueriesTest.java
(4 segments = the same segment on 2 "servers" x 2 segments each, BaseQueriesTest.java:209-242).
"""
import pytest

import kat_common as K
from pinot_amd.query import QueryContext


@pytest.fixture(scope="module")
def sv_segment(oracle):
    return K.kat_segment(oracle)


def test_segment_cardinalities(sv_segment):
    # BaseSingleValueQueriesTest.java:49-62 (column12's javadoc value is stale; the data holds 9 values)
    expect = {"column1": 6582, "column3": 21910, "column5": 1, "column6": 608, "column7": 146, "column9": 1737,
              "column11": 5, "column17": 24, "column18": 1440, "daysSinceEpoch": 2}
    for c, card in expect.items():
        assert sv_segment.columns[c].cardinality == card, c
    assert sv_segment.num_docs == 30000


@pytest.mark.parametrize("case", K.KAT["inner_segment_group_by"], ids=lambda c: c["holder"])
@pytest.mark.parametrize("with_filter", [False, True], ids=["no_filter", "filter"])
def test_inner_segment_group_by(oracle, sv_segment, case, with_filter):
    q = K.inner_query(case["group_by"], with_filter)
    r = oracle.run_groupby(K.SCHEMA, [sv_segment], q, combine=False)
    exp = case["filter" if with_filter else "no_filter"]
    assert r.holder == case["holder"]
    docs, in_filter, post, total = exp["stats"]
    assert r.stats == (docs, in_filter, post, total)
    key = K.key_tuple(case["group_by"], exp["key"])
    assert key in r.groups
    K.check_inner_values(r.groups[key], exp["values"])


@pytest.mark.parametrize("with_filter", [False, True], ids=["no_filter", "filter"])
def test_aggregation_only_totals(oracle, sv_segment, with_filter):
    """InnerSegmentAggregationSingleValueQueriesTest.java:55-75, as the single group of GROUP BY column5
    (cardinality 1): the group's values are the aggregation-only totals."""
    q = K.inner_query(["column5"], with_filter)
    r = oracle.run_groupby(K.SCHEMA, [sv_segment], q, combine=False)
    exp = K.KAT["inner_segment_aggregation_only"]["filter" if with_filter else "no_filter"]
    assert list(r.groups) == [("gFuH",)]
    K.check_inner_values(r.groups[("gFuH",)], exp["values"])
    assert r.stats[0] == exp["stats"][0]


@pytest.mark.parametrize("case", K.KAT["inter_segment_group_by"], ids=lambda c: "_".join(c["group_by"]))
def test_inter_segment_group_by(oracle, sv_segment, case):
    q = QueryContext(case["group_by"], [tuple(a) for a in case["aggs"]])
    r = oracle.run_groupby(K.SCHEMA, [sv_segment] * K.KAT["inter_segment_num_segments"], q, combine=True)
    assert r.stats == tuple(case["stats"])
    rows = {K.key_tuple(case["group_by"], k): v for k, v in case["rows"]}
    if case["complete"]:
        assert set(r.groups) == set(rows)
    for k, v in rows.items():
        assert [float(x) for x in r.groups[k]] == [float(x) for x in v], k


def test_num_groups_limit(oracle, sv_segment):
    """InterSegmentAggregationSingleValueQueriesTest.java:534-545: GROUP BY column1 reaches numGroupsLimit 1000."""
    q = QueryContext(["column1"], [("COUNT", "*")], None, num_groups_limit=1000)
    r = oracle.run_groupby(K.SCHEMA, [sv_segment] * 4, q, combine=True, max_initial_capacity=1000)
    assert r.holder == "INT_MAP"
    assert r.limit_reached
    q = QueryContext(["column1"], [("COUNT", "*")])
    assert not oracle.run_groupby(K.SCHEMA, [sv_segment] * 4, q, combine=True).limit_reached


@pytest.mark.parametrize("with_filter", [False, True], ids=["no_filter", "filter"])
def test_aggregation_only_inner_segment(oracle, sv_segment, with_filter):
    """InnerSegmentAggregationSingleValueQueriesTest.java:55-75: a true aggregation-only query (no GROUP BY):
    one group with the empty key, AggregationOperator statistics."""
    q = K.inner_query([], with_filter)
    r = oracle.run_groupby(K.SCHEMA, [sv_segment], q, combine=False)
    exp = K.KAT["inner_segment_aggregation_only"]["filter" if with_filter else "no_filter"]
    assert list(r.groups) == [()]
    K.check_inner_values(r.groups[()], exp["values"])
    assert r.stats == tuple(exp["stats"])


@pytest.mark.parametrize("case", K.KAT_AGG["cases"], ids=lambda c: "%s_%s" % (c["test"], c["variant"]))
def test_inter_segment_aggregation(oracle, sv_segment, case):
    """InterSegmentAggregationSingleValueQueriesTest SUM/COUNT/MIN/MAX/AVG KATs (values and statistics; the
    metadata / dictionary-based operators' zero post-filter entries included)."""
    from pinot_amd.executor import aggregation_defaults
    q = K.agg_case_query(case)
    r = oracle.run_groupby(K.SCHEMA, [sv_segment] * 4, q, combine=True)
    if q.group_by:
        values = K.top_group_values(q, list(r.groups.values()))
    else:
        values = r.groups[()] if r.groups else aggregation_defaults(q.aggregations)
    K.check_agg_case(case, q, r.stats, values)
