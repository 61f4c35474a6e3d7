"""The reference-interface views over a group-by result (pinot_amd.operators): GroupKeyGenerator iterators,
GroupByResultHolder accessors and AggregationGroupByResult.getResultForGroupId, on a result built on the host
(no device needed) -- the same objects the GPU operators return."""
from pinot_amd.executor import AvgPair, ExecutionStatistics, GroupByResult
from pinot_amd.operators import (DELIMITER, AggregationGroupByResult, GpuGroupKeyGenerator, IntermediateResultsBlock,
                                 _holders)


def _result():
    keys = [(1, "a"), (1, "b"), (7, "a")]
    values = [[3, 10.5, AvgPair(9.0, 3)], [1, -2.0, AvgPair(4.0, 1)], [2, 0.25, AvgPair(1.0, 2)]]
    return GroupByResult(keys=keys, values=values, stats=ExecutionStatistics([6, 0, 12, 100, 1, 1]))


AGGS = [("COUNT", "*"), ("SUM", "m"), ("AVG", "m")]


def test_group_key_generator_iterators():
    r = _result()
    gen = GpuGroupKeyGenerator(r, key_cards=[10, 2])
    assert gen.getNumKeys() == 3 and gen.getGlobalGroupKeyUpperBound() == 20
    keys = list(gen.getGroupKeys())
    assert [k._groupId for k in keys] == [0, 1, 2] and keys[2]._keys == [7, "a"]
    skeys = list(gen.getStringGroupKeys())
    assert skeys[1]._stringKey == "1" + DELIMITER + "b" and skeys[1].getKeys() == ["1", "b"]


def test_aggregation_group_by_result():
    r = _result()
    agb = AggregationGroupByResult(GpuGroupKeyGenerator(r), AGGS, _holders(r, AGGS))
    got = {}
    for sk in agb.getStringGroupKeyIterator():
        got[sk._stringKey] = [agb.getResultForKey(sk, i) for i in range(len(AGGS))]
    assert got["7" + DELIMITER + "a"] == [2, 0.25, AvgPair(1.0, 2)]
    assert isinstance(agb.getResultForGroupId(0, 0), int) and agb.getResultForGroupId(1, 1) == -2.0
    block = IntermediateResultsBlock(AGGS, r)
    assert block.getAggregationGroupByResult().getResultForGroupId(2, 0) == AvgPair(9.0, 3)
    assert block.get_aggregation_group_by_result() == r.string_keys()
    assert not block.getNumGroupsLimitReached()
