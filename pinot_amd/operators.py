"""Operator-level mirror of the reference interface on this path: the same names and result shapes as Pinot's own
operators, so a caller (and the tests) read a GPU result exactly as they read Pinot's.

  GpuAggregationGroupByOperator   AggregationGroupByOperator (core/operator/query/AggregationGroupByOperator.java:
                                  62-120): one segment -> IntermediateResultsBlock holding an AggregationGroupByResult
                                  and ExecutionStatistics.
  GpuGroupByCombineOperator       GroupByCombineOperator (core/operator/combine/GroupByCombineOperator.java:75-223):
                                  all segments of a server in one GPU pass, merged in the table-global key space.
  GpuAggregationOperator          AggregationOperator (core/operator/query/AggregationOperator.java:58-95).
  GpuAggregationOnlyCombineOperator  AggregationOnlyCombineOperator: the same over all segments in one pass.

The group-by result is exposed through the reference's own interfaces, as views over the columnar arrays the C ABI
returns (no per-group Python objects until a caller iterates):
  GpuGroupKeyGenerator     GroupKeyGenerator (core/query/aggregation/groupby/GroupKeyGenerator.java:29-110):
                           getGroupKeys / getStringGroupKeys iterators of GroupKey {_groupId, _keys} and
                           StringGroupKey {_groupId, _stringKey}, getNumKeys, getGlobalGroupKeyUpperBound;
  GpuGroupByResultHolder   DoubleGroupByResultHolder / ObjectGroupByResultHolder (GroupByResultHolder.java:32-69):
                           getDoubleResult(groupKey) / getResult(groupKey) (AvgPair for AVG);
  AggregationGroupByResult AggregationGroupByResult.java:31-81: getGroupKeyIterator, getStringGroupKeyIterator,
                           getResultForKey, getResultForGroupId (AggregationFunction.extractGroupByResult).
Group ids are dense [0, numKeys) in the result's order (ascending composite key -- hash-mode results of >= 4096 groups
in partition order, as the LONG_MAP holder's iterator runs in hash order), the order the ARRAY holder's
iterator produces.  Errors follow the reference: a bad literal raises BadQueryRequestException; a shape outside
the GPU path raises UnsupportedQueryError (the Java shim keeps Pinot's CPU operator for it).
"""
import numpy as np

from .executor import AvgPair, GroupByResult  # noqa: F401  (GroupByResult re-exported)
from .query import QueryContext, parse_query

DELIMITER = "\0"  # GroupKeyGenerator.DELIMITER


class GroupKey:
    """GroupKeyGenerator.GroupKey: _groupId and the group-by values _keys."""
    __slots__ = ("_groupId", "_keys")

    def __init__(self, group_id, keys):
        self._groupId = group_id
        self._keys = keys

    def __repr__(self):
        return "GroupKey(%d, %r)" % (self._groupId, self._keys)


class StringGroupKey:
    """GroupKeyGenerator.StringGroupKey: _groupId and the values joined by DELIMITER (getKeys splits them)."""
    __slots__ = ("_groupId", "_stringKey")

    def __init__(self, group_id, string_key):
        self._groupId = group_id
        self._stringKey = string_key

    def getKeys(self):
        return self._stringKey.split(DELIMITER)

    def __repr__(self):
        return "StringGroupKey(%d, %r)" % (self._groupId, self._stringKey)


def _key_str(x):
    """String form of a group-by value as DataTable / Object.toString renders it (doubles as Java does: 1.0)."""
    if isinstance(x, float):
        return repr(x) if x == x and x not in (float("inf"), float("-inf")) else \
            ("NaN" if x != x else ("Infinity" if x > 0 else "-Infinity"))
    return str(x)


class GpuGroupKeyGenerator:
    """GroupKeyGenerator over a GPU result: the per-column table-global dictIds (zero-copy views) decoded through
    the dictionary snapshot the result indexes."""

    def __init__(self, result, key_cards=None):
        self._r = result
        self._key_cards = key_cards

    def getNumKeys(self):
        return len(self._r)

    def getGlobalGroupKeyUpperBound(self):
        """Product of the group-by cardinalities (the ARRAY holder's key space), or the number of groups when the
        cardinalities are not known."""
        if not self._key_cards:
            return len(self._r)
        ub = 1
        for c in self._key_cards:
            ub *= max(int(c), 1)
        return ub

    def getCurrentGroupKeyUpperBound(self):
        return len(self._r)

    def getGroupKeys(self):
        for gid, key in enumerate(self._r.keys):
            yield GroupKey(gid, list(key))

    def getStringGroupKeys(self):
        for gid, key in enumerate(self._r.keys):
            yield StringGroupKey(gid, DELIMITER.join(_key_str(x) for x in key))


class GpuGroupByResultHolder:
    """Result holder of one aggregation function over the result's groups: DoubleGroupByResultHolder for COUNT / SUM /
    MIN / MAX (getDoubleResult), ObjectGroupByResultHolder of AvgPair for AVG (getResult)."""

    def __init__(self, function, values, counts=None):
        self.function = function
        self._values = values          # np.float64 [n] (COUNT / SUM / MIN / MAX; AVG: AvgPair.sum)
        self._counts = counts          # np.int64 [n] (AVG: AvgPair.count)

    def getDoubleResult(self, group_key):
        if self.function == "AVG":
            raise TypeError("AVG keeps AvgPair objects: getResult")
        return float(self._values[group_key])

    def getResult(self, group_key):
        if self.function == "AVG":
            return AvgPair(float(self._values[group_key]), int(self._counts[group_key]))
        return float(self._values[group_key])


def _holders(result, aggregations):
    """One holder per aggregation, over the result's columnar arrays."""
    out = []
    if result._col is not None:
        for (fn, _), (_, v, e, c) in zip(aggregations, result._col[2]):
            vals = v if v is not None else e.astype(np.float64)
            out.append(GpuGroupByResultHolder(fn, vals, c))
        return out
    values = result.values  # Python form (results built from key / value lists)
    for a, (fn, _) in enumerate(aggregations):
        col = [row[a] for row in values]
        if fn == "AVG":
            out.append(GpuGroupByResultHolder(fn, np.array([p.sum for p in col], dtype=np.float64),
                                              np.array([p.count for p in col], dtype=np.int64)))
        else:
            out.append(GpuGroupByResultHolder(fn, np.array(col, dtype=np.float64)))
    return out


class AggregationGroupByResult:
    """core/query/aggregation/groupby/AggregationGroupByResult.java:31-81."""

    def __init__(self, key_generator, aggregation_functions, result_holders):
        self._gen = key_generator
        self._functions = aggregation_functions
        self._holders = result_holders

    def getGroupKeyIterator(self):
        return self._gen.getGroupKeys()

    def getStringGroupKeyIterator(self):
        return self._gen.getStringGroupKeys()

    def getResultForKey(self, group_key, index):
        return self.getResultForGroupId(index, group_key._groupId)

    def getResultForGroupId(self, index, group_id):
        """AggregationFunction.extractGroupByResult: COUNT as a long, SUM / MIN / MAX as doubles, AVG an AvgPair."""
        fn = self._functions[index][0]
        h = self._holders[index]
        if fn == "COUNT":
            return int(h.getDoubleResult(group_id))
        return h.getResult(group_id)


class IntermediateResultsBlock:
    """core/operator/blocks/IntermediateResultsBlock.java:106-133 (group-by form)."""

    def __init__(self, aggregation_functions, result, key_cards=None):
        self.aggregation_functions = aggregation_functions
        self._result = result
        self._agb = AggregationGroupByResult(GpuGroupKeyGenerator(result, key_cards), aggregation_functions,
                                             _holders(result, aggregation_functions))

    def getAggregationGroupByResult(self):
        return self._agb

    def get_aggregation_group_by_result(self):
        """{stringKey: [results]} -- the StringGroupKey form of every group."""
        return self._result.string_keys()

    def get_group_by_result(self):
        return self._result

    def getNumGroupsLimitReached(self):
        return bool(getattr(self._result, "num_groups_limit_reached", False))


class AggregationResultsBlock:
    """IntermediateResultsBlock in its aggregation-only form (IntermediateResultsBlock.java:78-86)."""

    def __init__(self, aggregation_functions, result):
        self.aggregation_functions = aggregation_functions
        self._result = result

    def get_aggregation_result(self):
        return self._result.values

    def getAggregationResult(self):
        return list(self._result.values)


class _GpuOperatorBase:
    OPERATOR_NAME = None
    EXPLAIN_NAME = None

    def __init__(self, table, segment_handles, query):
        self.table = table
        self.segments = list(segment_handles)
        self.query = parse_query(query) if isinstance(query, str) else query
        assert isinstance(self.query, QueryContext)
        self._stats = None

    def _key_cards(self):
        return [len(self.table.dictionary(c)) for c in self.query.group_by]

    def nextBlock(self):
        result = self.table.execute_groupby(self.segments, self.query)
        self._stats = result.stats
        return IntermediateResultsBlock(self.query.aggregations, result, self._key_cards())

    next_block = nextBlock

    def getExecutionStatistics(self):
        return self._stats

    get_execution_statistics = getExecutionStatistics

    def getOperatorName(self):
        return self.OPERATOR_NAME

    def getChildOperators(self):
        """The fused GPU pass has no child operator chain (filter, projection and key generation run inside it)."""
        return []

    def toExplainString(self):
        """The reference's explain format: name(groupKeys:..., aggregations:...)."""
        aggs = ", ".join("%s(%s)" % (fn.lower(), c) for fn, c in self.query.aggregations)
        if self.query.group_by:
            return "%s(groupKeys:%s, aggregations:%s)" % (self.EXPLAIN_NAME, ", ".join(self.query.group_by), aggs)
        return "%s(aggregations:%s)" % (self.EXPLAIN_NAME, aggs)


class GpuAggregationGroupByOperator(_GpuOperatorBase):
    OPERATOR_NAME = "AggregationGroupByOperator"
    EXPLAIN_NAME = "AGGREGATE_GROUPBY"

    def __init__(self, table, segment_handle, query):
        super().__init__(table, [segment_handle], query)


class GpuGroupByCombineOperator(_GpuOperatorBase):
    OPERATOR_NAME = "GroupByCombineOperator"
    EXPLAIN_NAME = "COMBINE_GROUPBY"


class _GpuAggregationBase(_GpuOperatorBase):
    def nextBlock(self):
        result = self.table.execute_aggregation(self.segments, self.query)
        self._stats = result.stats
        return AggregationResultsBlock(self.query.aggregations, result)

    next_block = nextBlock


class GpuAggregationOperator(_GpuAggregationBase):
    OPERATOR_NAME = "AggregationOperator"
    EXPLAIN_NAME = "AGGREGATE"

    def __init__(self, table, segment_handle, query):
        super().__init__(table, [segment_handle], query)


class GpuAggregationOnlyCombineOperator(_GpuAggregationBase):
    OPERATOR_NAME = "AggregationOnlyCombineOperator"
    EXPLAIN_NAME = "COMBINE_AGGREGATE"
