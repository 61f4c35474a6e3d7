"""Operator-level mirror of the reference interface on this path, so a caller (and the tests) use the same
names and result shapes as Pinot's own operators:

  GpuAggregationGroupByOperator   AggregationGroupByOperator (core/operator/query/AggregationGroupByOperator.java:
                                  62-120): one segment -> IntermediateResultsBlock with an AggregationGroupByResult
                                  (group keys + per-function results) and ExecutionStatistics.
  GpuGroupByCombineOperator       GroupByCombineOperator (core/operator/combine/GroupByCombineOperator.java:75-223):
                                  all segments of a server in one GPU pass, merged in the table-global key space.
  GpuAggregationOperator          AggregationOperator (core/operator/query/AggregationOperator.java:58-95):
                                  aggregation-only queries (no GROUP BY), one result per function.
  GpuAggregationOnlyCombineOperator  AggregationOnlyCombineOperator: the same over all segments in one pass.
Errors follow the reference: a bad literal raises BadQueryRequestException; a shape outside the GPU path raises
UnsupportedQueryError (the Java shim keeps Pinot's CPU operator for it).
"""
from .executor import GroupByResult  # noqa: F401  (re-export)
from .query import QueryContext, parse_query


class IntermediateResultsBlock:
    """core/operator/blocks/IntermediateResultsBlock.java:106-133 (group-by form)."""

    def __init__(self, aggregation_functions, result):
        self.aggregation_functions = aggregation_functions
        self._result = result

    def get_aggregation_group_by_result(self):
        return self._result.string_keys()

    def get_group_by_result(self):
        return self._result


class AggregationResultsBlock:
    """IntermediateResultsBlock in its aggregation-only form (IntermediateResultsBlock.java:78-86)."""

    def __init__(self, aggregation_functions, result):
        self.aggregation_functions = aggregation_functions
        self._result = result

    def get_aggregation_result(self):
        return self._result.values


class _GpuOperatorBase:
    def __init__(self, table, segment_handles, query):
        self.table = table
        self.segments = list(segment_handles)
        self.query = parse_query(query) if isinstance(query, str) else query
        assert isinstance(self.query, QueryContext)
        self._stats = None

    def next_block(self):
        result = self.table.execute_groupby(self.segments, self.query)
        self._stats = result.stats
        return IntermediateResultsBlock(self.query.aggregations, result)

    def get_execution_statistics(self):
        return self._stats


class GpuAggregationGroupByOperator(_GpuOperatorBase):
    OPERATOR_NAME = "AggregationGroupByOperator"

    def __init__(self, table, segment_handle, query):
        super().__init__(table, [segment_handle], query)


class GpuGroupByCombineOperator(_GpuOperatorBase):
    OPERATOR_NAME = "GroupByCombineOperator"


class _GpuAggregationBase(_GpuOperatorBase):
    def next_block(self):
        result = self.table.execute_aggregation(self.segments, self.query)
        self._stats = result.stats
        return AggregationResultsBlock(self.query.aggregations, result)


class GpuAggregationOperator(_GpuAggregationBase):
    OPERATOR_NAME = "AggregationOperator"

    def __init__(self, table, segment_handle, query):
        super().__init__(table, [segment_handle], query)


class GpuAggregationOnlyCombineOperator(_GpuAggregationBase):
    OPERATOR_NAME = "AggregationOnlyCombineOperator"
