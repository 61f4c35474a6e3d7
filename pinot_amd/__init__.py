"""pinot_amd — MI355X-native executor for Apache Pinot's server-side filter -> group-by -> aggregation path.

The compute path is libpinotgpu.so (HIP kernels for gfx950 behind the C ABI in include/pinotgpu.h); this
package is the host layer over it: query model, pinned tables, plans, results, and the Pinot-named operator
mirror used by the tests and bench.py.
"""
from .build import LIB_PATH  # noqa: F401
from .query import FilterContext, Predicate, QueryContext, parse_query  # noqa: F401
from .segment import ColumnData, SegmentBuffers, load_v1_segment_dir  # noqa: F401


def __getattr__(name):
    # Lazily import the pieces that load the shared library.
    if name in ("GpuTable", "Plan", "GroupByResult", "ExecutionStatistics", "AvgPair"):
        from . import executor
        return getattr(executor, name)
    if name in ("GpuAggregationGroupByOperator", "GpuGroupByCombineOperator", "IntermediateResultsBlock"):
        from . import operators
        return getattr(operators, name)
    raise AttributeError(name)
