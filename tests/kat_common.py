"""Shared loaders for the reference known-answer tests (tests/golden/kat_sv.json) — used by both the oracle
(CPU) and the GPU parity tests."""
import json
import os

import numpy as np

from pinot_amd.query import QueryContext

HERE = os.path.dirname(os.path.abspath(__file__))
KAT = json.load(open(os.path.join(HERE, "golden", "kat_sv.json")))
SCHEMA = [(k, v) for k, v in KAT["schema"].items()]
TYPES = dict(SCHEMA)


def sv_columns():
    z = np.load(os.path.join(HERE, "golden", "sv_columns.npz"))
    cols = {}
    for name, t in SCHEMA:
        if t == "STRING":
            blob = z[name + "__blob"].tobytes()
            off = z[name + "__off"]
            cols[name] = [blob[off[i]:off[i + 1]].decode() for i in range(len(off) - 1)]
        else:
            cols[name] = z[name].astype(np.int64)
    return cols


def kat_segment(oracle, pairs=False):
    """The KAT segment as the reference's tests load it: column5 and daysSinceEpoch are sorted
    (SegmentColumnarIndexCreator detects sortedness; their predicates run as SortedIndexBasedFilterOperator), and no
    inverted index is loaded -- BaseSingleValueQueriesTest.java:139 loads with ImmutableSegmentLoader.load(dir,
    ReadMode.heap), a default IndexLoadingConfig without inverted-index columns, and PhysicalColumnIndexContainer
    loads an inverted index only for those columns (PhysicalColumnIndexContainer.java:79).  pairs=True stores the
    sorted columns in SortedIndexReaderImpl form (start, end docId per dictId) as the pinned segment holds them."""
    from dataclasses import replace
    from pinot_amd import _lib as L
    from pinot_amd.segment import SegmentBuffers
    seg = oracle.make_segment(SCHEMA, sv_columns())
    cols = dict(seg.columns)
    for name in KAT["sorted_columns"]:
        c = cols[name]
        if not pairs:
            cols[name] = replace(c, is_sorted=True)
            continue
        ids = np.zeros(seg.num_docs + 32, dtype=np.int32)
        import ctypes
        buf = ctypes.create_string_buffer(bytes(c.fwd_bytes) + b"\0" * 16, len(c.fwd_bytes) + 16)
        oracle.lib().or_bitset_read_ints(buf, ctypes.c_int64(0), c.bits_per_element, seg.num_docs, ids.ctypes.data)
        ids = ids[:seg.num_docs]
        assert np.all(np.diff(ids) >= 0), name
        pairs_b = b"".join(int(np.nonzero(ids == i)[0][0]).to_bytes(4, "big") +
                           int(np.nonzero(ids == i)[0][-1]).to_bytes(4, "big") for i in range(c.cardinality))
        cols[name] = replace(c, fwd_bytes=pairs_b, fwd_format=L.FWD_SORTED_PAIRS, is_sorted=True)
    return SegmentBuffers(seg.num_docs, cols)


def key_tuple(group_by, key_strings):
    return tuple(int(v) if TYPES[c] != "STRING" else v for c, v in zip(group_by, key_strings))


def inner_query(group_by, with_filter):
    flt = QueryContext.filter_from_json(KAT["query_filter"]) if with_filter else None
    return QueryContext(group_by, [tuple(a) for a in KAT["inner_segment_aggs"]], flt)


def check_inner_values(vals, expected):
    """QueriesTestUtils.testInnerSegmentAggregationGroupByResult (:77-99): count, sum, max, min as long/int;
    AvgPair sum as long, count."""
    count, s, mx, mn, avg = vals
    assert int(count) == expected[0]
    assert int(s) == expected[1]
    assert int(mx) == expected[2]
    assert int(mn) == expected[3]
    assert int(avg.sum) == expected[4]
    assert avg.count == expected[5]


# InterSegmentAggregationSingleValueQueriesTest KATs (tests/golden/kat_inter_agg.json): SUM/COUNT/MIN/MAX/AVG over
# 4 copies of the segment, aggregation-only and GROUP BY column9 (PQL: the top group per function).
KAT_AGG = json.load(open(os.path.join(HERE, "golden", "kat_inter_agg.json")))


def agg_case_query(case):
    from pinot_amd.query import parse_query
    q = parse_query(case["query"])
    if case["filter"]:
        q.filter = QueryContext.filter_from_json(KAT["query_filter"])
    if case["group_by"]:
        q.group_by = [KAT_AGG["group_by_column"]]
    return q


def pql_value(fn, v):
    """Broker formatting of an aggregation result (PQL): COUNT as a long, everything else '%.5f'; AVG is final."""
    if fn == "AVG":
        v = v.final() if hasattr(v, "final") else v
    return str(int(v)) if fn == "COUNT" else "%.5f" % float(v)


def top_group_values(q, groups):
    """AggregationGroupByTrimmingService order per function: MIN ascending, the others descending; the broker's
    first row per function."""
    out = []
    for a, (fn, _) in enumerate(q.aggregations):
        vals = [(g[a].final() if fn == "AVG" else g[a]) for g in groups]
        out.append(min(vals) if fn == "MIN" else max(vals))
    return out


def check_agg_case(case, q, stats, values):
    docs, in_filter, post, total = case["stats"]
    assert (stats[0], stats[1], stats[2], stats[3]) == (docs, in_filter, post, total), \
        (case["test"], case["variant"], stats)
    got = [pql_value(fn, v) for (fn, _), v in zip(q.aggregations, values)]
    assert got == case["values"], (case["test"], case["variant"], got)
