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
