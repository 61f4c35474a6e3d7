"""Range-index leaves on the GPU: a RANGE predicate on an unsorted, dictionary-encoded column
with a range index runs as Pinot's RangeIndexBasedFilterOperator (FilterOperatorUtils.java:57-62; the operator at
core/operator/filter/RangeIndexBasedFilterOperator.java:57-129) -- an index-based leaf ordered after the bitmap leaves
in an AND, whose numEntriesScannedInFilter is its partial-match scan (version 1, RangeIndexReaderImpl) or nothing
(version 2, BitSlicedRangeIndexReader).  Groups, values and the four statistics against the oracle, including
segments with and without the index in one plan, an inverted-index leaf beside it, OR / NOT shapes and EQ on the
range-indexed column (which ignores the index)."""
from dataclasses import replace

import numpy as np
import pytest

from pinot_amd.executor import GpuTable
from pinot_amd.query import parse_query
from pinot_amd.segment import SegmentBuffers
from pinot_amd.segment_files import build_inverted_index, build_range_index, build_range_index_bitsliced_header
from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu

SCHEMA = [("a", "INT"), ("b", "INT"), ("g", "INT"), ("v", "INT"), ("s", "INT")]
QUERIES = [
    "SELECT COUNT(*), SUM(v) FROM t WHERE a BETWEEN 100 AND 260 GROUP BY g",
    "SELECT COUNT(*), MAX(v) FROM t WHERE a > 420 AND v < 300 GROUP BY g",
    "SELECT COUNT(*) FROM t WHERE v < 800 AND a <= 40 GROUP BY g",  # scan first in the query, range leaf first in Pinot
    "SELECT COUNT(*), SUM(v) FROM t WHERE a < 30 OR b >= 55 GROUP BY g",
    "SELECT COUNT(*) FROM t WHERE b BETWEEN 10 AND 12 AND a BETWEEN 5 AND 300 AND v > 100 GROUP BY g",
    "SELECT COUNT(*) FROM t WHERE b = 17 AND a BETWEEN 5 AND 300 GROUP BY g",  # inverted EQ leaf + range leaf
    "SELECT COUNT(*) FROM t WHERE NOT a BETWEEN 100 AND 400 GROUP BY g",
    "SELECT COUNT(*) FROM t WHERE a = 7 GROUP BY g",  # EQ: no range index use
    "SELECT COUNT(*) FROM t WHERE s BETWEEN 2 AND 5 AND a < 250 GROUP BY g",  # sorted column: sorted leaf
    "SELECT SUM(v) FROM t WHERE a BETWEEN 0 AND 499",  # aggregation-only, a range covering the dictionary
]


def _dict_ids(values):
    return np.unique(np.asarray(values), return_inverse=True)[1]


def _segments(oracle, version):
    out = []
    for k, n in enumerate([150001, 65536, 1, 70000]):
        rng = np.random.default_rng(300 + k)
        cols = {"a": rng.integers(0, 500, n), "b": rng.integers(0, 60, n), "g": rng.integers(0, 8, n),
                "v": rng.integers(0, 1000, n), "s": np.sort(rng.integers(0, 10, n))}
        _SORTED_VALUES[n] = cols["s"]
        seg = oracle.make_segment(SCHEMA, cols)
        c = dict(seg.columns)
        for name in ("a", "b"):
            rb = build_range_index(_dict_ids(cols[name]), c[name].cardinality) if version == 1 else \
                build_range_index_bitsliced_header()
            c[name] = replace(c[name], range_bytes=rb)
        c["b"] = replace(c["b"], inv_bytes=build_inverted_index(_dict_ids(cols["b"]), c["b"].cardinality))
        c["s"] = replace(c["s"], is_sorted=True, range_bytes=build_range_index(_dict_ids(cols["s"]), c["s"].cardinality))
        out.append(SegmentBuffers(n, c))
    return out


def _gpu_form(seg):
    """The pinned form: the sorted column as SortedIndexReaderImpl (start, end) pairs (the oracle reads its fixed-bit
    view with the sorted flag)."""
    from pinot_amd import _lib as L
    from pinot_amd.segment_files import _sorted_pairs
    c = dict(seg.columns)
    s = c["s"]
    vals = np.frombuffer(s.dict_bytes, dtype=">i4")
    ids = np.searchsorted(vals, _SORTED_VALUES[seg.num_docs])
    c["s"] = replace(s, fwd_bytes=_sorted_pairs(ids, s.cardinality), fwd_format=L.FWD_SORTED_PAIRS)
    return SegmentBuffers(seg.num_docs, c)


_SORTED_VALUES = {}


def _without_range(seg):
    return SegmentBuffers(seg.num_docs, {k: replace(v, range_bytes=None) for k, v in seg.columns.items()})


@pytest.mark.parametrize("version", [1, 2])
def test_range_index_leaves_match_oracle(oracle, gpu_lib, version):
    segs = _segments(oracle, version)
    mixed = [s if k != 1 else _without_range(s) for k, s in enumerate(segs)]  # segment 1 lacks the range indexes
    t, tm = GpuTable(SCHEMA), GpuTable(SCHEMA)
    try:
        hs = [t.pin_segment(_gpu_form(s)) for s in segs]
        hm = [tm.pin_segment(_gpu_form(s)) for s in mixed]
        for sql in QUERIES:
            q = parse_query(sql)
            r, o = t.execute_groupby(hs, q), oracle.run_groupby(SCHEMA, segs, q)
            assert_same(r, o, q, SCHEMA)
            assert r.stats.as_tuple() == o.stats, (sql, r.stats, o.stats)
            rm, om = tm.execute_groupby(hm, q), oracle.run_groupby(SCHEMA, mixed, q)
            assert_same(rm, om, q, SCHEMA)
            assert rm.stats.as_tuple() == om.stats, (sql, rm.stats, om.stats)
        # detaching the index returns the scan statistics
        for h in hs:
            t.attach_range_index(h, "a", b"")
            t.attach_range_index(h, "b", b"")
        q = parse_query(QUERIES[1])
        plain = [_without_range(s) for s in segs]
        assert t.execute_groupby(hs, q).stats.as_tuple() == oracle.run_groupby(SCHEMA, plain, q).stats
    finally:
        t.close()
        tm.close()


def test_range_index_rejected_on_bad_file(oracle, gpu_lib):
    from pinot_amd import _lib as L
    seg = oracle.make_segment(SCHEMA, {"a": np.arange(100) % 7, "b": np.arange(100) % 3, "g": np.zeros(100, int),
                                       "v": np.arange(100), "s": np.arange(100)})
    t = GpuTable(SCHEMA)
    try:
        h = t.pin_segment(seg)
        good = build_range_index(_dict_ids(np.arange(100) % 7), 7)
        with pytest.raises(L.PinotGpuError) as e:
            t.attach_range_index(h, "a", good[:-3])
        assert e.value.code == L.PGPU_ERR_INVALID_ARGUMENT
        t.attach_range_index(h, "a", good)
        r = t.execute_groupby([h], parse_query("SELECT COUNT(*) FROM t WHERE a BETWEEN 2 AND 4 GROUP BY g"))
        assert r.as_dict() == {(0,): [int(((np.arange(100) % 7 >= 2) & (np.arange(100) % 7 <= 4)).sum())]}
    finally:
        t.close()
