"""Range indexes on the host (no GPU): the library's reader of `<column>.bitmap.range` files (pgpu_range_index_check,
pgpu_range_index_partial_entries: RangeIndexReaderImpl / BitSlicedRangeIndexReader) against a direct numpy restatement
of RangeIndexCreator's ranges, and the oracle's RangeIndexBasedFilterOperator statistics (FilterOperatorUtils.java:57-62,
RangeIndexBasedFilterOperator.java:57-129) on queries over range-indexed columns.  No serialised range index ships
with the reference, so the file format is pinned by its writer and reader sources only (parity unpinned for the
bytes); the statistics are pinned by the oracle's restatement of the reader and operator."""
import ctypes
from dataclasses import replace

import numpy as np
import pytest

from pinot_amd import _lib as L
from pinot_amd.query import parse_query
from pinot_amd.segment import SegmentBuffers
from pinot_amd.segment_files import build_range_index, build_range_index_bitsliced_header


def _dict_ids(values):
    return np.unique(np.asarray(values), return_inverse=True)[1]


def _ranges(ids):
    """RangeIndexCreator.seal's ranges over the sorted dictIds: (first dictId, last dictId, docs)."""
    vals = np.sort(ids)
    n = vals.size
    per = (n + 19) // 20
    out, start = [], 0
    for i in range(n):
        if i > start + per and vals[i] != vals[i - 1]:
            out.append((vals[start], vals[i - 1], i - start))
            start = i
    out.append((vals[start], vals[n - 1], n - start))
    return out


def _partial(ranges, lo, hi):
    """RangeIndexReaderImpl.getPartiallyMatchingDocIds size for dictIds [lo, hi] (findRangeId over the starts)."""
    starts = [r[0] for r in ranges]

    def rid(v):
        for i, s in enumerate(starts):
            if v < s:
                return i - 1
        return len(starts) - 1 if v <= ranges[-1][1] else len(starts)
    f, t = rid(lo), rid(hi)
    out = lambda i: i < 0 or i >= len(ranges)  # noqa: E731
    if out(f):
        return 0 if out(t) else ranges[t][2]
    if out(t):
        return ranges[f][2]
    return ranges[f][2] if f == t else ranges[f][2] + ranges[t][2]


def _check(b, card, docs):
    lib = L.load()
    v, nr, tot = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
    rc = lib.pgpu_range_index_check(b, len(b), card, docs, ctypes.byref(v), ctypes.byref(nr), ctypes.byref(tot))
    return rc, v.value, nr.value, tot.value


def _partial_lib(b, card, docs, lo, hi):
    e = ctypes.c_int64()
    L.check(L.load().pgpu_range_index_partial_entries(b, len(b), card, docs, lo, hi, ctypes.byref(e)))
    return e.value


@pytest.mark.parametrize("card,docs,skew", [(50, 1000, False), (3000, 150001, False), (7, 70000, True),
                                            (1, 10, False), (200, 1, False)])
def test_reader_matches_creator_ranges(card, docs, skew):
    rng = np.random.default_rng(card + docs)
    ids = (rng.zipf(1.5, docs) % card) if skew else rng.integers(0, card, docs)
    ids = np.asarray(ids, dtype=np.int64)
    b = build_range_index(ids, card)
    rc, v, nr, tot = _check(b, card, docs)
    ranges = _ranges(ids)
    assert (rc, v, nr, tot) == (0, 1, len(ranges), docs)
    for lo, hi in [(0, card - 1), (0, 0), (card - 1, card - 1)] + \
            [tuple(sorted(rng.integers(0, card, 2))) for _ in range(40)]:
        assert _partial_lib(b, card, docs, int(lo), int(hi)) == _partial(ranges, lo, hi), (lo, hi)


def test_reader_versions_and_malformed_files():
    ids = np.random.default_rng(3).integers(0, 40, 5000)
    b = build_range_index(ids, 40)
    assert _check(build_range_index_bitsliced_header(), 40, 5000)[:3] == (0, 2, 0)
    assert _partial_lib(build_range_index_bitsliced_header(), 40, 5000, 3, 9) == 0  # exact: no partial scan
    assert _check(b"\x00\x00\x00\x07" + b"\x00" * 32, 40, 5000)[:2] == (0, 0)  # unknown version: skipped
    bad = [b[:-1], b[:20], b[:4] + b"\x00\x00\x00\x04LONG" + b[11:], bytearray(b)]
    bad[3][-40] ^= 0xFF  # a corrupted bitmap payload / header
    for x in bad[:3]:
        assert _check(bytes(x), 40, 5000)[0] == L.PGPU_ERR_INVALID_ARGUMENT
    assert _check(b, 40, 4999)[0] == L.PGPU_ERR_INVALID_ARGUMENT  # bitmaps cover other documents
    assert _check(b, 10, 5000)[0] == L.PGPU_ERR_INVALID_ARGUMENT  # range bounds past the dictionary


SCHEMA = [("a", "INT"), ("b", "INT"), ("g", "INT"), ("v", "INT")]


def _segments(oracle, version):
    segs = []
    for k, n in enumerate([40000, 70001]):
        rng = np.random.default_rng(90 + k)
        cols = {"a": rng.integers(0, 500, n), "b": rng.integers(0, 60, n), "g": rng.integers(0, 8, n),
                "v": rng.integers(0, 1000, n)}
        seg = oracle.make_segment(SCHEMA, cols)
        c = dict(seg.columns)
        for name in ("a", "b"):
            rb = build_range_index(_dict_ids(cols[name]), c[name].cardinality) if version == 1 else \
                build_range_index_bitsliced_header()
            c[name] = replace(c[name], range_bytes=rb)
        segs.append((SegmentBuffers(n, c), cols))
    return segs


@pytest.mark.parametrize("version", [1, 2])
def test_oracle_range_index_statistics(oracle, version):
    """RANGE leaves on range-indexed columns: same groups as without the index; numEntriesScannedInFilter is the
    partial-match scan (version 1) or nothing (version 2) for the leaf itself, an index-based AND child otherwise."""
    segs = _segments(oracle, version)
    plain = [SegmentBuffers(s.num_docs, {k: replace(v, range_bytes=None) for k, v in s.columns.items()})
             for s, _ in segs]
    idx = [s for s, _ in segs]
    for sql in ("SELECT COUNT(*), SUM(v) FROM t WHERE a BETWEEN 100 AND 260 GROUP BY g",
                "SELECT COUNT(*) FROM t WHERE a > 420 AND v < 300 GROUP BY g",
                "SELECT COUNT(*) FROM t WHERE a < 30 OR b >= 55 GROUP BY g",
                "SELECT COUNT(*) FROM t WHERE b BETWEEN 10 AND 12 AND a BETWEEN 5 AND 300 GROUP BY g",
                "SELECT COUNT(*) FROM t WHERE a = 7 GROUP BY g"):
        q = parse_query(sql)
        o, p = oracle.run_groupby(SCHEMA, idx, q), oracle.run_groupby(SCHEMA, plain, q)
        assert o.groups == p.groups, sql
        assert o.stats[0] == p.stats[0], sql
        if sql.endswith("a = 7 GROUP BY g"):  # EQ: the range index is not used
            assert o.stats == p.stats
    # the single-leaf case against the reader directly: entries = the partial ranges' docs of each segment
    q = parse_query("SELECT COUNT(*) FROM t WHERE a BETWEEN 100 AND 260 GROUP BY g")
    want = 0
    for s, cols in segs:
        ids = _dict_ids(cols["a"])
        vals = np.unique(cols["a"])
        lo, hi = int(np.searchsorted(vals, 100)), int(np.searchsorted(vals, 260, side="right")) - 1
        want += _partial(_ranges(ids), lo, hi) if version == 1 else 0
    assert oracle.run_groupby(SCHEMA, idx, q).stats[1] == want
    # AND with a scan: the scan's applyAnd runs over the range leaf's docs (an index-based child)
    q = parse_query("SELECT COUNT(*) FROM t WHERE a > 420 AND v < 300 GROUP BY g")
    want = 0
    for s, cols in segs:
        vals = np.unique(cols["a"])
        lo = int(np.searchsorted(vals, 420, side="right"))
        want += (_partial(_ranges(_dict_ids(cols["a"])), lo, len(vals) - 1) if version == 1 else 0) + \
            int((cols["a"] > 420).sum())
    assert oracle.run_groupby(SCHEMA, idx, q).stats[1] == want


def test_filter_entries_scanned_range_index_leaf():
    """pgpu_filter_entries_scanned with a PGPU_LEAF_RANGE_INDEX child: an index-based AND child ranked after the
    bitmap leaves (its own partial scan excluded), so the scan's applyAnd counts the range leaf's docs."""
    lib = L.load()
    n = 1000
    rng = np.random.default_rng(5)
    m0 = rng.random(n) < 0.3
    m1 = rng.random(n) < 0.5
    words = []
    for m in (m0, m1):
        by = np.packbits(m.astype(np.uint8), bitorder="little")
        words.append(np.ascontiguousarray(np.pad(by, (0, (-by.size) % 4)).view("<u4")))
    ops = (L.FilterOpC * 3)(L.FilterOpC(L.OP_PRED, 0), L.FilterOpC(L.OP_PRED, 1), L.FilterOpC(L.OP_AND, 2))
    types = np.array([L.LEAF_SCAN, L.LEAF_RANGE_INDEX], dtype=np.int32)
    masks = (ctypes.c_void_p * 2)(words[0].ctypes.data, words[1].ctypes.data)
    out = ctypes.c_int64()
    L.check(lib.pgpu_filter_entries_scanned(ops, 3, types.ctypes.data_as(L.c_i32p),
                                            ctypes.cast(masks, ctypes.POINTER(ctypes.c_void_p)), 2, n,
                                            ctypes.byref(out)))
    assert out.value == int(m1.sum())  # the scan (leaf 0) runs over the range leaf's docs
