"""numEntriesScannedInFilter: the host replay of Pinot's docId iterators (pgpu_filter_entries_scanned,
filter_stats.cpp) against the oracle's per-document iterators, on random filters over segments with sorted columns
(SortedIndexBasedFilterOperator), inverted indexes (BitmapBasedFilterOperator) and scans; CPU only.  The device
plans use the same module for the shapes they do not count in the scan kernel."""
import ctypes

import numpy as np
import pytest

import kat_common as K
from pinot_amd import _lib as L
from pinot_amd.query import FilterContext, Predicate, QueryContext


def _leaf_sets(oracle, schema, seg, q):
    """Per predicate: (Pinot leaf type in this segment, match bitmap as u32 words)."""
    preds, ops = [], []
    q.filter.postfix(preds, ops)
    cols = dict(seg.columns)
    out = []
    for p in preds:
        one = QueryContext([], [("COUNT", "*")], FilterContext.pred(p))
        bm = oracle.filter_bitmap(schema, seg, one).view(np.uint32).copy()
        n = seg.num_docs
        bits = np.unpackbits(bm.view(np.uint8), bitorder="little")[:n]
        c = cols[p.column]
        if not bits.any():
            t = L.LEAF_EMPTY
        elif bits.all():
            t = L.LEAF_MATCH_ALL
        elif c.is_sorted:
            t = L.LEAF_SORTED
        elif p.type != "RANGE" and getattr(c, "inv_bytes", None) is not None:
            t = L.LEAF_BITMAP
        else:
            t = L.LEAF_SCAN
        out.append((t, bm))
    return preds, ops, out


def host_entries(oracle, schema, seg, q):
    lib = L.load()
    preds, ops, leaves = _leaf_sets(oracle, schema, seg, q)
    fo = (L.FilterOpC * max(len(ops), 1))(*[L.FilterOpC(o, a) for o, a in ops])
    types = (ctypes.c_int32 * max(len(leaves), 1))(*[t for t, _ in leaves])
    masks = (ctypes.c_void_p * max(len(leaves), 1))(*[m.ctypes.data for _, m in leaves])
    out = ctypes.c_int64()
    L.check(lib.pgpu_filter_entries_scanned(fo, len(ops), types, masks, len(leaves), seg.num_docs, ctypes.byref(out)))
    return out.value


def test_kat_filter_entries(oracle):
    """84134 entries for the reference's filter on its segment (InnerSegmentAggregationSingleValueQueriesTest.java:69):
    the sorted daysSinceEpoch leaf, column1 / column3 applyAnd scans, then the leap-frog with the OR of the
    column6 / column11 scans."""
    seg = K.kat_segment(oracle)
    q = K.inner_query(["column9"], True)
    assert host_entries(oracle, K.SCHEMA, seg, q) == 84134


SCHEMA = [("s", "INT"), ("a", "INT"), ("b", "INT"), ("c", "INT"), ("d", "INT")]


def _segment(oracle, rng, n):
    from dataclasses import replace
    from pinot_amd.segment import SegmentBuffers
    seg = oracle.make_segment(SCHEMA, {"s": np.sort(rng.integers(0, 12, n)), "a": rng.integers(0, 6, n),
                                       "b": rng.integers(0, 40, n), "c": rng.integers(0, 4, n),
                                       "d": rng.integers(0, 300, n)})
    cols = dict(seg.columns)
    cols["s"] = replace(cols["s"], is_sorted=True)
    if rng.random() < 0.7:
        cols["a"] = replace(cols["a"], inv_bytes=b"x")  # only the presence matters to the model
    if rng.random() < 0.5:
        cols["b"] = replace(cols["b"], inv_bytes=b"x")
    return SegmentBuffers(n, cols)


def _pred(rng):
    col = ["s", "a", "b", "c", "d"][int(rng.integers(0, 5))]
    top = {"s": 12, "a": 6, "b": 40, "c": 4, "d": 300}[col]
    v = [str(int(x)) for x in rng.integers(0, top, 3)]
    k = int(rng.integers(0, 5))
    if k == 0:
        return Predicate.eq(col, v[0])
    if k == 1:
        return Predicate.not_eq(col, v[0])
    if k == 2:
        return Predicate.in_(col, v)
    if k == 3:
        return Predicate.not_in(col, v[:2])
    lo, hi = sorted(int(x) for x in v[:2])
    return Predicate.range(col, str(lo), str(hi), bool(rng.random() < 0.5), bool(rng.random() < 0.5))


def _filter(rng, depth=0):
    if depth < 2 and rng.random() < 0.6:
        kids = [_filter(rng, depth + 1) for _ in range(int(rng.integers(2, 5)))]
        f = FilterContext.and_(*kids) if rng.random() < 0.55 else FilterContext.or_(*kids)
        return FilterContext.not_(f) if rng.random() < 0.1 else f
    return FilterContext.pred(_pred(rng))


@pytest.mark.parametrize("seed", range(8))
def test_random_filters_match_oracle(oracle, seed):
    rng = np.random.default_rng(500 + seed)
    for _ in range(25):
        seg = _segment(oracle, rng, int(rng.integers(1, 3000)))
        q = QueryContext(["c"], [("COUNT", "*")], _filter(rng))
        o = oracle.run_groupby(SCHEMA, [seg], q, combine=False)
        assert host_entries(oracle, SCHEMA, seg, q) == o.stats[1], q.filter
