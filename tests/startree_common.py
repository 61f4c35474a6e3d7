"""Helpers of the star-tree tests: the C4 schema, star-tree oracle inputs derived from a query
(predicate composites -> matching dictIds per dimension, evaluated by the C oracle's own predicate evaluators over
an identity segment of the dimension's dictionary), and the expected answer in value space."""
import os
import sys

import numpy as np

from pinot_amd import _lib as L
from pinot_amd.executor import AvgPair
from pinot_amd.query import FilterContext, QueryContext

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import startree_oracle as SO  # noqa: E402

C4_SCHEMA = [("d1", "INT"), ("d2", "INT"), ("d3", "INT"), ("d4", "INT"), ("m", "INT"), ("md", "DOUBLE")]
C4_SPLIT = ["d1", "d2", "d3", "d4"]
C4_PAIRS = [("SUM", "m"), ("COUNT", "*"), ("MIN", "m"), ("MAX", "m"), ("AVG", "m"), ("SUM", "md")]
FN = {"COUNT": SO.COUNT, "SUM": SO.SUM, "MIN": SO.MIN, "MAX": SO.MAX, "AVG": SO.AVG}


def c4_columns(rng, n, cards=(100, 50, 20, 10)):
    cols = {}
    for name, card in zip(C4_SPLIT, cards):
        cols[name] = rng.integers(0, card, n).astype(np.int64)
    cols["m"] = rng.integers(0, 1000, n).astype(np.int64)
    cols["md"] = rng.uniform(-1e3, 1e3, n)
    return cols


def dictionary_values(col):
    w = col.entry_width
    raw = col.dict_bytes
    if col.data_type == L.INT:
        return np.frombuffer(raw, dtype=">i4").astype(np.int64)
    if col.data_type == L.LONG:
        return np.frombuffer(raw, dtype=">i8").astype(np.int64)
    if col.data_type == L.DOUBLE:
        return np.frombuffer(raw, dtype=">f8").astype(np.float64)
    return np.frombuffer(raw, dtype=">f4").astype(np.float64)


def composites(flt):
    """StarTreeUtils.extractPredicateEvaluatorsMap shape: AND of (predicate | OR of predicates on one column)."""
    if flt is None:
        return []
    if flt.type == FilterContext.PREDICATE:
        return [flt]
    if flt.type == FilterContext.OR:
        return [flt]
    assert flt.type == FilterContext.AND
    out = []
    for c in flt.children:
        out += composites(c)
    return out


def _column_of(f):
    if f.type == FilterContext.PREDICATE:
        return f.predicate.column
    cols = {_column_of(c) for c in f.children}
    assert len(cols) == 1
    return cols.pop()


def pred_match(oracle, seg, schema, flt, split):
    """{split-order dim: bool array over the segment dictIds} for the query's predicate composites (always-true
    composites dropped, as isAlwaysTrue evaluators are)."""
    types = dict(schema)
    out = {}
    for comp in composites(flt):
        col = _column_of(comp)
        c = seg.columns[col]
        ident = oracle.make_segment([(col, types[col])], {col: dictionary_values(c)})
        q = QueryContext([col], [("COUNT", "*")], comp)
        bm = oracle.filter_bitmap([(col, types[col])], ident, q)
        m = np.unpackbits(bm.view(np.uint8), bitorder="little")[:c.cardinality].astype(bool)
        if m.all():
            continue
        d = split.index(col)
        out[d] = out[d] & m if d in out else m
    return out


def startree_answer(oracle, seg, schema, star, q, split, pairs):
    """The star-tree oracle's answer in value space: {value tuple: [values]} plus (docs, entries in filter)."""
    pm = pred_match(oracle, seg, schema, q.filter, split)
    gdims = [split.index(c) for c in q.group_by]
    dim_bits = [seg.columns[c].bits_per_element for c in split]
    aggs = []
    for fn, col in q.aggregations:
        m = next(i for i, (f, c) in enumerate(pairs) if f == fn and (fn == "COUNT" or c == col))
        aggs.append((FN[fn], m))
    res, docs, scanned = SO.groupby(star, dim_bits, pm, gdims, aggs)
    dicts = {c: dictionary_values(seg.columns[c]) for c in q.group_by}
    out = {}
    for key, vals in res.items():
        vkey = tuple(int(dicts[c][k]) for c, k in zip(q.group_by, key))
        out[vkey] = [AvgPair(*v) if isinstance(v, tuple) else v for v in vals]
    return out, docs, scanned


C4_QUERIES = [
    "SELECT SUM(m), COUNT(*) FROM t WHERE d3 IN (1, 5, 7) GROUP BY d1, d2",
    "SELECT SUM(m), COUNT(*), MIN(m), MAX(m) FROM t GROUP BY d4",
    "SELECT COUNT(*), AVG(m) FROM t WHERE d1 BETWEEN 10 AND 40 AND d4 <> 3 GROUP BY d2",
    "SELECT SUM(m), SUM(md) FROM t WHERE d2 = 7 OR d2 = 9 GROUP BY d3",
    "SELECT COUNT(*) FROM t WHERE d1 NOT IN (1, 2, 3) AND d3 < 5 GROUP BY d4, d1",
    "SELECT MAX(m), MIN(m) FROM t WHERE d4 >= 8 GROUP BY d1",
]
