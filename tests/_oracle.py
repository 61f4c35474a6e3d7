"""ctypes bridge to oracle/liboracle.so — the CPU restatement of the reference path (test infrastructure only).

Builds segments in Pinot's byte format (dictionary + fixed-bit forward index) from raw column values, and runs
queries through the restated per-segment operator + combine.  Results come back keyed by python value tuples.
"""
import ctypes
import os
import subprocess

import numpy as np

from pinot_amd import _lib as L
from pinot_amd.executor import AvgPair
from pinot_amd.segment import ColumnData, SegmentBuffers

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "liboracle.so")


def build_oracle():
    src = [os.path.join(ORACLE_DIR, f) for f in ("oracle.c", "oracle.h", "Makefile")]
    if not os.path.exists(ORACLE_LIB) or any(os.path.getmtime(s) > os.path.getmtime(ORACLE_LIB) for s in src):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    return ORACLE_LIB


class OrColumn(ctypes.Structure):
    _fields_ = [("data_type", ctypes.c_int32), ("cardinality", ctypes.c_int32), ("bits", ctypes.c_int32),
                ("entry_width", ctypes.c_int32), ("padding_byte", ctypes.c_int32), ("is_sorted", ctypes.c_int32),
                ("has_inverted", ctypes.c_int32), ("dict", ctypes.c_void_p), ("fwd", ctypes.c_void_p),
                ("raw", ctypes.c_int32), ("fwd_len", ctypes.c_int64), ("range_index", ctypes.c_void_p),
                ("range_index_len", ctypes.c_int64)]


class OrStarTree(ctypes.Structure):
    _fields_ = [("num_nodes", ctypes.c_int32), ("nodes", ctypes.POINTER(ctypes.c_int32)), ("num_docs", ctypes.c_int32),
                ("num_dims", ctypes.c_int32), ("dim_columns", ctypes.POINTER(ctypes.c_int32)),
                ("dim_fwd", ctypes.POINTER(ctypes.c_void_p)), ("num_metrics", ctypes.c_int32),
                ("metric_fn", ctypes.POINTER(ctypes.c_int32)), ("metric_column", ctypes.POINTER(ctypes.c_int32)),
                ("metric_f64", ctypes.POINTER(ctypes.c_void_p)), ("metric_i64", ctypes.POINTER(ctypes.c_void_p))]


class OrSegment(ctypes.Structure):
    _fields_ = [("num_docs", ctypes.c_int32), ("num_columns", ctypes.c_int32), ("columns", ctypes.POINTER(OrColumn)),
                ("star_tree", ctypes.POINTER(OrStarTree))]


class OrPredicate(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("column", ctypes.c_int32), ("num_values", ctypes.c_int32),
                ("values", ctypes.POINTER(ctypes.c_char_p)), ("lower_inclusive", ctypes.c_int32),
                ("upper_inclusive", ctypes.c_int32)]


class OrFilterOp(ctypes.Structure):
    _fields_ = [("op", ctypes.c_int32), ("arg", ctypes.c_int32)]


class OrAgg(ctypes.Structure):
    _fields_ = [("fn", ctypes.c_int32), ("column", ctypes.c_int32)]


class OrQuery(ctypes.Structure):
    _fields_ = [("num_predicates", ctypes.c_int32), ("predicates", ctypes.POINTER(OrPredicate)),
                ("num_filter_ops", ctypes.c_int32), ("filter", ctypes.POINTER(OrFilterOp)),
                ("num_group_by", ctypes.c_int32), ("group_by", ctypes.POINTER(ctypes.c_int32)),
                ("num_aggs", ctypes.c_int32), ("aggs", ctypes.POINTER(OrAgg)),
                ("num_groups_limit", ctypes.c_int32), ("max_initial_result_holder_capacity", ctypes.c_int32),
                ("combine", ctypes.c_int32), ("use_star_tree", ctypes.c_int32)]


class OrResult(ctypes.Structure):
    _fields_ = [("num_groups", ctypes.c_int64), ("key_blob", ctypes.POINTER(ctypes.c_uint8)),
                ("key_offsets", ctypes.POINTER(ctypes.c_int64)), ("values", ctypes.POINTER(ctypes.c_double)),
                ("avg_counts", ctypes.POINTER(ctypes.c_int64)), ("num_docs_scanned", ctypes.c_int64),
                ("num_entries_scanned_in_filter", ctypes.c_int64), ("num_entries_scanned_post_filter", ctypes.c_int64),
                ("num_total_docs", ctypes.c_int64), ("holder_kind", ctypes.c_int32),
                ("num_groups_limit_reached", ctypes.c_int32)]


class OrGenSpec(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("column_index", ctypes.c_int32), ("lo", ctypes.c_int64),
                ("hi", ctypes.c_int64), ("n", ctypes.c_int32), ("cdf", ctypes.POINTER(ctypes.c_double)),
                ("ids", ctypes.POINTER(ctypes.c_int64)), ("table", ctypes.POINTER(ctypes.c_double))]


HOLDERS = {0: "ARRAY", 1: "INT_MAP", 2: "LONG_MAP", 3: "ARRAY_MAP"}
_lib = None


def lib():
    global _lib
    if _lib is None:
        build_oracle()
        o = ctypes.CDLL(ORACLE_LIB)
        o.or_num_bits_per_value.restype = ctypes.c_int
        o.or_bitset_read_int.restype = ctypes.c_int32
        o.or_bitset_read_int.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]
        o.or_bitset_read_ints.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        o.or_bitset_write_int.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int32]
        o.or_bitset_write_ints.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        o.or_fwd_num_bytes.restype = ctypes.c_int64
        o.or_fwd_num_bytes.argtypes = [ctypes.c_int64, ctypes.c_int]
        o.or_read_dict_ids.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                       ctypes.c_void_p]
        for f in ("or_build_column_i64", "or_build_column_f64"):
            getattr(o, f).restype = ctypes.c_int
            getattr(o, f).argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        o.or_build_column_str.restype = ctypes.c_int
        o.or_build_column_str.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        o.or_execute_groupby.restype = ctypes.c_int
        o.or_execute_groupby.argtypes = [ctypes.POINTER(OrSegment), ctypes.c_int, ctypes.POINTER(OrQuery), ctypes.c_int,
                                         ctypes.POINTER(OrResult), ctypes.c_char_p, ctypes.c_int]
        o.or_free_result.argtypes = [ctypes.POINTER(OrResult)]
        o.or_filter_bitmap.restype = ctypes.c_int
        o.or_filter_bitmap.argtypes = [ctypes.POINTER(OrSegment), ctypes.POINTER(OrQuery), ctypes.c_void_p,
                                       ctypes.c_char_p, ctypes.c_int]
        o.or_bytes_alg.restype = ctypes.c_int64
        o.or_bytes_alg.argtypes = [ctypes.POINTER(OrSegment), ctypes.POINTER(OrQuery), ctypes.c_void_p]
        o.or_splitmix64.restype = ctypes.c_uint64
        o.or_splitmix64.argtypes = [ctypes.c_uint64]
        o.or_zipf_cdf.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_void_p]
        o.or_double_table.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_void_p]
        o.or_gen_i64.argtypes = [ctypes.POINTER(OrGenSpec), ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
        o.or_gen_f64.argtypes = [ctypes.POINTER(OrGenSpec), ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
        _lib = o
    return _lib


# ----------------------------------------------------------------------------------------------- builders
def build_column(dtype, values):
    """Pinot segment creation for one column: (sorted distinct) dictionary + fixed-bit forward index."""
    o = lib()
    bits, width = ctypes.c_int(), ctypes.c_int()
    if dtype == L.STRING:
        enc = [v.encode("utf-8") if isinstance(v, str) else bytes(v) for v in values]
        n = len(enc)
        blob = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8).copy()
        off = np.zeros(n + 1, dtype=np.int64)
        off[1:] = np.cumsum([len(e) for e in enc])
        maxw = max([len(e) for e in enc] + [1])
        d = np.zeros(max(n, 1) * maxw, dtype=np.uint8)
        f = np.zeros(o.or_fwd_num_bytes(n, 31) + 16, dtype=np.uint8)
        card = o.or_build_column_str(blob.ctypes.data, off.ctypes.data, n, d.ctypes.data, f.ctypes.data,
                                     ctypes.byref(bits), ctypes.byref(width))
    else:
        n = len(values)
        f = np.zeros(o.or_fwd_num_bytes(n, 31) + 16, dtype=np.uint8)
        if dtype in (L.INT, L.LONG):
            a = np.ascontiguousarray(values, dtype=np.int64)
            d = np.zeros(max(n, 1) * 8, dtype=np.uint8)
            card = o.or_build_column_i64(dtype, a.ctypes.data, n, d.ctypes.data, f.ctypes.data,
                                         ctypes.byref(bits), ctypes.byref(width))
        else:
            a = np.ascontiguousarray(values, dtype=np.float64)
            d = np.zeros(max(n, 1) * 8, dtype=np.uint8)
            card = o.or_build_column_f64(dtype, a.ctypes.data, n, d.ctypes.data, f.ctypes.data,
                                         ctypes.byref(bits), ctypes.byref(width))
    nfwd = o.or_fwd_num_bytes(n, bits.value)
    return ColumnData(dtype, card, bits.value, width.value, d[:card * width.value].tobytes(), f[:nfwd].tobytes())


def make_segment(schema, columns):
    """schema: [(name, type)], columns: name -> values.  Returns SegmentBuffers."""
    n = None
    cols = {}
    for name, t in schema:
        tt = L.TYPE_NAMES[t] if isinstance(t, str) else t
        vals = columns[name]
        n = len(vals) if n is None else n
        assert len(vals) == n
        cols[name] = build_column(tt, vals)
    return SegmentBuffers(n or 0, cols)


# ----------------------------------------------------------------------------------------------- queries
class _OrSeg:
    def __init__(self, schema, seg):
        self.keep = []
        cols = (OrColumn * len(schema))()
        for i, (name, t) in enumerate(schema):
            c = seg.columns[name]
            d = ctypes.create_string_buffer(bytes(c.dict_bytes), max(len(c.dict_bytes), 1))
            f = ctypes.create_string_buffer(bytes(c.fwd_bytes) + b"\0" * 16, len(c.fwd_bytes) + 16)
            self.keep += [d, f]
            rng = getattr(c, "range_bytes", None)
            r = ctypes.create_string_buffer(bytes(rng), max(len(rng), 1)) if rng else None
            self.keep.append(r)
            cols[i] = OrColumn(c.data_type, c.cardinality, c.bits_per_element, c.entry_width, c.padding_byte,
                               int(c.is_sorted), int(getattr(c, "inv_bytes", None) is not None),
                               ctypes.cast(d, ctypes.c_void_p), ctypes.cast(f, ctypes.c_void_p),
                               int(c.fwd_format == L.FWD_RAW_FIXED), len(c.fwd_bytes),
                               ctypes.cast(r, ctypes.c_void_p) if r is not None else None, len(rng) if rng else 0)
        self.keep.append(cols)
        self.seg = OrSegment(seg.num_docs, len(schema), cols)
        star = getattr(seg, "star_arrays", None)  # StarTree.arrays() of the segment's star-tree, if any
        if star is not None:
            self.seg.star_tree = ctypes.pointer(self._star(star))

    def _star(self, a):
        keep = self.keep
        nodes = np.ascontiguousarray(a["nodes"], dtype=np.int32)
        dims = np.ascontiguousarray(a["dim_columns"], dtype=np.int32)
        fwd = [ctypes.create_string_buffer(bytes(f) + b"\0" * 16, len(f) + 16) for f in a["dim_fwd"]]
        fwd_p = (ctypes.c_void_p * max(len(fwd), 1))(*[ctypes.cast(f, ctypes.c_void_p) for f in fwd])
        fns = np.ascontiguousarray([m[0] for m in a["metrics"]], dtype=np.int32)
        mcols = np.ascontiguousarray([m[1] for m in a["metrics"]], dtype=np.int32)
        f64 = [None if x is None else np.ascontiguousarray(x, dtype=np.float64) for x in a["metric_f64"]]
        i64 = [None if x is None else np.ascontiguousarray(x, dtype=np.int64) for x in a["metric_i64"]]
        f_p = (ctypes.c_void_p * max(len(f64), 1))(*[None if x is None else x.ctypes.data for x in f64])
        i_p = (ctypes.c_void_p * max(len(i64), 1))(*[None if x is None else x.ctypes.data for x in i64])
        keep += [nodes, dims, fwd, fwd_p, fns, mcols, f64, i64, f_p, i_p]
        st = OrStarTree(len(nodes), nodes.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), int(a["num_docs"]), len(dims),
                        dims.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), fwd_p, len(fns),
                        fns.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                        mcols.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), f_p, i_p)
        keep.append(st)
        return st


def _or_query(schema, q, combine=True, max_initial_capacity=10000, use_star_tree=False):
    idx = {n: i for i, (n, _) in enumerate(schema)}
    keep = []
    preds, ops = [], []
    if q.filter is not None:
        q.filter.postfix(preds, ops)
    pc = (OrPredicate * max(len(preds), 1))()
    codes = {"EQ": 0, "NOT_EQ": 1, "IN": 2, "NOT_IN": 3, "RANGE": 4}
    for i, p in enumerate(preds):
        vals = (ctypes.c_char_p * max(len(p.values), 1))(*[v.encode() for v in p.values])
        keep.append(vals)
        pc[i] = OrPredicate(codes[p.type], idx[p.column], len(p.values), vals, int(p.lower_inclusive),
                            int(p.upper_inclusive))
    oc = (OrFilterOp * max(len(ops), 1))(*[OrFilterOp(o, a) for o, a in ops])
    gb = (ctypes.c_int32 * max(len(q.group_by), 1))(*[idx[c] for c in q.group_by])
    fns = {"COUNT": 0, "SUM": 1, "MIN": 2, "MAX": 3, "AVG": 4}
    ac = (OrAgg * max(len(q.aggregations), 1))(*[OrAgg(fns[f], -1 if c == "*" else idx[c]) for f, c in q.aggregations])
    keep += [pc, oc, gb, ac]
    oq = OrQuery(len(preds), pc, len(ops), oc, len(q.group_by), gb, len(q.aggregations), ac, q.num_groups_limit,
                 max_initial_capacity, int(combine), int(use_star_tree))
    return oq, keep


class OracleResult:
    def __init__(self, groups, stats, holder, limit_reached):
        self.groups = groups   # key tuple -> [values] (AVG -> AvgPair, COUNT -> int)
        self.stats = stats     # (docsScanned, inFilter, postFilter, totalDocs)
        self.holder = holder
        self.limit_reached = limit_reached


def _decode_key(blob, types):
    out, p = [], 0
    for t in types:
        if t in (L.INT, L.LONG):
            out.append(int(np.frombuffer(blob[p:p + 8], dtype=np.int64)[0]))
            p += 8
        elif t in (L.FLOAT, L.DOUBLE):
            out.append(float(np.frombuffer(blob[p:p + 8], dtype=np.float64)[0]))
            p += 8
        else:
            n = int(np.frombuffer(blob[p:p + 4], dtype=np.uint32)[0])
            out.append(blob[p + 4:p + 4 + n].decode("utf-8", errors="surrogateescape"))
            p += 4 + n
    return tuple(out)


def run_groupby(schema, segments, q, nthreads=8, combine=True, max_initial_capacity=10000, decode=True,
                use_star_tree=False):
    """decode=False: run the operator + combine only and return the group count (bench timing leg)."""
    o = lib()
    segs = [_OrSeg(schema, s) for s in segments]
    arr = (OrSegment * max(len(segs), 1))(*[s.seg for s in segs])
    oq, keep = _or_query(schema, q, combine, max_initial_capacity, use_star_tree)
    res = OrResult()
    msg = ctypes.create_string_buffer(512)
    rc = o.or_execute_groupby(arr, len(segs), ctypes.byref(oq), nthreads, ctypes.byref(res), msg, 512)
    if rc != 0:
        raise RuntimeError("oracle error %d: %s" % (rc, msg.value.decode()))
    try:
        if not decode:
            return res.num_groups
        types = {n: (L.TYPE_NAMES[t] if isinstance(t, str) else t) for n, t in schema}
        ktypes = [types[c] for c in q.group_by]
        n = res.num_groups
        na = len(q.aggregations)
        blob = ctypes.string_at(res.key_blob, res.key_offsets[n]) if n else b""
        groups = {}
        for gi in range(n):
            k = _decode_key(blob[res.key_offsets[gi]:res.key_offsets[gi + 1]], ktypes)
            vals = []
            for a, (fn, _) in enumerate(q.aggregations):
                v = res.values[a * n + gi]
                if fn == "AVG":
                    vals.append(AvgPair(v, res.avg_counts[a * n + gi]))
                elif fn == "COUNT":
                    vals.append(int(v))
                else:
                    vals.append(float(v))
            groups[k] = vals
        stats = (res.num_docs_scanned, res.num_entries_scanned_in_filter, res.num_entries_scanned_post_filter,
                 res.num_total_docs)
        return OracleResult(groups, stats, HOLDERS[res.holder_kind], bool(res.num_groups_limit_reached))
    finally:
        o.or_free_result(ctypes.byref(res))


def run_groupby_arrays(schema, segments, q, nthreads=8, combine=True, max_initial_capacity=10000, use_star_tree=False):
    """run_groupby for numeric group-by keys, returned as numpy arrays (large results: millions of groups):
    (keys [n, num_group_by] int64 / float64, values [num_aggs, n] float64, avg_counts [num_aggs, n] int64, stats)."""
    o = lib()
    types = {n: (L.TYPE_NAMES[t] if isinstance(t, str) else t) for n, t in schema}
    ktypes = [types[c] for c in q.group_by]
    assert all(t != L.STRING for t in ktypes), "numeric group-by keys only"
    segs = [_OrSeg(schema, s) for s in segments]
    arr = (OrSegment * max(len(segs), 1))(*[s.seg for s in segs])
    oq, keep = _or_query(schema, q, combine, max_initial_capacity, use_star_tree)
    res = OrResult()
    msg = ctypes.create_string_buffer(512)
    rc = o.or_execute_groupby(arr, len(segs), ctypes.byref(oq), nthreads, ctypes.byref(res), msg, 512)
    if rc != 0:
        raise RuntimeError("oracle error %d: %s" % (rc, msg.value.decode()))
    try:
        n, nk, na = res.num_groups, len(ktypes), len(q.aggregations)
        raw = np.frombuffer(ctypes.string_at(res.key_blob, n * nk * 8), dtype=np.uint8) if n and nk else \
            np.zeros(0, dtype=np.uint8)
        keys = np.zeros((n, nk), dtype=object if len(set(ktypes)) > 1 else np.float64)
        words = raw.view(np.int64).reshape(n, nk) if n and nk else np.zeros((n, nk), dtype=np.int64)
        if all(t in (L.INT, L.LONG) for t in ktypes):
            keys = words.copy()
        else:
            keys = np.stack([words[:, j] if t in (L.INT, L.LONG) else words[:, j].view(np.float64)
                             for j, t in enumerate(ktypes)], axis=1).astype(np.float64) if nk else keys
        vals = np.ctypeslib.as_array(res.values, shape=(na * n,)).reshape(na, n).copy() if n and na else \
            np.zeros((na, n))
        cnts = np.ctypeslib.as_array(res.avg_counts, shape=(na * n,)).reshape(na, n).copy() if n and na else \
            np.zeros((na, n), dtype=np.int64)
        stats = (res.num_docs_scanned, res.num_entries_scanned_in_filter, res.num_entries_scanned_post_filter,
                 res.num_total_docs)
        return keys, vals, cnts, stats
    finally:
        o.or_free_result(ctypes.byref(res))


def filter_bitmap(schema, seg, q):
    o = lib()
    s = _OrSeg(schema, seg)
    oq, keep = _or_query(schema, q)
    out = np.zeros(max((seg.num_docs + 63) // 64, 1), dtype=np.uint64)
    msg = ctypes.create_string_buffer(512)
    rc = o.or_filter_bitmap(ctypes.byref(s.seg), ctypes.byref(oq), out.ctypes.data, msg, 512)
    if rc != 0:
        raise RuntimeError("oracle error %d: %s" % (rc, msg.value.decode()))
    return out


def bytes_alg(schema, seg, q, bitmap):
    s = _OrSeg(schema, seg)
    oq, keep = _or_query(schema, q)
    return int(lib().or_bytes_alg(ctypes.byref(s.seg), ctypes.byref(oq), bitmap.ctypes.data))


# ----------------------------------------------------------------------------------------------- data
def zipf_cdf(n, s=1.0):
    out = np.zeros(n, dtype=np.float64)
    lib().or_zipf_cdf(n, s, out.ctypes.data)
    return out


def double_table(n, column_index, lo, hi):
    out = np.zeros(n, dtype=np.float64)
    lib().or_double_table(n, column_index, lo, hi, out.ctypes.data)
    return out


def gen_values(spec, row0, n):
    """spec: dict as for GpuTable.generate_segment."""
    kinds = {"UNIFORM": 0, "ZIPF": 1, "TABLE": 2}
    keep = []
    g = OrGenSpec()
    g.kind = kinds[spec["kind"]]
    g.column_index = spec["column_index"]
    g.lo = int(spec.get("lo", 0))
    g.hi = int(spec.get("hi", 0))
    if spec["kind"] == "ZIPF":
        cdf = np.ascontiguousarray(spec["cdf"], dtype=np.float64)
        ids = np.ascontiguousarray(spec["ids"], dtype=np.int64)
        keep += [cdf, ids]
        g.n = len(cdf)
        g.cdf = cdf.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
        g.ids = ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
    if spec["kind"] == "TABLE":
        tab = np.ascontiguousarray(spec["table"], dtype=np.float64)
        keep.append(tab)
        g.n = len(tab)
        g.table = tab.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
        out = np.zeros(n, dtype=np.float64)
        lib().or_gen_f64(ctypes.byref(g), row0, n, out.ctypes.data)
        return out
    out = np.zeros(n, dtype=np.int64)
    lib().or_gen_i64(ctypes.byref(g), row0, n, out.ctypes.data)
    return out


# ------------------------------------------------------------------------------------------ result comparison
def gpu_result_arrays(table, r, q):
    """A GPU GroupByResult as (keys [n, k] in value space, values [num_aggs, n] float64, AVG counts), keys sorted."""
    cols = r.gid_columns
    keys = np.stack([np.asarray(table.dictionary(c))[g] for c, g in zip(q.group_by, cols)], axis=1) if cols else \
        np.zeros((len(r), 0))
    vals, cnts = [], []
    for fn, v, e, c in r._col[2]:
        vals.append(v if v is not None else e.astype(np.float64))
        cnts.append(c if c is not None else np.zeros(len(r), dtype=np.int64))
    return sort_by_key(keys, np.array(vals).reshape(len(q.aggregations), len(r)),
                       np.array(cnts).reshape(len(q.aggregations), len(r)))


def sort_by_key(keys, vals, cnts):
    order = np.lexsort(keys.T[::-1]) if keys.shape[1] else np.arange(len(keys))
    return keys[order], vals[:, order], cnts[:, order]


def compare_result_arrays(table, r, orc, q, schema, rel=1e-9, check_stats=True):
    """The parity bar of the path against run_groupby_arrays' output: same groups, bit-exact COUNT / integer SUM /
    MIN / MAX and AVG counts, FLOAT / DOUBLE sums within `rel` relative (1e-6 absolute near zero).  check_stats: True
    = every statistic, "docs" = numDocsScanned only (index-backed leaves scan no entries), False = none (star-tree
    plans scan pre-aggregated documents).  Returns a dict (ok, groups, max_rel_err of the FP sums, first mismatch)
    instead of raising: bench.py reports it in its line."""
    return compare_arrays(gpu_result_arrays(table, r, q), r.stats.as_tuple(), orc, q, schema, rel, check_stats)


def compare_arrays(gpu, gpu_stats, orc, q, schema, rel=1e-9, check_stats=True):
    """compare_result_arrays on a GPU answer already in array form: gpu = (keys, values, AVG counts) as
    gpu_result_arrays returns them (sorted by key), gpu_stats the 4 statistics; orc as run_groupby_arrays returns it."""
    types = {n: t for n, t in schema}
    gk, gv, gc = gpu
    ok_, ov, oc, ostats = orc
    ok_, ov, oc = sort_by_key(ok_.astype(gk.dtype) if len(ok_) else ok_.reshape(0, gk.shape[1]), ov, oc)
    out = {"ok": True, "groups": int(len(gk)), "max_rel_err_fp_sum": 0.0, "mismatch": None}

    def bad(msg):
        out["ok"] = False
        out["mismatch"] = out["mismatch"] or msg

    if gk.shape != ok_.shape or not np.array_equal(gk, ok_):
        bad("groups differ: gpu %s, oracle %s" % (gk.shape, ok_.shape))
        return out
    for a, (fn, col) in enumerate(q.aggregations):
        fp = col != "*" and types[col] in ("FLOAT", "DOUBLE")
        if fp and fn in ("SUM", "AVG"):
            den = np.maximum(np.abs(ov[a]), 1e-300)
            err = np.where(np.abs(gv[a] - ov[a]) <= 1e-6, 0.0, np.abs(gv[a] - ov[a]) / den)
            e = float(err.max()) if len(err) else 0.0
            out["max_rel_err_fp_sum"] = max(out["max_rel_err_fp_sum"], e)
            if e > rel:
                bad("%s(%s): relative error %.3g" % (fn, col, e))
        elif not np.array_equal(gv[a], ov[a]):
            i = int(np.nonzero(gv[a] != ov[a])[0][0])
            bad("%s(%s) group %d: gpu %r, oracle %r" % (fn, col, i, gv[a][i], ov[a][i]))
        if fn == "AVG" and not np.array_equal(gc[a], oc[a]):
            bad("AVG(%s) counts" % col)
    if check_stats is True and tuple(gpu_stats) != tuple(ostats):
        bad("statistics: gpu %s, oracle %s" % (tuple(gpu_stats), tuple(ostats)))
    elif check_stats == "docs" and gpu_stats[0] != ostats[0]:
        bad("numDocsScanned: gpu %d, oracle %d" % (gpu_stats[0], ostats[0]))
    return out


def concat_arrays(parts):
    """Disjoint per-rank answers (gpu_result_arrays triples: reduce-scattered key ranges, hash owners' shares) as one
    answer sorted by key."""
    parts = list(parts)
    keys = np.concatenate([p[0] for p in parts], axis=0)
    vals = np.concatenate([p[1] for p in parts], axis=1)
    cnts = np.concatenate([p[2] for p in parts], axis=1)
    return sort_by_key(keys, vals, cnts)


def merge_partial_arrays(parts, aggregations):
    """The merge of per-server partial results (run_groupby_arrays outputs, one per rank's segments), as the broker
    merges server responses (GroupByDataTableReducer / GroupByOrderByCombineOperator.java:170-181): per group COUNT,
    SUM and AVG's (sum, count) add, MIN / MAX take the min / max; the statistics add.  numpy, independent of the
    device combine it checks (no group-count limit may bind: the bench's workloads never reach theirs)."""
    parts = list(parts)
    keys = np.concatenate([p[0] for p in parts], axis=0)
    vals = np.concatenate([p[1] for p in parts], axis=1)
    cnts = np.concatenate([p[2] for p in parts], axis=1)
    stats = tuple(int(sum(p[3][i] for p in parts)) for i in range(4))
    if len(keys) == 0:
        return keys, vals, cnts, stats
    keys, vals, cnts = sort_by_key(keys, vals, cnts)
    new = np.ones(len(keys), dtype=bool)
    if keys.shape[1]:
        new[1:] = np.any(keys[1:] != keys[:-1], axis=1)
    else:
        new[1:] = False
    starts = np.nonzero(new)[0]
    mv = np.empty((vals.shape[0], len(starts)), dtype=vals.dtype)
    mc = np.empty((cnts.shape[0], len(starts)), dtype=cnts.dtype)
    for a, (fn, _) in enumerate(aggregations):
        red = np.minimum if fn == "MIN" else np.maximum if fn == "MAX" else np.add
        mv[a] = red.reduceat(vals[a], starts)
        mc[a] = np.add.reduceat(cnts[a], starts)
    return keys[starts], mv, mc, stats


def segments_from_table(table, handles, schema, docs):
    """Each pinned segment's Pinot bytes read back from HBM, as the oracle's input."""
    segs = []
    for h in handles:
        cols = {}
        for name, typ in schema:
            card, bits, d, f = table.segment_column_bytes(int(h), name)
            tcode = L.TYPE_NAMES[typ] if isinstance(typ, str) else typ
            cols[name] = ColumnData(tcode, card, bits, 4 if tcode in (L.INT, L.FLOAT) else 8, d, f)
        segs.append(SegmentBuffers(docs, cols))
    return segs
