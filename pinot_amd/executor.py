"""Host layer over the C ABI: a pinned table, query plans and decoded group-by results.

GpuTable      one Pinot table's segments pinned in one GPU's HBM + the table-global dictionaries
              (the key space that replaces GroupByCombineOperator's by-value merge).
Plan          a compiled query over a segment list: execute (async, dense group table in device memory,
              optionally a caller-owned buffer such as a torch tensor so RCCL can reduce it), finalize.
GroupByResult decoded groups {key tuple: [aggregation results]} + ExecutionStatistics.
"""
import ctypes

import numpy as np

from . import _lib as L
from .query import QueryContext


class ExecutionStatistics:
    """core/operator/ExecutionStatistics.java:42 (+ segment counters)."""

    def __init__(self, stats6):
        (self.num_docs_scanned, self.num_entries_scanned_in_filter, self.num_entries_scanned_post_filter,
         self.num_total_docs, self.num_segments_processed, self.num_segments_matched) = [int(x) for x in stats6]

    def as_tuple(self):
        return (self.num_docs_scanned, self.num_entries_scanned_in_filter, self.num_entries_scanned_post_filter,
                self.num_total_docs)

    def __repr__(self):
        return "ExecutionStatistics(docsScanned=%d, inFilter=%d, postFilter=%d, totalDocs=%d)" % self.as_tuple()


class AvgPair:
    """core/query/aggregation/function/customobject/AvgPair."""
    __slots__ = ("sum", "count")

    def __init__(self, s, c):
        self.sum, self.count = float(s), int(c)

    def final(self):
        return self.sum / self.count if self.count else float("-inf")  # AvgAggregationFunction.java:185-192

    def __eq__(self, o):
        return isinstance(o, AvgPair) and self.sum == o.sum and self.count == o.count

    def __repr__(self):
        return "AvgPair(%r, %d)" % (self.sum, self.count)


class GroupByResult:
    def __init__(self, keys, values, stats, exact=None):
        self.keys = keys            # list of key tuples (python values), ascending composite key
        self.values = values        # list (per group) of lists (per aggregation)
        self.stats = stats
        self.exact = exact or {}    # agg index -> np.int64 array of exact integer accumulators

    def as_dict(self):
        return {k: v for k, v in zip(self.keys, self.values)}

    def string_keys(self):
        """GroupKeyGenerator.StringGroupKey form: values joined by GroupKeyGenerator.DELIMITER ('\\0')."""
        return {"\0".join(_key_str(x) for x in k): v for k, v in zip(self.keys, self.values)}

    def __len__(self):
        return len(self.keys)


def _key_str(x):
    if isinstance(x, float):
        return repr(x)
    return str(x)


class GpuTable:
    def __init__(self, schema, device=0):
        """schema: list of (column name, type name 'INT'|'LONG'|'FLOAT'|'DOUBLE'|'STRING')."""
        self.lib = L.load()
        self.names = [n for n, _ in schema]
        self.types = [L.TYPE_NAMES[t] if isinstance(t, str) else int(t) for _, t in schema]
        self.index = {n: i for i, n in enumerate(self.names)}
        self.device = device
        names = (ctypes.c_char_p * len(self.names))(*[n.encode() for n in self.names])
        types = (ctypes.c_int32 * len(self.types))(*self.types)
        h = ctypes.c_void_p()
        L.check(self.lib.pgpu_table_create(device, len(self.names), names, types, ctypes.byref(h)))
        self.handle = h
        self._dict_cache = {}

    def close(self):
        if self.handle:
            self.lib.pgpu_table_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ------------------------------------------------------------------ segments
    def pin_segment(self, seg):
        """Pins SegmentBuffers (ImmutableSegmentLoader.load time); returns the segment handle."""
        cols = (L.ColumnBuffers * len(self.names))()
        keep = []
        for i, name in enumerate(self.names):
            c = seg.columns[name]
            d = ctypes.create_string_buffer(bytes(c.dict_bytes), max(len(c.dict_bytes), 1))
            f = ctypes.create_string_buffer(bytes(c.fwd_bytes), max(len(c.fwd_bytes), 1))
            keep += [d, f]
            cols[i].cardinality = c.cardinality
            cols[i].bits_per_element = c.bits_per_element
            cols[i].entry_width = c.entry_width
            cols[i].padding_byte = c.padding_byte
            cols[i].fwd_format = c.fwd_format
            cols[i].dict = ctypes.cast(d, ctypes.c_void_p)
            cols[i].dict_len = len(c.dict_bytes)
            cols[i].fwd = ctypes.cast(f, ctypes.c_void_p)
            cols[i].fwd_len = len(c.fwd_bytes)
        desc = L.SegmentDesc(seg.num_docs, len(self.names), cols)
        h = ctypes.c_int64()
        L.check(self.lib.pgpu_pin_segment(self.handle, ctypes.byref(desc), ctypes.byref(h)))
        self._dict_cache.clear()
        return h.value

    def attach_startree(self, handle, star_tree):
        """Pins a StarTree (pinot_amd.startree) for the pinned segment `handle`."""
        from .startree import attach
        attach(self, handle, star_tree)

    def unpin_segment(self, handle):
        L.check(self.lib.pgpu_unpin_segment(self.handle, handle))
        self._dict_cache.clear()

    def generate_segment(self, gen_columns, row0, num_docs):
        """Builds a synthetic segment on the device (BASELINE.md §3 generators). gen_columns: list of dicts
        {kind: 'UNIFORM'|'ZIPF'|'TABLE', column_index, lo, hi, cdf, ids, table} in table column order."""
        arr = (L.GenColumnC * len(gen_columns))()
        keep = []
        for i, g in enumerate(gen_columns):
            kind = {"UNIFORM": L.GEN_UNIFORM, "ZIPF": L.GEN_ZIPF, "TABLE": L.GEN_TABLE}[g["kind"]]
            arr[i].kind = kind
            arr[i].column_index = g["column_index"]
            arr[i].lo = int(g.get("lo", 0))
            arr[i].hi = int(g.get("hi", 0))
            if kind == L.GEN_ZIPF:
                cdf = np.ascontiguousarray(g["cdf"], dtype=np.float64)
                ids = np.ascontiguousarray(g["ids"], dtype=np.int64)
                keep += [cdf, ids]
                arr[i].n = len(cdf)
                arr[i].cdf = L.ptr(cdf, ctypes.c_double)
                arr[i].ids = L.ptr(ids, ctypes.c_int64)
            elif kind == L.GEN_TABLE:
                tab = np.ascontiguousarray(g["table"], dtype=np.float64)
                keep.append(tab)
                arr[i].n = len(tab)
                arr[i].table = L.ptr(tab, ctypes.c_double)
        h = ctypes.c_int64()
        L.check(self.lib.pgpu_generate_segment(self.handle, arr, len(gen_columns), int(row0), int(num_docs),
                                               ctypes.byref(h)))
        self._dict_cache.clear()
        return h.value

    def segment_column_bytes(self, handle, column):
        ci = self.index[column]
        card, bits = ctypes.c_int32(), ctypes.c_int32()
        dl, fl = ctypes.c_int64(), ctypes.c_int64()
        L.check(self.lib.pgpu_segment_column_info(self.handle, handle, ci, ctypes.byref(card), ctypes.byref(bits),
                                                  ctypes.byref(dl), ctypes.byref(fl)))
        d = np.zeros(max(dl.value, 1), dtype=np.uint8)
        f = np.zeros(max(fl.value, 1), dtype=np.uint8)
        L.check(self.lib.pgpu_segment_column_bytes(self.handle, handle, ci, L.ptr(d, ctypes.c_uint8),
                                                   L.ptr(f, ctypes.c_uint8)))
        return card.value, bits.value, d[:dl.value].tobytes(), f[:fl.value].tobytes()

    def num_segments(self):
        n = ctypes.c_int32()
        L.check(self.lib.pgpu_table_num_segments(self.handle, ctypes.byref(n)))
        return n.value

    def device_bytes(self):
        return int(self.lib.pgpu_table_device_bytes(self.handle))

    # ------------------------------------------------------------------ dictionaries
    def add_dictionary_values(self, column, values):
        ci = self.index[column]
        t = self.types[ci]
        if t in (L.INT, L.LONG):
            a = np.ascontiguousarray(values, dtype=np.int64)
            L.check(self.lib.pgpu_table_add_dictionary_values(self.handle, ci, len(a), L.ptr(a, ctypes.c_int64),
                                                              None, None, None))
        elif t in (L.FLOAT, L.DOUBLE):
            a = np.ascontiguousarray(values, dtype=np.float64)
            L.check(self.lib.pgpu_table_add_dictionary_values(self.handle, ci, len(a), None,
                                                              L.ptr(a, ctypes.c_double), None, None))
        else:
            enc = [v.encode() if isinstance(v, str) else bytes(v) for v in values]
            blob = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8).copy()
            off = np.zeros(len(enc) + 1, dtype=np.int64)
            off[1:] = np.cumsum([len(e) for e in enc])
            L.check(self.lib.pgpu_table_add_dictionary_values(self.handle, ci, len(enc), None, None,
                                                              L.ptr(blob, ctypes.c_uint8), L.ptr(off, ctypes.c_int64)))
        self._dict_cache.clear()

    def dictionary(self, column):
        """Table-global dictionary of `column` (sorted values; the group ids of results index it)."""
        if column in self._dict_cache:
            return self._dict_cache[column]
        ci = self.index[column]
        n = ctypes.c_int64()
        L.check(self.lib.pgpu_table_dictionary_size(self.handle, ci, ctypes.byref(n)))
        t = self.types[ci]
        if t in (L.INT, L.LONG):
            a = np.zeros(max(n.value, 1), dtype=np.int64)
            L.check(self.lib.pgpu_table_dictionary_i64(self.handle, ci, L.ptr(a, ctypes.c_int64)))
            vals = [int(x) for x in a[:n.value]]
        elif t in (L.FLOAT, L.DOUBLE):
            a = np.zeros(max(n.value, 1), dtype=np.float64)
            L.check(self.lib.pgpu_table_dictionary_f64(self.handle, ci, L.ptr(a, ctypes.c_double)))
            vals = [float(x) for x in a[:n.value]]
        else:
            off = np.zeros(n.value + 1, dtype=np.int64)
            L.check(self.lib.pgpu_table_dictionary_str(self.handle, ci, None, 0, L.ptr(off, ctypes.c_int64)))
            blob = np.zeros(max(int(off[-1]), 1), dtype=np.uint8)
            L.check(self.lib.pgpu_table_dictionary_str(self.handle, ci, L.ptr(blob, ctypes.c_uint8), len(blob),
                                                       L.ptr(off, ctypes.c_int64)))
            b = blob.tobytes()
            vals = [b[off[i]:off[i + 1]].decode("utf-8", errors="surrogateescape") for i in range(n.value)]
        self._dict_cache[column] = vals
        return vals

    # ------------------------------------------------------------------ readers
    def read_dict_ids(self, handle, column, doc_ids):
        """ForwardIndexReader.readDictIds on the pinned copy (GPU unpack)."""
        docs = np.ascontiguousarray(doc_ids, dtype=np.int32)
        out = np.zeros(max(len(docs), 1), dtype=np.int32)
        L.check(self.lib.pgpu_read_dict_ids(self.handle, handle, self.index[column], L.ptr(docs, ctypes.c_int32),
                                            len(docs), L.ptr(out, ctypes.c_int32)))
        return out[:len(docs)]

    def filter_bitmap(self, handle, query, num_docs):
        q, keep = query.to_c(self.index)
        out = np.zeros(max((num_docs + 63) // 64, 1), dtype=np.uint64)
        L.check(self.lib.pgpu_filter_bitmap(self.handle, handle, ctypes.byref(q), L.ptr(out, ctypes.c_uint64)))
        return out

    # ------------------------------------------------------------------ queries
    def plan(self, handles, query):
        return Plan(self, handles, query)

    def execute_groupby(self, handles, query, stream=None):
        with Plan(self, handles, query) as p:
            p.execute(stream)
            return p.finalize(stream)


class Plan:
    def __init__(self, table, handles, query):
        if isinstance(query, str):
            from .query import parse_query
            query = parse_query(query)
        self.table = table
        self.query = query
        self.lib = table.lib
        hs = handles if isinstance(handles, np.ndarray) and handles.dtype == np.int64 else \
            np.ascontiguousarray(list(handles), dtype=np.int64)
        q, keep = query.to_c(table.index)
        h = ctypes.c_void_p()
        L.check(self.lib.pgpu_plan_create(table.handle, L.ptr(hs, ctypes.c_int64), len(hs), ctypes.byref(q),
                                          ctypes.byref(h)))
        self.handle = h
        self.num_segments = len(hs)

    def close(self):
        if self.handle:
            self.lib.pgpu_plan_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def layout(self):
        """(num_slots, num_keys, slot_kinds) of the dense group table ([num_slots][num_keys] 8-byte words)."""
        ns, nk = ctypes.c_int32(), ctypes.c_int64()
        kinds = (ctypes.c_int32 * 32)()
        L.check(self.lib.pgpu_plan_layout(self.handle, ctypes.byref(ns), ctypes.byref(nk), kinds))
        return ns.value, nk.value, [kinds[i] for i in range(ns.value)]

    def execute(self, stream=None, d_table=None):
        L.check(self.lib.pgpu_plan_execute(self.handle, ctypes.c_void_p(stream or 0), ctypes.c_void_p(d_table or 0)))

    def scanned_segments(self):
        """Per plan segment: True if scanned (its filter does not fold to always-false)."""
        out = np.zeros(max(self.num_segments, 1), dtype=np.uint8)
        L.check(self.lib.pgpu_plan_scanned_segments(self.handle, L.ptr(out, ctypes.c_uint8)))
        return out[:self.num_segments].astype(bool)

    def timing_us(self):
        out = (ctypes.c_double * 3)()
        L.check(self.lib.pgpu_plan_timing(self.handle, out))
        return out[0], out[1]

    def finalize(self, stream=None, d_table=None):
        r = ctypes.c_void_p()
        L.check(self.lib.pgpu_plan_finalize(self.handle, ctypes.c_void_p(stream or 0), ctypes.c_void_p(d_table or 0),
                                            ctypes.byref(r)))
        try:
            return _decode_result(self.table, self.query, r)
        finally:
            self.lib.pgpu_result_destroy(r)


def _decode_result(table, query, r):
    lib = table.lib
    n = ctypes.c_int64()
    L.check(lib.pgpu_result_num_groups(r, ctypes.byref(n)))
    n = n.value
    nk = len(query.group_by)
    gids = np.zeros(max(n * nk, 1), dtype=np.int32)
    L.check(lib.pgpu_result_group_ids(r, L.ptr(gids, ctypes.c_int32)))
    gids = gids[:n * nk].reshape(n, nk) if n else np.zeros((0, nk), dtype=np.int32)
    dicts = [table.dictionary(c) for c in query.group_by]
    keys = [tuple(dicts[j][int(gids[i, j])] for j in range(nk)) for i in range(n)]
    cols = []
    exact = {}
    for a, (fn, _) in enumerate(query.aggregations):
        v = np.zeros(max(n, 1), dtype=np.float64)
        L.check(lib.pgpu_result_values(r, a, L.ptr(v, ctypes.c_double)))
        v = v[:n]
        e = np.zeros(max(n, 1), dtype=np.int64)
        if lib.pgpu_result_values_i64(r, a, L.ptr(e, ctypes.c_int64)) == L.PGPU_OK:
            exact[a] = e[:n].copy()
        if fn == "AVG":
            c = np.zeros(max(n, 1), dtype=np.int64)
            L.check(lib.pgpu_result_avg_counts(r, a, L.ptr(c, ctypes.c_int64)))
            cols.append([AvgPair(v[i], c[i]) for i in range(n)])
        elif fn == "COUNT":
            cols.append([int(x) for x in e[:n]] if a in exact else [int(x) for x in v])
        else:
            cols.append([float(x) for x in v])
    values = [[cols[a][i] for a in range(len(cols))] for i in range(n)]
    st = np.zeros(6, dtype=np.int64)
    L.check(lib.pgpu_result_stats(r, L.ptr(st, ctypes.c_int64)))
    return GroupByResult(keys, values, ExecutionStatistics(st), exact)
