"""Host layer over the C ABI: a pinned table, query plans and decoded group-by results.

GpuTable      one Pinot table's segments pinned in one GPU's HBM + the table-global dictionaries
              (the key space that replaces GroupByCombineOperator's by-value merge).
Plan          a compiled query over a segment list: execute (async, dense group table in device memory,
              optionally a caller-owned buffer such as a torch tensor so RCCL can reduce it), finalize.
GroupByResult decoded groups {key tuple: [aggregation results]} + ExecutionStatistics.
"""
import ctypes
import time

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
    """Groups in the C result's order (ascending composite key; hash-mode results of >= 4096 groups in partition
    order, as the LONG_MAP holder iterates in hash order), held columnar (numpy) as the C ABI returns them; the Python form
    ({key tuple: [aggregation results]}) is built on first use of `keys` / `values` / `as_dict()`."""

    def __init__(self, keys=None, values=None, stats=None, exact=None, columnar=None, holder=None, table=None,
                 query=None, n=None):
        self.stats = stats
        self.num_groups_limit_reached = False
        self._holder, self._table, self._query = holder, table, query  # the C result behind the columnar views
        self._exact = exact         # agg index -> np.int64 array of exact integer accumulators
        self._keys, self._values = keys, values
        # columnar: (dicts, [per group-by column: [n] int32 dictIds], per-agg (fn, values f64 | None,
        # exact i64 | None, counts | None), n) -- numpy views of the C result's pinned buffer; or a loader
        # returning (columnar, exact), called on first use (a compact C result is decoded then, not before)
        self._col_data = None if callable(columnar) else columnar
        self._col_loader = columnar if callable(columnar) else None
        self._n = len(keys) if keys is not None else (n if n is not None else
                                                       (columnar[3] if self._col_data is not None else 0))

    @property
    def _col(self):
        if self._col_loader is not None:
            self._col_data, self._exact = self._col_loader()
            self._col_loader = None
        return self._col_data

    @property
    def exact(self):
        if self._col_loader is not None:
            self._col  # noqa: B018 -- loads the columns (and the exact accumulators)
        return self._exact or {}

    @property
    def gid_columns(self):
        """Per group-by column, the [n] table-global dictIds of the groups (zero-copy)."""
        return self._col[1]

    @property
    def gids(self):
        """[n, num_group_by] table-global dictIds of the groups."""
        cols = self._col[1]
        return np.stack(cols, axis=1) if cols and self._n else np.zeros((self._n, len(cols)), dtype=np.int32)

    @property
    def keys(self):
        if self._keys is None:
            dicts, cols = self._col[0], self._col[1]
            vals = [np.asarray(d)[c].tolist() if self._n else [] for d, c in zip(dicts, cols)]
            self._keys = list(zip(*vals)) if vals else [()] * self._n
        return self._keys

    @property
    def values(self):
        if self._values is None:
            cols = []
            for fn, v, e, c in self._col[2]:
                if v is None:
                    v = e.astype(np.float64)
                if fn == "AVG":
                    cols.append([AvgPair(x, y) for x, y in zip(v.tolist(), c.tolist())])
                elif fn == "COUNT":
                    cols.append((e if e is not None else v.astype(np.int64)).tolist())
                else:
                    cols.append(v.tolist())
            self._values = [list(r) for r in zip(*cols)] if cols else [[] for _ in range(self._n)]
        return self._values

    def as_dict(self):
        return {k: v for k, v in zip(self.keys, self.values)}

    def string_keys(self):
        """GroupKeyGenerator.StringGroupKey form: values joined by GroupKeyGenerator.DELIMITER ('\\0')."""
        return {"\0".join(_key_str(x) for x in k): v for k, v in zip(self.keys, self.values)}

    def __len__(self):
        return self._n

    # ---- after the combine (server_response.cpp)
    def trim_sql(self, query=None):
        """The server's SQL-mode combined table (GroupByOrderByCombineOperator + IndexedTable.finish): the top
        max(limit * 5, minServerGroupTrimSize) groups in ORDER BY order, `limit` groups without ORDER BY, every group
        when server trim is off (query.min_server_group_trim_size <= 0)."""
        query = query or self._query
        keep, spec = query.sql_trim_c()
        out = ctypes.c_void_p()
        L.check(self._table.lib.pgpu_result_trim_sql(self._holder.r, ctypes.byref(spec), ctypes.byref(out)))
        return _decode_result(self._table, query, _ResultHolder(self._table.lib, out))

    def trim_pql(self, limit, final=False):
        """AggregationGroupByTrimmingService: per aggregation the [(key tuple, value)] of its top groups (MIN
        ascending, the others descending; final=True: the broker's top `limit`, else the server trim)."""
        lib, na = self._table.lib, len(self._query.aggregations)
        counts = np.zeros(max(na, 1), dtype=np.int64)
        L.check(lib.pgpu_result_trim_pql(self._holder.r, limit, int(final), None, 0, L.ptr(counts, ctypes.c_int64)))
        cap = int(counts.max()) if na else 0
        rows = np.zeros(max(na * cap, 1), dtype=np.int64)
        L.check(lib.pgpu_result_trim_pql(self._holder.r, limit, int(final), L.ptr(rows, ctypes.c_int64), cap,
                                         L.ptr(counts, ctypes.c_int64)))
        keys, values = self.keys, self.values
        out = []
        for a in range(na):
            sel = rows[a * cap:a * cap + counts[a]]
            out.append([(keys[i], values[i][a]) for i in sel.tolist()])
        return out

    def datatable(self):
        """The server response bytes (DataTable V3, IntermediateResultsBlock.getResultDataTable) of these rows."""
        lib = self._table.lib
        n = ctypes.c_int64()
        L.check(lib.pgpu_result_datatable(self._holder.r, self._table.handle, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(max(n.value, 1))
        L.check(lib.pgpu_result_datatable(self._holder.r, self._table.handle, buf, n.value, ctypes.byref(n)))
        return buf.raw[:n.value]


def broker_reduce_sql(datatables, query):
    """GroupByDataTableReducer (SQL): merges the servers' DataTable V3 responses, ORDER BY, LIMIT, final results;
    returns the BrokerResponseNative as a dict (resultTable + statistics)."""
    import json
    lib = L.load()
    keep, spec = query.sql_trim_c()
    bufs = [ctypes.create_string_buffer(bytes(b), max(len(b), 1)) for b in datatables]
    ptrs = (ctypes.c_void_p * max(len(bufs), 1))(*[ctypes.cast(b, ctypes.c_void_p) for b in bufs])
    lens = np.array([len(b) for b in datatables] or [0], dtype=np.int64)
    n = ctypes.c_int64()
    L.check(lib.pgpu_broker_reduce_sql(ptrs, L.ptr(lens, ctypes.c_int64), len(bufs), ctypes.byref(spec), None, 0,
                                       ctypes.byref(n)))
    out = ctypes.create_string_buffer(n.value + 1)
    L.check(lib.pgpu_broker_reduce_sql(ptrs, L.ptr(lens, ctypes.c_int64), len(bufs), ctypes.byref(spec), out,
                                       n.value + 1, ctypes.byref(n)))
    return json.loads(out.value.decode("utf-8"))


def aggregation_defaults(aggregations):
    """Results of aggregation functions over no documents: their result holders' initial values
    (SumAggregationFunction.java:33 0.0, MinAggregationFunction.java:33 +inf, MaxAggregationFunction.java:33 -inf,
    CountAggregationFunction.java:38 0, AvgAggregationFunction: AvgPair(0.0, 0))."""
    out = []
    for fn, _ in aggregations:
        out.append({"COUNT": 0, "SUM": 0.0, "MIN": float("inf"), "MAX": float("-inf")}.get(fn, None)
                   if fn != "AVG" else AvgPair(0.0, 0))
    return out


class AggregationResult:
    """Aggregation-only result (AggregationOperator / AggregationOnlyCombineOperator): one value per function in
    query order, and ExecutionStatistics."""

    def __init__(self, values, stats):
        self.values = values
        self.stats = stats

    def __repr__(self):
        return "AggregationResult(%r, %r)" % (self.values, self.stats)


def _key_str(x):
    if isinstance(x, float):
        return repr(x)
    return str(x)


class GpuTable:
    def __init__(self, schema, device=0, config=None):
        """schema: list of (column name, type name 'INT'|'LONG'|'FLOAT'|'DOUBLE'|'STRING'); config: executor settings
        (pgpu_config field -> value, see set_config)."""
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
        self._snapshots = {}  # dictionary snapshot id -> values (results index the snapshot their plan saw)
        if config:
            self.set_config(**config)

    # ------------------------------------------------------------------ executor settings
    def config(self):
        """The table's pgpu_config as a dict (pgpu_table_get_config)."""
        c = L.ConfigC()
        L.check(self.lib.pgpu_table_get_config(self.handle, ctypes.byref(c)))
        return {f: getattr(c, f) for f in L.CONFIG_FIELDS}

    def set_config(self, **fields):
        """pgpu_table_set_config: the named fields changed, the others kept (plan_cache, partitioned_group_by,
        hash_partitions, hash_partition_bits, hash_partition_lds_kb, lds_table_kb, plan_chunk_segments, stream_chunks,
        compact_results, star_tree_workgroups, dense_selectivity, slot_weight_step -- include/pinotgpu.h).  Plans made afterwards use
        them (the compiled-plan cache is cleared)."""
        cur = self.config()
        bad = set(fields) - set(cur)
        if bad:
            raise ValueError("unknown config fields: %s" % sorted(bad))
        cur.update(fields)
        c = L.ConfigC(ctypes.sizeof(L.ConfigC), **cur)
        L.check(self.lib.pgpu_table_set_config(self.handle, ctypes.byref(c)))

    def reset_config(self):
        """The library's defaults (pgpu_config_default)."""
        c = L.ConfigC()
        L.check(self.lib.pgpu_config_default(ctypes.byref(c)))
        L.check(self.lib.pgpu_table_set_config(self.handle, ctypes.byref(c)))

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
        try:
            for name in self.names:
                inv = getattr(seg.columns[name], "inv_bytes", None)
                if inv is not None:
                    self.attach_inverted_index(h.value, name, inv)
                rng = getattr(seg.columns[name], "range_bytes", None)
                if rng is not None:
                    self.attach_range_index(h.value, name, rng)
        except Exception:
            self.lib.pgpu_unpin_segment(self.handle, h.value)  # no half-loaded segment stays pinned
            raise
        return h.value

    def attach_inverted_index(self, handle, column, inv_bytes):
        """Pins a column's bitmap inverted index (BitmapInvertedIndexReader bytes) for the pinned segment `handle`:
        EQ / NOT_EQ / IN / NOT_IN on it then run as BitmapBasedFilterOperator leaves."""
        buf = ctypes.create_string_buffer(bytes(inv_bytes), max(len(inv_bytes), 1))
        L.check(self.lib.pgpu_attach_inverted_index(self.handle, handle, self.names.index(column),
                                                    ctypes.cast(buf, ctypes.c_void_p), len(inv_bytes)))

    def attach_range_index(self, handle, column, range_bytes):
        """Pins a column's range index (RangeIndexReaderImpl / BitSlicedRangeIndexReader bytes) for the pinned segment
        `handle`: RANGE predicates on it then run as RangeIndexBasedFilterOperator leaves (b"" detaches it)."""
        buf = ctypes.create_string_buffer(bytes(range_bytes), max(len(range_bytes), 1))
        L.check(self.lib.pgpu_attach_range_index(self.handle, handle, self.names.index(column),
                                                 ctypes.cast(buf, ctypes.c_void_p), len(range_bytes)))

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

    def result_dictionary(self, r, key, column):
        """Values of the table-global dictionary snapshot that group-by key `key` of C result `r` indexes (cached
        by snapshot id: unchanged until a pin grows the column's dictionary)."""
        sid, n = ctypes.c_uint64(), ctypes.c_int64()
        L.check(self.lib.pgpu_result_key_dictionary(r, key, ctypes.byref(sid), ctypes.byref(n)))
        vals = self._snapshots.get(sid.value)
        if vals is not None:
            return vals
        n = n.value
        t = self.types[self.index[column]]
        if t in (L.INT, L.LONG):
            a = np.zeros(max(n, 1), dtype=np.int64)
            L.check(self.lib.pgpu_result_key_dictionary_i64(r, key, L.ptr(a, ctypes.c_int64)))
            vals = [int(x) for x in a[:n]]
        elif t in (L.FLOAT, L.DOUBLE):
            a = np.zeros(max(n, 1), dtype=np.float64)
            L.check(self.lib.pgpu_result_key_dictionary_f64(r, key, L.ptr(a, ctypes.c_double)))
            vals = [float(x) for x in a[:n]]
        else:
            off = np.zeros(n + 1, dtype=np.int64)
            L.check(self.lib.pgpu_result_key_dictionary_str(r, key, None, 0, L.ptr(off, ctypes.c_int64)))
            blob = np.zeros(max(int(off[-1]), 1), dtype=np.uint8)
            L.check(self.lib.pgpu_result_key_dictionary_str(r, key, L.ptr(blob, ctypes.c_uint8), len(blob),
                                                            L.ptr(off, ctypes.c_int64)))
            b = blob.tobytes()
            vals = [b[off[i]:off[i + 1]].decode("utf-8", errors="surrogateescape") for i in range(n)]
        if len(self._snapshots) > 64:
            self._snapshots.clear()
        self._snapshots[sid.value] = vals
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
    def execute_aggregation(self, handles, query, stream=None):
        """Aggregation-only query (no GROUP BY) over the segments: AggregationOperator per segment +
        AggregationOnlyCombineOperator (core/operator/query/AggregationOperator.java:58-95)."""
        assert not query.group_by, "execute_aggregation takes a query without GROUP BY"
        r = self.execute_groupby(handles, query, stream)
        vals = r.values[0] if len(r) else aggregation_defaults(query.aggregations)
        return AggregationResult(list(vals), r.stats)

    def plan(self, handles, query):
        return Plan(self, handles, query)

    def execute_groupby(self, handles, query, stream=None):
        with Plan(self, handles, query, execute=(stream, None)) as p:
            return p.finalize(stream)

    def plan_execute(self, handles, query, stream=None, d_table=None):
        """Plan + execute, streamed (pgpu_plan_create_execute): chunks of segments are launched while the rest
        is still being planned.  Returns the executed Plan (finalize it, or merge across GPUs first)."""
        return Plan(self, handles, query, execute=(stream, d_table))


class Plan:
    def __init__(self, table, handles, query, execute=None):
        """execute=(stream, d_table): create and execute in one streamed call (pgpu_plan_create_execute)."""
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
        if execute is None:
            L.check(self.lib.pgpu_plan_create(table.handle, L.ptr(hs, ctypes.c_int64), len(hs), ctypes.byref(q),
                                              ctypes.byref(h)))
        else:
            stream, d_table = execute
            L.check(self.lib.pgpu_plan_create_execute(table.handle, L.ptr(hs, ctypes.c_int64), len(hs),
                                                      ctypes.byref(q), ctypes.c_void_p(stream or 0),
                                                      ctypes.c_void_p(d_table or 0), ctypes.byref(h)))
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

    def cancel(self):
        """pgpu_plan_cancel: from any thread; a finalize waiting on this plan raises QueryCancelledError."""
        L.check(self.lib.pgpu_plan_cancel(self.handle))

    def leaf_kinds(self):
        """{kernel leaf kind: (segment, leaf) pairs} of the scanned segments (pgpu_plan_leaf_kinds), e.g. "bitdir"
        for inverted-index leaves read in place, "bitmap" for ones materialised per query."""
        out = np.zeros(len(L.LEAF_KIND_NAMES), dtype=np.int64)
        L.check(self.lib.pgpu_plan_leaf_kinds(self.handle, L.ptr(out, ctypes.c_int64)))
        return {n: int(v) for n, v in zip(L.LEAF_KIND_NAMES, out) if v}

    def group_path(self):
        """The group-by path of the plan's scan (pgpu_plan_group_path): "lds", "global", "hash", "partitioned" or
        "hash_partitioned"."""
        out = ctypes.c_int32(-1)
        L.check(self.lib.pgpu_plan_group_path(self.handle, ctypes.byref(out)))
        return L.GROUP_PATH_NAMES[out.value]

    def execute(self, stream=None, d_table=None):
        L.check(self.lib.pgpu_plan_execute(self.handle, ctypes.c_void_p(stream or 0), ctypes.c_void_p(d_table or 0)))

    def scanned_segments(self):
        """Per plan segment: True if scanned (its filter does not fold to always-false)."""
        out = np.zeros(max(self.num_segments, 1), dtype=np.uint8)
        L.check(self.lib.pgpu_plan_scanned_segments(self.handle, L.ptr(out, ctypes.c_uint8)))
        return out[:self.num_segments].astype(bool)

    def timing_us(self):
        """(execute, scan launches summed, number of scan launches, star-tree kernels) in microseconds; the query
        carried timing=True (PGPU_OPT_TIMING), else PinotGpuError."""
        out = (ctypes.c_double * 4)()
        L.check(self.lib.pgpu_plan_timing(self.handle, out))
        return out[0], out[1], out[2], out[3]

    def star_metric_bytes(self):
        """Bytes of the star-tree metric arrays the last execution read: 64-B sectors holding a matched document
        (-1: not read back for this plan's table size)."""
        fn = getattr(self.lib, "pgpu_plan_star_metric_bytes", None)  # (an older library of an A/B run: -1)
        if fn is None:
            return -1
        out = ctypes.c_int64(0)
        L.check(fn(self.handle, ctypes.byref(out)))
        return out.value

    def star_work(self):
        """(star-tree segments, their nodes, star-tree documents read) of the last finalized execution."""
        out = (ctypes.c_int64 * 3)()
        L.check(self.lib.pgpu_plan_star_work(self.handle, out))
        return out[0], out[1], out[2]

    def finalize(self, stream=None, d_table=None):
        """Waits for the execution, compacts the group table and returns the decoded result.  `finalize_us`
        holds (C ABI finalize incl. the wait for the kernels, decode into numpy) in microseconds."""
        r = ctypes.c_void_p()
        t0 = time.perf_counter()
        L.check(self.lib.pgpu_plan_finalize(self.handle, ctypes.c_void_p(stream or 0), ctypes.c_void_p(d_table or 0),
                                            ctypes.byref(r)))
        t1 = time.perf_counter()
        holder = _ResultHolder(self.lib, r)
        res = _decode_result(self.table, self.query, holder)
        self.finalize_us = ((t1 - t0) * 1e6, (time.perf_counter() - t1) * 1e6)
        return res

    def exchange_counts(self, stream, nparts):
        """Per-owner group counts of this executed hash-mode table (pgpu_plan_exchange_counts; waits for the plan)."""
        counts = np.zeros(nparts, dtype=np.int64)
        L.check(self.lib.pgpu_plan_exchange_counts(self.handle, ctypes.c_void_p(stream or 0), nparts,
                                                   L.ptr(counts, ctypes.c_int64)))
        return counts

    def exchange_export(self, stream, nparts, kinds, d_out, cap):
        """The table's records [key, slot words] grouped by owner rank into device memory d_out (cap records)."""
        k = np.ascontiguousarray(kinds, dtype=np.int32)
        L.check(self.lib.pgpu_plan_exchange_export(self.handle, ctypes.c_void_p(stream or 0), nparts,
                                                   L.ptr(k, ctypes.c_int32), ctypes.c_void_p(d_out or 0), cap))

    def exchange_merge(self, stream, kinds, d_records, n):
        """Replaces the table by the merge of n received records (device); finalize returns them."""
        k = np.ascontiguousarray(kinds, dtype=np.int32)
        L.check(self.lib.pgpu_plan_exchange_merge(self.handle, ctypes.c_void_p(stream or 0), L.ptr(k, ctypes.c_int32),
                                                  ctypes.c_void_p(d_records or 0), n))

    def finalize_range(self, stream, d_shard, key_begin, key_count):
        """Finalize of this rank's key-range shard of the merged dense table (combine.reduce_scatter_group_table):
        the groups with keys in [key_begin, key_begin + key_count)."""
        return _finalize_range(self, stream, d_shard, key_begin, key_count)


def _finalize_range(plan, stream, d_shard, key_begin, key_count):
    r = ctypes.c_void_p()
    t0 = time.perf_counter()
    L.check(plan.lib.pgpu_plan_finalize_range(plan.handle, ctypes.c_void_p(stream or 0), ctypes.c_void_p(d_shard),
                                              key_begin, key_count, ctypes.byref(r)))
    t1 = time.perf_counter()
    res = _decode_result(plan.table, plan.query, _ResultHolder(plan.lib, r))
    plan.finalize_us = ((t1 - t0) * 1e6, (time.perf_counter() - t1) * 1e6)
    return res


class _ResultHolder:
    """Owns a pgpu_result; numpy views of its pinned columns reference this object, so the C result lives until
    the last view is gone."""

    def __init__(self, lib, r):
        self.lib, self.r = lib, r

    def __del__(self):
        if self.r:
            self.lib.pgpu_result_destroy(self.r)
            self.r = None


class _View:
    def __init__(self, owner, addr, n, typestr):
        self.owner = owner
        self.__array_interface__ = {"shape": (n,), "typestr": typestr, "data": (addr, True), "version": 3}


def _view(holder, addr, n, dtype):
    if n == 0 or not addr:
        return np.zeros(0, dtype=dtype)
    return np.asarray(_View(holder, addr, n, np.dtype(dtype).str))


def _decode_result(table, query, holder):
    """Columnar result over zero-copy views of the C result (pgpu_result_*_view), built on first use: a result the
    C side holds in compact form (large dense tables) is only decoded when its rows are read."""
    lib, r = table.lib, holder.r
    n = ctypes.c_int64()
    L.check(lib.pgpu_result_num_groups(r, ctypes.byref(n)))
    n = n.value
    nk = len(query.group_by)

    def load():
        ptr = ctypes.c_void_p()
        cols = []
        for j in range(nk):
            L.check(lib.pgpu_result_group_ids_view(r, j, ctypes.byref(ptr)))
            cols.append(_view(holder, ptr.value, n, np.int32))
        dicts = [table.result_dictionary(r, j, c) for j, c in enumerate(query.group_by)]
        aggs = []
        exact = {}
        form = ctypes.c_int32()
        for a, (fn, _) in enumerate(query.aggregations):
            L.check(lib.pgpu_result_words_view(r, a, ctypes.byref(ptr), ctypes.byref(form)))
            e = v = c = None
            if form.value == 0:
                exact[a] = e = _view(holder, ptr.value, n, np.int64)
            elif form.value == 1:
                v = _view(holder, ptr.value, n, np.float64)
            else:
                v = np.empty(max(n, 1), dtype=np.float64)
                L.check(lib.pgpu_result_values(r, a, L.ptr(v, ctypes.c_double)))
                v = v[:n]
            if fn == "AVG":
                L.check(lib.pgpu_result_words_view(r, -1, ctypes.byref(ptr), ctypes.byref(form)))
                c = _view(holder, ptr.value, n, np.int64)
            aggs.append((fn, v, e, c))
        return (dicts, cols, aggs, n), exact

    st = np.zeros(6, dtype=np.int64)
    L.check(lib.pgpu_result_stats(r, L.ptr(st, ctypes.c_int64)))
    reached = ctypes.c_int32()
    L.check(lib.pgpu_result_groups_limit_reached(r, ctypes.byref(reached)))
    res = GroupByResult(stats=ExecutionStatistics(st), columnar=load, holder=holder, table=table, query=query, n=n)
    res.num_groups_limit_reached = bool(reached.value)
    return res
